// DART / GOSS / RF boosting variants.
// DART: reference src/boosting/dart.hpp:60-200 (drop in GetTrainingScore, normalize after
//   the new tree, xgboost_dart_mode, uniform vs weighted drop).
// GOSS: reference src/boosting/goss.hpp:78-170 (per-block top-k by |g*h|, the remaining
//   rows sampled with the sequential rest_need/rest_all probability, scaled by
//   (cnt-top_k)/other_k; no subsampling during the first 1/learning_rate iterations).
// RF: reference src/boosting/rf.hpp:33-200 (gradients computed once from the averaged
//   init score, shrinkage 1, running average of tree outputs).
// With a device learner the training score lives in HBM: every score mutation goes
// through TrainScore*(), and GOSS samples on the device too (DeviceSample from GBDT::Bagging,
// src/device/sample_kernels.hip: the same per-block generators as the host draw).
#include <algorithm>
#include <cmath>

#include "lgbm_amd/boosting.h"
#include "lgbm_amd/common.h"
#include "lgbm_amd/log.h"

namespace lgbm_amd {

// ------------------------------------------------------------------------ DART
void DART::Init(const Config* cfg, const Dataset* train_data, const ObjectiveFunction* objective,
                const std::vector<const Metric*>& training_metrics) {
  GBDT::Init(cfg, train_data, objective, training_metrics);
  random_for_drop_ = Random(config_->drop_seed);
  sum_weight_ = 0.0;
}

void DART::ResetConfig(const Config* cfg) {
  GBDT::ResetConfig(cfg);
  random_for_drop_ = Random(config_->drop_seed);
  sum_weight_ = 0.0;
}

bool DART::TrainOneIter(const score_t* g, const score_t* h) {
  is_update_score_cur_iter_ = false;
  if (GBDT::TrainOneIter(g, h)) return true;
  Normalize();
  if (!config_->uniform_drop) {
    tree_weight_.push_back(shrinkage_rate_);
    sum_weight_ += shrinkage_rate_;
  }
  return false;
}

void DART::PrepareScoreForGradients() {
  if (!is_update_score_cur_iter_) {
    DroppingTrees();
    is_update_score_cur_iter_ = true;
  }
}

const double* DART::GetTrainingScore(int64_t* out_len) {
  PrepareScoreForGradients();
  *out_len = static_cast<int64_t>(num_data_) * num_class_;
  return HostTrainScore();
}

bool DART::EvalAndCheckEarlyStopping() {
  OutputMetric(iter_);
  return false;
}

void DART::DroppingTrees() {
  drop_index_.clear();
  const bool skip = random_for_drop_.NextFloat() < config_->skip_drop;
  if (!skip) {
    double rate = config_->drop_rate;
    if (!config_->uniform_drop) {
      const double inv_avg = static_cast<double>(tree_weight_.size()) / sum_weight_;
      if (config_->max_drop > 0) rate = std::min(rate, config_->max_drop * inv_avg / sum_weight_);
      for (int i = 0; i < iter_; ++i) {
        if (random_for_drop_.NextFloat() < rate * tree_weight_[i] * inv_avg) {
          drop_index_.push_back(num_init_iteration_ + i);
          if (drop_index_.size() >= static_cast<size_t>(config_->max_drop)) break;
        }
      }
    } else {
      if (config_->max_drop > 0) rate = std::min(rate, config_->max_drop / static_cast<double>(iter_));
      for (int i = 0; i < iter_; ++i) {
        if (random_for_drop_.NextFloat() < rate) {
          drop_index_.push_back(num_init_iteration_ + i);
          if (drop_index_.size() >= static_cast<size_t>(config_->max_drop)) break;
        }
      }
    }
  }
  for (int i : drop_index_) {
    for (int k = 0; k < num_tree_per_iteration_; ++k) {
      Tree* t = models_[static_cast<size_t>(i) * num_tree_per_iteration_ + k].get();
      t->Shrinkage(-1.0);
      TrainScoreAddTree(t, k);
    }
  }
  const double lr = config_->learning_rate;
  const double nd = static_cast<double>(drop_index_.size());
  if (!config_->xgboost_dart_mode) {
    shrinkage_rate_ = lr / (1.0f + nd);
  } else {
    shrinkage_rate_ = drop_index_.empty() ? lr : lr / (lr + nd);
  }
}

void DART::Normalize() {
  const double k = static_cast<double>(drop_index_.size());
  const double lr = config_->learning_rate;
  for (int i : drop_index_) {
    for (int c = 0; c < num_tree_per_iteration_; ++c) {
      Tree* t = models_[static_cast<size_t>(i) * num_tree_per_iteration_ + c].get();
      // valid scores: the tree is currently at -w; scale to the normalized weight minus w
      t->Shrinkage(!config_->xgboost_dart_mode ? 1.0f / (k + 1.0f) : shrinkage_rate_);
      for (auto& su : valid_score_updater_) su->AddScore(t, c);
      // train scores: the dropped tree was removed entirely; add back the normalized tree
      t->Shrinkage(!config_->xgboost_dart_mode ? -k : -k / lr);
      TrainScoreAddTree(t, c);
    }
    if (!config_->uniform_drop) {
      const size_t j = static_cast<size_t>(i - num_init_iteration_);
      if (!config_->xgboost_dart_mode) {
        sum_weight_ -= tree_weight_[j] * (1.0f / (k + 1.0f));
        tree_weight_[j] *= (k / (k + 1.0f));
      } else {
        sum_weight_ -= tree_weight_[j] * (1.0f / (k + lr));
        tree_weight_[j] *= (k / (k + lr));
      }
    }
  }
}

// ------------------------------------------------------------------------ GOSS
void GOSS::Init(const Config* cfg, const Dataset* train_data, const ObjectiveFunction* objective,
                const std::vector<const Metric*>& training_metrics) {
  GBDT::Init(cfg, train_data, objective, training_metrics);
  ResetGoss();
  const size_t total = static_cast<size_t>(num_data_) * num_tree_per_iteration_;
  gradients_.resize(total, 0.0f);
  hessians_.resize(total, 0.0f);
}

void GOSS::ResetTrainingData(const Dataset* train_data, const ObjectiveFunction* objective,
                             const std::vector<const Metric*>& training_metrics) {
  GBDT::ResetTrainingData(train_data, objective, training_metrics);
  ResetGoss();
}

void GOSS::ResetConfig(const Config* cfg) {
  GBDT::ResetConfig(cfg);
  ResetGoss();
}

void GOSS::ResetGoss() {
  LGBM_CHECK_LE(config_->top_rate + config_->other_rate, 1.0f);
  LGBM_CHECK(config_->top_rate > 0.0f && config_->other_rate > 0.0f);
  if (config_->bagging_freq > 0 && config_->bagging_fraction != 1.0f) Log::Fatal("Cannot use bagging in GOSS");
  Log::Info("Using GOSS");
  balanced_bagging_ = false;
  bag_data_indices_.resize(num_data_);
  bagging_rands_.clear();
  for (data_size_t i = 0; i < (num_data_ + kBaggingRandBlock - 1) / kBaggingRandBlock; ++i) {
    bagging_rands_.emplace_back(config_->bagging_seed + i);
  }
  device_sampler_seed_ = config_->bagging_seed;
  device_sampler_reset_ = true;
  bag_data_cnt_ = num_data_;
}

bool GOSS::TrainOneIter(const score_t* g, const score_t* h) {
  if (g != nullptr) {
    LGBM_CHECK(h != nullptr);
    const size_t total = static_cast<size_t>(num_data_) * num_tree_per_iteration_;
    std::copy(g, g + total, gradients_.begin());
    std::copy(h, h + total, hessians_.begin());
    return GBDT::TrainOneIter(gradients_.data(), hessians_.data());
  }
  LGBM_CHECK(h == nullptr);
  return GBDT::TrainOneIter(nullptr, nullptr);
}

data_size_t GOSS::BaggingHelper(data_size_t start, data_size_t cnt, data_size_t* buffer) {
  if (cnt <= 0) return 0;
  const int K = num_tree_per_iteration_;
  auto row_weight = [&](data_size_t r) {
    score_t s = 0.0f;
    for (int k = 0; k < K; ++k) {
      const size_t idx = static_cast<size_t>(k) * num_data_ + r;
      s += std::fabs(gradients_[idx] * hessians_[idx]);
    }
    return s;
  };
  std::vector<score_t> tmp(cnt);
  for (data_size_t i = 0; i < cnt; ++i) tmp[i] = row_weight(start + i);
  data_size_t top_k = std::max<data_size_t>(1, static_cast<data_size_t>(cnt * config_->top_rate));
  const data_size_t other_k = static_cast<data_size_t>(cnt * config_->other_rate);
  // (top_k)-th largest value: the threshold of the "large gradient" set
  std::nth_element(tmp.begin(), tmp.begin() + (top_k - 1), tmp.end(), std::greater<score_t>());
  const score_t threshold = tmp[top_k - 1];
  const score_t multiply = static_cast<score_t>(cnt - top_k) / other_k;
  data_size_t left = 0, right = cnt, big = 0;
  for (data_size_t i = 0; i < cnt; ++i) {
    const data_size_t r = start + i;
    if (row_weight(r) >= threshold) {
      buffer[left++] = r;
      ++big;
    } else {
      const data_size_t sampled = left - big;
      const data_size_t rest_need = other_k - sampled;
      const data_size_t rest_all = (cnt - i) - (top_k - big);
      const double prob = rest_need / static_cast<double>(rest_all);
      if (bagging_rands_[r / kBaggingRandBlock].NextFloat() < prob) {
        buffer[left++] = r;
        for (int k = 0; k < K; ++k) {
          const size_t idx = static_cast<size_t>(k) * num_data_ + r;
          gradients_[idx] *= multiply;
          hessians_[idx] *= multiply;
        }
      } else {
        buffer[--right] = r;
      }
    }
  }
  return left;
}

void GOSS::Bagging(int iter) {
  bag_data_cnt_ = num_data_;
  if (iter < static_cast<int>(1.0f / config_->learning_rate)) return;
  const data_size_t dev_cnt = DeviceBagging(true);
  if (dev_cnt >= 0) {
    bag_data_cnt_ = dev_cnt;
    return;
  }
  const int64_t total = static_cast<int64_t>(num_data_) * num_tree_per_iteration_;
  if (device_learner_ != nullptr) device_learner_->DownloadGradients(gradients_.data(), hessians_.data(), total);
  bag_data_cnt_ = RunBagging([this](data_size_t s, data_size_t c, data_size_t* b) { return BaggingHelper(s, c, b); });
  if (device_learner_ != nullptr) device_learner_->UploadGradients(gradients_.data(), hessians_.data(), total);
  tree_learner_->SetBaggingData(nullptr, bag_data_indices_.data(), bag_data_cnt_);
}

// ------------------------------------------------------------------------ RF
void RF::Init(const Config* cfg, const Dataset* train_data, const ObjectiveFunction* objective,
              const std::vector<const Metric*>& training_metrics) {
  LGBM_CHECK(cfg->bagging_freq > 0 && cfg->bagging_fraction < 1.0f && cfg->bagging_fraction > 0.0f);
  LGBM_CHECK(cfg->feature_fraction <= 1.0f && cfg->feature_fraction > 0.0f);
  GBDT::Init(cfg, train_data, objective, training_metrics);
  if (num_init_iteration_ > 0) {
    for (int k = 0; k < num_tree_per_iteration_; ++k) MultiplyScore(k, 1.0f / num_init_iteration_);
  } else {
    LGBM_CHECK(train_data->metadata().init_score() == nullptr);
  }
  LGBM_CHECK_EQ(num_tree_per_iteration_, num_class_);
  shrinkage_rate_ = 1.0f;
  Boosting();
}

void RF::ResetConfig(const Config* cfg) {
  LGBM_CHECK(cfg->bagging_freq > 0 && cfg->bagging_fraction < 1.0f && cfg->bagging_fraction > 0.0f);
  LGBM_CHECK(cfg->feature_fraction <= 1.0f && cfg->feature_fraction > 0.0f);
  GBDT::ResetConfig(cfg);
  shrinkage_rate_ = 1.0f;
}

void RF::ResetTrainingData(const Dataset* train_data, const ObjectiveFunction* objective,
                           const std::vector<const Metric*>& training_metrics) {
  GBDT::ResetTrainingData(train_data, objective, training_metrics);
  if (iter_ + num_init_iteration_ > 0) {
    for (int k = 0; k < num_tree_per_iteration_; ++k) TrainScoreMultiply(1.0f / (iter_ + num_init_iteration_), k);
  }
  LGBM_CHECK_EQ(num_tree_per_iteration_, num_class_);
  Boosting();
}

void RF::Boosting() {
  if (objective_ == nullptr) {
    Log::Fatal("RF mode do not support custom objective function, please use built-in objectives.");
  }
  init_scores_.assign(num_tree_per_iteration_, 0.0);
  for (int k = 0; k < num_tree_per_iteration_; ++k) init_scores_[k] = BoostFromAverage(k, false);
  const size_t total = static_cast<size_t>(num_data_) * num_tree_per_iteration_;
  std::vector<double> tmp(total);
  for (int k = 0; k < num_tree_per_iteration_; ++k) {
    std::fill(tmp.begin() + static_cast<size_t>(k) * num_data_, tmp.begin() + static_cast<size_t>(k + 1) * num_data_,
              init_scores_[k]);
  }
  gradients_.resize(total);
  hessians_.resize(total);
  objective_->GetGradients(tmp.data(), gradients_.data(), hessians_.data());
  if (device_learner_ != nullptr) {
    device_learner_->UploadGradients(gradients_.data(), hessians_.data(), static_cast<int64_t>(total));
  }
}

bool RF::TrainOneIter(const score_t* g, const score_t* h) {
  LGBM_CHECK(g == nullptr && h == nullptr);
  Bagging(iter_);
  const score_t* grad = device_learner_ != nullptr ? device_learner_->device_gradients() : gradients_.data();
  const score_t* hess = device_learner_ != nullptr ? device_learner_->device_hessians() : hessians_.data();
  for (int k = 0; k < num_tree_per_iteration_; ++k) {
    const size_t off = static_cast<size_t>(k) * num_data_;
    std::unique_ptr<Tree> tree(new Tree(2, false));
    if (class_need_train_[k]) tree.reset(tree_learner_->Train(grad + off, hess + off));
    const double n_before = iter_ + num_init_iteration_;
    if (tree->num_leaves() > 1) {
      const double pred = init_scores_[k];
      auto residual = [pred](const label_t* label, int i) { return static_cast<double>(label[i]) - pred; };
      tree_learner_->RenewTreeOutput(tree.get(), objective_, residual, num_data_, bag_data_indices_.data(),
                                     bag_data_cnt_);
      if (std::fabs(init_scores_[k]) > kEpsilon) tree->AddBias(init_scores_[k]);
      MultiplyScore(k, n_before);
      UpdateScore(tree.get(), k);
      MultiplyScore(k, 1.0 / (n_before + 1));
    } else if (models_.size() < static_cast<size_t>(num_tree_per_iteration_)) {
      double output = 0.0;
      if (!class_need_train_[k]) output = objective_->BoostFromScore(k);
      tree->AsConstantTree(output);
      MultiplyScore(k, n_before);
      UpdateScore(tree.get(), k);
      MultiplyScore(k, 1.0 / (n_before + 1));
    }
    models_.push_back(std::move(tree));
  }
  ++iter_;
  return false;
}

void RF::RollbackOneIter() {
  if (iter_ <= 0) return;
  const int cur = iter_ + num_init_iteration_ - 1;
  for (int k = 0; k < num_tree_per_iteration_; ++k) {
    Tree* t = models_[static_cast<size_t>(cur) * num_tree_per_iteration_ + k].get();
    t->Shrinkage(-1.0);
    MultiplyScore(k, iter_ + num_init_iteration_);
    TrainScoreAddTree(t, k);
    for (auto& su : valid_score_updater_) su->AddScore(t, k);
    MultiplyScore(k, 1.0f / (iter_ + num_init_iteration_ - 1));
  }
  for (int k = 0; k < num_tree_per_iteration_; ++k) models_.pop_back();
  --iter_;
}

void RF::MultiplyScore(int k, double v) {
  TrainScoreMultiply(v, k);
  for (auto& su : valid_score_updater_) su->MultiplyScore(v, k);
}

void RF::AddValidDataset(const Dataset* valid, const std::vector<const Metric*>& metrics) {
  GBDT::AddValidDataset(valid, metrics);
  if (iter_ + num_init_iteration_ > 0) {
    for (int k = 0; k < num_tree_per_iteration_; ++k) {
      valid_score_updater_.back()->MultiplyScore(1.0f / (iter_ + num_init_iteration_), k);
    }
  }
}

}  // namespace lgbm_amd
