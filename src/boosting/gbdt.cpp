// GBDT training driver (reference src/boosting/gbdt.cpp:42-797).
#include <omp.h>

#include <chrono>
#include <cmath>
#include <cstdlib>
#include <fstream>
#include <sstream>

#include "lgbm_amd/boosting.h"
#include "lgbm_amd/common.h"
#include "lgbm_amd/log.h"
#include "lgbm_amd/network.h"
#include "lgbm_amd/tuning.h"

namespace lgbm_amd {

// ------------------------------------------------------------------ ScoreUpdater
ScoreUpdater::ScoreUpdater(const Dataset* data, int ntpi)
    : data_(data), num_data_(data->num_data()), num_tree_per_iteration_(ntpi) {
  score_.assign(static_cast<size_t>(num_data_) * ntpi, 0.0);
  const double* init = data->metadata().init_score();
  if (init != nullptr) {
    if (data->metadata().num_init_score() % num_data_ != 0 || data->metadata().num_init_score() / num_data_ != ntpi) {
      Log::Fatal("Number of class for initial score error");
    }
    has_init_score_ = true;
    std::copy(init, init + score_.size(), score_.begin());
  }
}

void ScoreUpdater::AttachDevice(DeviceTreeLearner* dl, int slot) {
  device_ = dl;
  device_slot_ = slot;
  host_stale_ = false;
}

void ScoreUpdater::SyncFromDevice() {
  if (device_ == nullptr || !host_stale_) return;
  device_->ValidScoreToHost(device_slot_, score_.data());
  host_stale_ = false;
}

void ScoreUpdater::AddScore(double v, int k) {
  if (device_ != nullptr) {
    device_->ValidAddConst(device_slot_, v, k);
    host_stale_ = true;
    return;
  }
  double* s = score_.data() + static_cast<size_t>(k) * num_data_;
#pragma omp parallel for schedule(static, 512) if (num_data_ >= 1024)
  for (data_size_t i = 0; i < num_data_; ++i) s[i] += v;
}

void ScoreUpdater::MultiplyScore(double v, int k) {
  if (device_ != nullptr) {
    device_->ValidMultiply(device_slot_, v, k);
    host_stale_ = true;
    return;
  }
  double* s = score_.data() + static_cast<size_t>(k) * num_data_;
#pragma omp parallel for schedule(static, 512) if (num_data_ >= 1024)
  for (data_size_t i = 0; i < num_data_; ++i) s[i] *= v;
}

void ScoreUpdater::AddScore(const Tree* tree, int k) {
  if (device_ != nullptr) {
    device_->ValidAddTree(device_slot_, tree, k);
    host_stale_ = true;
    return;
  }
  tree->AddPredictionToScore(data_, num_data_, score_.data() + static_cast<size_t>(k) * num_data_);
}

void ScoreUpdater::AddScore(const Tree* tree, const data_size_t* idx, data_size_t n, int k) {
  tree->AddPredictionToScore(data_, idx, n, score_.data() + static_cast<size_t>(k) * num_data_);
}

void ScoreUpdater::AddScore(const TreeLearner* learner, const Tree* tree, int k) {
  learner->AddPredictionToScore(tree, score_.data() + static_cast<size_t>(k) * num_data_);
}

// ------------------------------------------------------------------ GBDT
GBDT::GBDT() = default;
GBDT::~GBDT() = default;

GBDT* GBDT::CreateBoosting(const std::string& type, const char* model_filename) {
  GBDT* b = nullptr;
  if (model_filename == nullptr || model_filename[0] == '\0') {
    if (type == "gbdt") b = new GBDT();
    else if (type == "dart") b = new DART();
    else if (type == "goss") b = new GOSS();
    else if (type == "rf") b = new RF();
    else Log::Fatal("Unknown boosting type %s", type.c_str());
    return b;
  }
  std::ifstream f(model_filename, std::ios::binary);
  if (!f) Log::Fatal("Could not open %s", model_filename);
  std::string s((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  if (!common::StartsWith(s, "tree")) Log::Fatal("Unknown model format or submodel type in model file %s", model_filename);
  if (type == "dart") b = new DART();
  else if (type == "goss") b = new GOSS();
  else if (type == "rf") b = new RF();
  else b = new GBDT();
  b->LoadModelFromString(s.data(), s.size());
  return b;
}

void GBDT::Init(const Config* cfg, const Dataset* train_data, const ObjectiveFunction* objective,
                const std::vector<const Metric*>& training_metrics) {
  LGBM_CHECK(train_data != nullptr);
  train_data_ = train_data;
  if (!cfg->monotone_constraints.empty()) {
    LGBM_CHECK_EQ(static_cast<size_t>(train_data->num_total_features()), cfg->monotone_constraints.size());
  }
  if (!cfg->feature_contri.empty()) {
    LGBM_CHECK_EQ(static_cast<size_t>(train_data->num_total_features()), cfg->feature_contri.size());
  }
  iter_ = 0;
  num_iteration_for_pred_ = 0;
  max_feature_idx_ = 0;
  num_class_ = cfg->num_class;
  config_.reset(new Config(*cfg));
  early_stopping_round_ = config_->early_stopping_round;
  es_first_metric_only_ = config_->first_metric_only;
  shrinkage_rate_ = config_->learning_rate;
  forced_splits_text_.clear();
  if (!config_->forcedsplits_filename.empty()) {
    std::ifstream f(config_->forcedsplits_filename);
    std::stringstream ss;
    ss << f.rdbuf();
    forced_splits_text_ = ss.str();
  }
  objective_ = objective;
  num_tree_per_iteration_ = objective_ != nullptr ? objective_->NumModelPerIteration() : num_class_;
  is_constant_hessian_ = GetIsConstHessian(objective);
  tree_learner_.reset(TreeLearner::CreateTreeLearner(config_->tree_learner, config_->device_type, config_.get()));
  tree_learner_->Init(train_data_, is_constant_hessian_);
  tree_learner_->SetForcedSplit(forced_splits_text_);
  device_learner_ = dynamic_cast<DeviceTreeLearner*>(tree_learner_.get());
  training_metrics_ = training_metrics;
  train_score_updater_.reset(new ScoreUpdater(train_data_, num_tree_per_iteration_));
  host_score_fresh_ = true;
  num_data_ = train_data_->num_data();
  if (device_learner_ != nullptr) {
    device_learner_->InitScores(num_tree_per_iteration_, train_data_->metadata().init_score());
  } else if (objective_ != nullptr) {
    const size_t total = static_cast<size_t>(num_data_) * num_tree_per_iteration_;
    gradients_.resize(total);
    hessians_.resize(total);
  }
  max_feature_idx_ = train_data_->num_total_features() - 1;
  label_idx_ = train_data_->label_idx();
  feature_names_ = train_data_->feature_names();
  feature_infos_ = train_data_->feature_infos();
  monotone_constraints_ = config_->monotone_constraints;
  ResetBaggingConfig(config_.get(), true);
  class_need_train_.assign(num_tree_per_iteration_, true);
  if (objective_ != nullptr && objective_->SkipEmptyClass()) {
    LGBM_CHECK_EQ(num_tree_per_iteration_, num_class_);
    for (int k = 0; k < num_class_; ++k) class_need_train_[k] = objective_->ClassNeedTrain(k);
  }
}

void GBDT::AddValidDataset(const Dataset* valid, const std::vector<const Metric*>& metrics) {
  if (!train_data_->CheckAlign(*valid)) {
    Log::Fatal("Cannot add validation data, since it has different bin mappers with training data");
  }
  std::unique_ptr<ScoreUpdater> su(new ScoreUpdater(valid, num_tree_per_iteration_));
  for (int i = 0; i < iter_; ++i) {
    for (int k = 0; k < num_tree_per_iteration_; ++k) {
      su->AddScore(models_[(i + num_init_iteration_) * num_tree_per_iteration_ + k].get(), k);
    }
  }
  if (device_learner_ != nullptr) {
    // binned validation rows and their scores move to the device: one traversal kernel per
    // tree instead of a host pass (falls back to the host if the layouts differ)
    const int slot = device_learner_->AddValidData(valid, num_tree_per_iteration_, su->score());
    if (slot >= 0) su->AttachDevice(device_learner_, slot);
  }
  valid_score_updater_.push_back(std::move(su));
  valid_metrics_.emplace_back(metrics);
  if (early_stopping_round_ > 0) {
    auto n = metrics.size();
    best_iter_.emplace_back(n, 0);
    best_score_.emplace_back(n, kMinScore);
    best_msg_.emplace_back(n);
  }
}

void GBDT::ResetTrainingData(const Dataset* train_data, const ObjectiveFunction* objective,
                             const std::vector<const Metric*>& training_metrics) {
  if (train_data != train_data_ && !train_data_->CheckAlign(*train_data)) {
    Log::Fatal("Cannot reset training data, since new training data has different bin mappers");
  }
  objective_ = objective;
  if (objective_ != nullptr) LGBM_CHECK_EQ(num_tree_per_iteration_, objective_->NumModelPerIteration());
  is_constant_hessian_ = GetIsConstHessian(objective);
  training_metrics_ = training_metrics;
  if (train_data != train_data_) {
    train_data_ = train_data;
    train_score_updater_.reset(new ScoreUpdater(train_data_, num_tree_per_iteration_));
    for (int i = 0; i < iter_; ++i) {
      for (int k = 0; k < num_tree_per_iteration_; ++k) {
        train_score_updater_->AddScore(models_[(i + num_init_iteration_) * num_tree_per_iteration_ + k].get(), k);
      }
    }
    num_data_ = train_data_->num_data();
    if (objective_ != nullptr && device_learner_ == nullptr) {
      const size_t total = static_cast<size_t>(num_data_) * num_tree_per_iteration_;
      gradients_.resize(total);
      hessians_.resize(total);
    }
    max_feature_idx_ = train_data_->num_total_features() - 1;
    label_idx_ = train_data_->label_idx();
    feature_names_ = train_data_->feature_names();
    feature_infos_ = train_data_->feature_infos();
    tree_learner_->ResetTrainingData(train_data, is_constant_hessian_);
    if (device_learner_ != nullptr) {
      device_learner_->InitScores(num_tree_per_iteration_, nullptr);
      for (int k = 0; k < num_tree_per_iteration_; ++k) {
        device_learner_->SyncScoreFromHost(train_score_updater_->score() + static_cast<size_t>(k) * num_data_, k);
      }
    }
    host_score_fresh_ = true;
    ResetBaggingConfig(config_.get(), true);
  }
}

void GBDT::ResetConfig(const Config* cfg) {
  std::unique_ptr<Config> nc(new Config(*cfg));
  if (!cfg->monotone_constraints.empty()) {
    LGBM_CHECK_EQ(static_cast<size_t>(train_data_->num_total_features()), cfg->monotone_constraints.size());
  }
  if (!cfg->feature_contri.empty()) {
    LGBM_CHECK_EQ(static_cast<size_t>(train_data_->num_total_features()), cfg->feature_contri.size());
  }
  early_stopping_round_ = nc->early_stopping_round;
  shrinkage_rate_ = nc->learning_rate;
  if (tree_learner_ != nullptr) tree_learner_->ResetConfig(nc.get());
  if (train_data_ != nullptr) ResetBaggingConfig(nc.get(), false);
  if (config_->forcedsplits_filename != nc->forcedsplits_filename) {
    forced_splits_text_.clear();
    if (!nc->forcedsplits_filename.empty()) {
      std::ifstream f(nc->forcedsplits_filename);
      std::stringstream ss;
      ss << f.rdbuf();
      forced_splits_text_ = ss.str();
    }
    if (tree_learner_ != nullptr) tree_learner_->SetForcedSplit(forced_splits_text_);
  }
  config_ = std::move(nc);  // the learner already holds this object's address
}

void GBDT::ResetBaggingConfig(const Config* cfg, bool is_change_dataset) {
  data_size_t num_pos = objective_ != nullptr ? objective_->NumPositiveData() : 0;
  const bool balance = (cfg->pos_bagging_fraction < 1.0 || cfg->neg_bagging_fraction < 1.0) && num_pos > 0;
  if ((cfg->bagging_fraction < 1.0 || balance) && cfg->bagging_freq > 0) {
    need_re_bagging_ = false;
    if (!is_change_dataset && config_ != nullptr && config_.get() != cfg &&
        config_->bagging_fraction == cfg->bagging_fraction && config_->bagging_freq == cfg->bagging_freq &&
        config_->pos_bagging_fraction == cfg->pos_bagging_fraction &&
        config_->neg_bagging_fraction == cfg->neg_bagging_fraction) {
      return;
    }
    if (balance) {
      balanced_bagging_ = true;
      bag_data_cnt_ = static_cast<data_size_t>(num_pos * cfg->pos_bagging_fraction) +
                      static_cast<data_size_t>((num_data_ - num_pos) * cfg->neg_bagging_fraction);
    } else {
      bag_data_cnt_ = static_cast<data_size_t>(cfg->bagging_fraction * num_data_);
    }
    bag_data_indices_.resize(num_data_);
    bagging_rands_.clear();
    for (data_size_t i = 0; i < (num_data_ + kBaggingRandBlock - 1) / kBaggingRandBlock; ++i) {
      bagging_rands_.emplace_back(config_->bagging_seed + i);
    }
    device_sampler_seed_ = config_->bagging_seed;
    device_sampler_reset_ = true;
    need_re_bagging_ = true;
  } else {
    bag_data_cnt_ = num_data_;
    bag_data_indices_.clear();
    tree_learner_->SetBaggingData(nullptr, nullptr, num_data_);
  }
}

data_size_t GBDT::RunBagging(const std::function<data_size_t(data_size_t, data_size_t, data_size_t*)>& helper) {
  // block layout of the reference's ParallelPartitionRunner<..., FORCE_SIZE> (threading.h:100-176):
  // nblock = min(threads, ceil(n/1024)), block size rounded up to a multiple of 1024
  const data_size_t n = num_data_;
  int nthreads = config_->num_threads > 0 ? config_->num_threads : omp_get_max_threads();
  int nblock = std::min<int>(nthreads, static_cast<int>((n + kBaggingRandBlock - 1) / kBaggingRandBlock));
  data_size_t bs = n;
  if (nblock > 1) {
    bs = (n + nblock - 1) / nblock;
    bs = (bs + kBaggingRandBlock - 1) / kBaggingRandBlock * kBaggingRandBlock;
  } else {
    nblock = 1;
  }
  std::vector<data_size_t> buf(n);
  std::vector<data_size_t> lc(nblock, 0), rc(nblock, 0), off(nblock, 0);
#pragma omp parallel for schedule(static, 1)
  for (int b = 0; b < nblock; ++b) {
    const data_size_t s = b * bs;
    const data_size_t c = std::min(bs, n - s);
    off[b] = s;
    if (c <= 0) continue;
    data_size_t l = helper(s, c, buf.data() + s);
    std::reverse(buf.begin() + s + l, buf.begin() + s + c);
    lc[b] = l;
    rc[b] = c - l;
  }
  std::vector<data_size_t> lw(nblock, 0), rw(nblock, 0);
  for (int b = 1; b < nblock; ++b) {
    lw[b] = lw[b - 1] + lc[b - 1];
    rw[b] = rw[b - 1] + rc[b - 1];
  }
  const data_size_t left = lw[nblock - 1] + lc[nblock - 1];
  for (int b = 0; b < nblock; ++b) {
    std::copy_n(buf.begin() + off[b], lc[b], bag_data_indices_.begin() + lw[b]);
    std::copy_n(buf.begin() + off[b] + lc[b], rc[b], bag_data_indices_.begin() + left + rw[b]);
  }
  return left;
}

data_size_t GBDT::BaggingHelper(data_size_t start, data_size_t cnt, data_size_t* buffer) {
  if (cnt <= 0) return 0;
  data_size_t left = 0, right = cnt;
  const label_t* label = train_data_->metadata().label();
  for (data_size_t i = 0; i < cnt; ++i) {
    const data_size_t idx = start + i;
    bool in_bag;
    if (balanced_bagging_) {
      const bool pos = label[idx] > 0;
      in_bag = bagging_rands_[idx / kBaggingRandBlock].NextFloat() <
               (pos ? config_->pos_bagging_fraction : config_->neg_bagging_fraction);
    } else {
      in_bag = bagging_rands_[idx / kBaggingRandBlock].NextFloat() < config_->bagging_fraction;
    }
    if (in_bag) buffer[left++] = idx;
    else buffer[--right] = idx;
  }
  return left;
}

void GBDT::Bagging(int iter) {
  common::ScopedTimer timer("GBDT::Bagging");
  if ((bag_data_cnt_ < num_data_ && config_->bagging_freq > 0 && iter % config_->bagging_freq == 0) ||
      need_re_bagging_) {
    need_re_bagging_ = false;
    const data_size_t dev_cnt = DeviceBagging(false);
    if (dev_cnt >= 0) {
      bag_data_cnt_ = dev_cnt;
      Log::Debug("Re-bagging on the device, using %d data to train", bag_data_cnt_);
      return;
    }
    bag_data_cnt_ = RunBagging([this](data_size_t s, data_size_t c, data_size_t* b) { return BaggingHelper(s, c, b); });
    Log::Debug("Re-bagging, using %d data to train", bag_data_cnt_);
    tree_learner_->SetBaggingData(nullptr, bag_data_indices_.data(), bag_data_cnt_);
  }
}

// the MI355X learner draws the bag itself: same generators (Random(bagging_seed + block)
// per 1024 rows), so bagging is bit-identical to the host draw; GOSS equals the
// reference's draw with one sampling block per 1024 rows (see src/device/sample_kernels.hip)
data_size_t GBDT::DeviceBagging(bool goss) {
  if (device_learner_ == nullptr) return -1;
  const char* e = tuning::Get(tuning::Knob::HostBagging);
  if (e != nullptr && e[0] == '1') return -1;
  DeviceSampleSpec sp;
  sp.goss = goss;
  sp.balanced = balanced_bagging_;
  sp.reset = device_sampler_reset_;
  sp.seed = device_sampler_seed_;
  sp.fraction = config_->bagging_fraction;
  sp.pos_fraction = config_->pos_bagging_fraction;
  sp.neg_fraction = config_->neg_bagging_fraction;
  sp.top_rate = config_->top_rate;
  sp.other_rate = config_->other_rate;
  sp.num_tree_per_iteration = num_tree_per_iteration_;
  sp.label = train_data_->metadata().label();
  // leaf-output renewal (L1 / quantile / MAPE) reads the bag on the host
  DeviceRenewSpec renew;
  const bool need_host = objective_ != nullptr && objective_->IsRenewTreeOutput() && !objective_->DeviceRenew(&renew);
  sp.host_indices = need_host ? &bag_data_indices_ : nullptr;
  device_sampler_reset_ = false;
  return device_learner_->DeviceSample(sp);
}

std::vector<double> GBDT::EvalValid(int i, int j) const {
  const Metric* m = valid_metrics_[i][j];
  const int slot = valid_score_updater_[i]->device_slot();
  const char* hm = tuning::Get(tuning::Knob::HostMetrics);  // =1: every metric on the host (A/B)
  const bool host_metrics = hm != nullptr && hm[0] == '1';
  if (slot >= 0 && device_learner_ != nullptr && !host_metrics) {
    const DeviceMetricSpec spec = m->DeviceSpec(objective_);
    std::vector<double> sums;
    if (spec.kind != 0 && device_learner_->ValidEval(slot, spec, &sums)) return m->FinishDevice(sums);
  }
  return m->Eval(valid_score_updater_[i]->score(), objective_);
}

std::vector<double> GBDT::EvalTrain(const Metric* m) {
  const char* hm = tuning::Get(tuning::Knob::HostMetrics);
  if (device_learner_ != nullptr && !(hm != nullptr && hm[0] == '1')) {
    const DeviceMetricSpec spec = m->DeviceSpec(objective_);
    std::vector<double> sums;
    if (spec.kind != 0 && device_learner_->TrainEval(spec, &sums)) return m->FinishDevice(sums);
  }
  return m->Eval(HostTrainScore(), objective_);
}

double* GBDT::HostTrainScore() {
  if (device_learner_ != nullptr && !host_score_fresh_) {
    for (int k = 0; k < num_tree_per_iteration_; ++k) {
      device_learner_->SyncScoreToHost(train_score_updater_->score() + static_cast<size_t>(k) * num_data_, k);
    }
    host_score_fresh_ = true;
  }
  return train_score_updater_->score();
}

void GBDT::TrainScoreAdd(double v, int k) {
  if (device_learner_ != nullptr) {
    device_learner_->AddConstToScore(v, k);
    host_score_fresh_ = false;
  } else {
    train_score_updater_->AddScore(v, k);
  }
}

void GBDT::TrainScoreMultiply(double v, int k) {
  if (device_learner_ != nullptr) {
    device_learner_->MultiplyScore(v, k);
    host_score_fresh_ = false;
  } else {
    train_score_updater_->MultiplyScore(v, k);
  }
}

void GBDT::TrainScoreAddTree(const Tree* tree, int k) {
  if (device_learner_ != nullptr) {
    device_learner_->AddTreeToScore(tree, k);
    host_score_fresh_ = false;
  } else {
    train_score_updater_->AddScore(tree, k);
  }
}

const double* GBDT::GetTrainingScore(int64_t* out_len) {
  *out_len = static_cast<int64_t>(num_data_) * num_class_;
  return HostTrainScore();
}

void GBDT::Boosting() {
  common::ScopedTimer timer("GBDT::Boosting");
  if (objective_ == nullptr) Log::Fatal("No object function provided");
  PrepareScoreForGradients();
  if (device_learner_ != nullptr) {
    DeviceGradSpec spec = objective_->DeviceSpec();
    if (spec.kind != DeviceGradKind::None && device_learner_->ComputeGradients(spec, num_tree_per_iteration_)) return;
    // objectives without a device kernel: host gradients from a host score mirror
    const size_t total = static_cast<size_t>(num_data_) * num_tree_per_iteration_;
    gradients_.resize(total);
    hessians_.resize(total);
    objective_->GetGradients(HostTrainScore(), gradients_.data(), hessians_.data());
    device_learner_->UploadGradients(gradients_.data(), hessians_.data(), static_cast<int64_t>(total));
    return;
  }
  objective_->GetGradients(HostTrainScore(), gradients_.data(), hessians_.data());
}

double GBDT::BoostFromAverage(int class_id, bool update_scorer) {
  if (models_.empty() && !train_score_updater_->has_init_score() && objective_ != nullptr) {
    if (config_->boost_from_average || (train_data_ != nullptr && train_data_->num_features() == 0)) {
      double init = objective_->BoostFromScore(class_id);
      if (Network::num_machines() > 1) init = Network::GlobalSyncUpByMean(init);
      if (std::fabs(init) > kEpsilon) {
        if (update_scorer) {
          TrainScoreAdd(init, class_id);
          for (auto& su : valid_score_updater_) su->AddScore(init, class_id);
        }
        Log::Info("Start training from score %lf", init);
        return init;
      }
    } else {
      const std::string n = objective_->GetName();
      if (n == "regression_l1" || n == "quantile" || n == "mape") {
        Log::Warning("Disabling boost_from_average in %s may cause the slow convergence", n.c_str());
      }
    }
  }
  return 0.0;
}

void GBDT::LogIteration(double grad_ms, double bag_ms, const std::vector<double>& tree_ms, double renew_ms,
                        double score_ms, double total_ms, const std::vector<int>& leaves,
                        const std::vector<int>& device, const std::vector<int>& rounds,
                        const std::vector<int>& expansions, const std::vector<int>& graphs, double coll_bytes) {
  std::ostringstream o;
  o.precision(6);
  o << "{\"iter\": " << iter_ << ", \"rank\": " << Network::rank() << ", \"ms\": " << total_ms
    << ", \"gradients_ms\": " << grad_ms << ", \"bagging_ms\": " << bag_ms << ", \"tree_ms\": [";
  for (size_t i = 0; i < tree_ms.size(); ++i) o << (i ? ", " : "") << tree_ms[i];
  o << "], \"renew_ms\": " << renew_ms << ", \"score_update_ms\": " << score_ms << ", \"leaves\": [";
  for (size_t i = 0; i < leaves.size(); ++i) o << (i ? ", " : "") << leaves[i];
  o << "], \"device_resident\": [";
  for (size_t i = 0; i < device.size(); ++i) o << (i ? ", " : "") << (device[i] ? "true" : "false");
  o << "], \"rounds\": [";
  for (size_t i = 0; i < rounds.size(); ++i) o << (i ? ", " : "") << rounds[i];
  o << "], \"expansions\": [";
  for (size_t i = 0; i < expansions.size(); ++i) o << (i ? ", " : "") << expansions[i];
  o << "], \"graph\": [";
  for (size_t i = 0; i < graphs.size(); ++i) o << (i ? ", " : "") << (graphs[i] ? "true" : "false");
  o << "], \"collective_bytes\": " << coll_bytes << "}\n";
  *iter_log_ << o.str();
  iter_log_->flush();
}

bool GBDT::SpeculationSafe(bool own_gradients) const {
  const Config& c = *config_;
  const bool bagging = c.bagging_freq > 0 && (c.bagging_fraction < 1.0 || c.pos_bagging_fraction < 1.0 ||
                                              c.neg_bagging_fraction < 1.0);
  return own_gradients && num_tree_per_iteration_ == 1 && !bagging && !need_re_bagging_ && bag_data_cnt_ == num_data_ &&
         !(objective_ != nullptr && objective_->IsRenewTreeOutput());
}

bool GBDT::TrainOneIter(const score_t* gradients, const score_t* hessians) {
  common::ScopedTimer timer("GBDT::TrainOneIter");
  if (!iter_log_checked_) {
    iter_log_checked_ = true;
    if (const char* path = tuning::Get(tuning::Knob::IterLog)) {
      std::string p(path);
      if (Network::num_machines() > 1) p += ".rank" + std::to_string(Network::rank());
      iter_log_.reset(new std::ofstream(p, std::ios::app));
      if (!*iter_log_) iter_log_.reset();
    }
  }
  using Clock = std::chrono::steady_clock;
  auto ms_since = [](Clock::time_point t) { return std::chrono::duration<double, std::milli>(Clock::now() - t).count(); };
  const auto t_iter = Clock::now();
  double grad_ms = 0, bag_ms = 0, renew_ms = 0, score_ms = 0, coll_bytes = 0;
  std::vector<double> tree_ms;
  std::vector<int> leaves, device, rounds, expansions, graphs;
  std::vector<double> init_scores(num_tree_per_iteration_, 0.0);
  const score_t* grad = gradients;
  const score_t* hess = hessians;
  if (gradients == nullptr || hessians == nullptr) {
    for (int k = 0; k < num_tree_per_iteration_; ++k) init_scores[k] = BoostFromAverage(k, true);
    Boosting();
    if (device_learner_ != nullptr) {
      grad = device_learner_->device_gradients();
      hess = device_learner_->device_hessians();
    } else {
      grad = gradients_.data();
      hess = hessians_.data();
    }
  } else if (device_learner_ != nullptr) {
    const int64_t total = static_cast<int64_t>(num_data_) * num_tree_per_iteration_;
    device_learner_->UploadGradients(gradients, hessians, total);
    grad = device_learner_->device_gradients();
    hess = device_learner_->device_hessians();
  }
  if (iter_log_) {
    if (device_learner_ != nullptr) device_learner_->Synchronize();
    grad_ms = ms_since(t_iter);
  }
  auto t_phase = Clock::now();
  Bagging(iter_);
  if (iter_log_) bag_ms = ms_since(t_phase);
  bool should_continue = false;
  for (int k = 0; k < num_tree_per_iteration_; ++k) {
    const size_t off = static_cast<size_t>(k) * num_data_;
    std::unique_ptr<Tree> tree(new Tree(2, false));
    t_phase = Clock::now();
    if (class_need_train_[k] && train_data_->num_features() > 0) {
      // the tree goes into the training scores right after its shrinkage unless its leaves
      // are renewed first: the device learner may add it while the host builds the Tree
      if (device_learner_ != nullptr && num_tree_per_iteration_ == 1 &&
          !(objective_ != nullptr && objective_->IsRenewTreeOutput())) {
        device_learner_->ExpectTrainingScoreUpdate(shrinkage_rate_);
      }
      if (device_learner_ != nullptr) device_learner_->AllowSpeculation(SpeculationSafe(gradients == nullptr));
      tree.reset(tree_learner_->Train(grad + off, hess + off));
      if (device_learner_ != nullptr) {
        const auto st = device_learner_->LastTreeStats();
        growth_stats_[0] += 1;
        growth_stats_[1] += st.device_mode ? 1 : 0;
        growth_stats_[2] += st.rounds;
        growth_stats_[3] += st.expansions;
        growth_stats_[4] += st.splits;
        growth_stats_[5] += st.collective_bytes;
        growth_stats_[6] += st.speculated ? 1 : 0;
      }
    }
    if (iter_log_) {
      tree_ms.push_back(ms_since(t_phase));
      leaves.push_back(tree->num_leaves());
      const auto st = device_learner_ != nullptr ? device_learner_->LastTreeStats() : DeviceTreeLearner::TreeStats();
      device.push_back(st.device_mode ? 1 : 0);
      rounds.push_back(st.rounds);
      expansions.push_back(st.expansions);
      graphs.push_back(st.graph ? 1 : 0);
      coll_bytes += st.collective_bytes;
    }
    if (tree->num_leaves() > 1) {
      should_continue = true;
      t_phase = Clock::now();
      if (objective_ != nullptr && objective_->IsRenewTreeOutput() &&
          !(device_learner_ != nullptr && device_learner_->RenewTreeOutputOnDevice(tree.get(), objective_, k))) {
        const double* sp = HostTrainScore() + off;
        auto residual = [sp](const label_t* label, int i) { return static_cast<double>(label[i]) - sp[i]; };
        tree_learner_->RenewTreeOutput(tree.get(), objective_, residual, num_data_, bag_data_indices_.data(),
                                       bag_data_cnt_);
      }
      if (iter_log_) renew_ms += ms_since(t_phase);
      tree->Shrinkage(shrinkage_rate_);
      t_phase = Clock::now();
      UpdateScore(tree.get(), k);
      if (iter_log_) {
        if (device_learner_ != nullptr) device_learner_->Synchronize();
        score_ms += ms_since(t_phase);
      }
      if (std::fabs(init_scores[k]) > kEpsilon) tree->AddBias(init_scores[k]);
    } else if (models_.size() < static_cast<size_t>(num_tree_per_iteration_)) {
      double output = 0.0;
      if (!class_need_train_[k]) {
        if (objective_ != nullptr) output = objective_->BoostFromScore(k);
      } else {
        output = init_scores[k];
      }
      tree->AsConstantTree(output);
      TrainScoreAdd(output, k);
      for (auto& su : valid_score_updater_) su->AddScore(output, k);
    }
    models_.push_back(std::move(tree));
  }
  if (!should_continue) {
    Log::Warning("Stopped training because there are no more leaves that meet the split requirements");
    if (models_.size() > static_cast<size_t>(num_tree_per_iteration_)) {
      for (int k = 0; k < num_tree_per_iteration_; ++k) models_.pop_back();
    }
    return true;
  }
  if (iter_log_) {
    if (device_learner_ != nullptr) device_learner_->Synchronize();
    LogIteration(grad_ms, bag_ms, tree_ms, renew_ms, score_ms, ms_since(t_iter), leaves, device, rounds, expansions, graphs, coll_bytes);
  }
  ++iter_;
  return false;
}

void GBDT::UpdateScore(const Tree* tree, int k) {
  common::ScopedTimer timer("GBDT::UpdateScore");
  if (device_learner_ != nullptr) {
    device_learner_->AddTrainedTreeToScore(tree, k);
    host_score_fresh_ = false;
  } else {
    train_score_updater_->AddScore(tree_learner_.get(), tree, k);
    if (num_data_ - bag_data_cnt_ > 0) {
      train_score_updater_->AddScore(tree, bag_data_indices_.data() + bag_data_cnt_, num_data_ - bag_data_cnt_, k);
    }
  }
  for (auto& su : valid_score_updater_) su->AddScore(tree, k);
}

void GBDT::RollbackOneIter() {
  if (iter_ <= 0) return;
  for (int k = 0; k < num_tree_per_iteration_; ++k) {
    auto& t = models_[models_.size() - num_tree_per_iteration_ + k];
    t->Shrinkage(-1.0);
    TrainScoreAddTree(t.get(), k);
    for (auto& su : valid_score_updater_) su->AddScore(t.get(), k);
  }
  for (int k = 0; k < num_tree_per_iteration_; ++k) models_.pop_back();
  --iter_;
}

void GBDT::Train(int snapshot_freq, const std::string& model_output_path) {
  common::ScopedTimer timer("GBDT::Train");
  bool finished = false;
  auto start = std::chrono::steady_clock::now();
  for (int it = 0; it < config_->num_iterations && !finished; ++it) {
    finished = TrainOneIter(nullptr, nullptr);
    if (!finished) finished = EvalAndCheckEarlyStopping();
    auto now = std::chrono::steady_clock::now();
    Log::Info("%f seconds elapsed, finished iteration %d",
              std::chrono::duration<double, std::milli>(now - start).count() * 1e-3, it + 1);
    if (snapshot_freq > 0 && (it + 1) % snapshot_freq == 0) {
      std::string out = model_output_path + ".snapshot_iter_" + std::to_string(it + 1);
      SaveModelToFile(0, -1, config_->saved_feature_importance_type, out.c_str());
    }
  }
}

void GBDT::RefitTree(const std::vector<std::vector<int>>& leaf_pred) {
  LGBM_CHECK_GT(leaf_pred.size(), 0u);
  LGBM_CHECK_EQ(static_cast<size_t>(num_data_), leaf_pred.size());
  LGBM_CHECK_EQ(models_.size(), leaf_pred[0].size());
  const int num_iter = static_cast<int>(models_.size()) / num_tree_per_iteration_;
  std::vector<int> lp(num_data_);
  for (int it = 0; it < num_iter; ++it) {
    Boosting();
    if (device_learner_ != nullptr) {
      const size_t total = static_cast<size_t>(num_data_) * num_tree_per_iteration_;
      gradients_.resize(total);
      hessians_.resize(total);
      device_learner_->DownloadGradients(gradients_.data(), hessians_.data(), static_cast<int64_t>(total));
    }
    for (int k = 0; k < num_tree_per_iteration_; ++k) {
      const int mi = it * num_tree_per_iteration_ + k;
      for (data_size_t i = 0; i < num_data_; ++i) {
        lp[i] = leaf_pred[i][mi];
        LGBM_CHECK_LT(lp[i], models_[mi]->num_leaves());
      }
      const size_t off = static_cast<size_t>(k) * num_data_;
      Tree* nt;
      if (device_learner_ != nullptr) {
        // refit is a host operation: use a CPU learner over the same data
        std::unique_ptr<TreeLearner> cpu(TreeLearner::CreateTreeLearner("serial", "cpu", config_.get()));
        cpu->Init(train_data_, is_constant_hessian_);
        nt = cpu->FitByExistingTree(models_[mi].get(), lp, gradients_.data() + off, hessians_.data() + off);
        device_learner_->AddTreeToScore(nt, k);
        host_score_fresh_ = false;
      } else {
        nt = tree_learner_->FitByExistingTree(models_[mi].get(), lp, gradients_.data() + off, hessians_.data() + off);
        train_score_updater_->AddScore(tree_learner_.get(), nt, k);
      }
      models_[mi].reset(nt);
    }
  }
}

bool GBDT::EvalAndCheckEarlyStopping() {
  std::string best_msg = OutputMetric(iter_);
  const bool met = !best_msg.empty();
  if (met) {
    Log::Info("Early stopping at iteration %d, the best iteration round is %d", iter_, iter_ - early_stopping_round_);
    Log::Info("Output of best iteration round:\n%s", best_msg.c_str());
    for (int i = 0; i < early_stopping_round_ * num_tree_per_iteration_; ++i) models_.pop_back();
  }
  return met;
}

std::string GBDT::OutputMetric(int iter) {
  const bool need_output = (iter % config_->metric_freq) == 0;
  std::string ret;
  std::stringstream msg;
  std::vector<std::pair<size_t, size_t>> met_pairs;
  if (need_output) {
    for (auto* m : training_metrics_) {
      auto names = m->GetName();
      auto scores = EvalTrain(m);
      for (size_t k = 0; k < names.size(); ++k) {
        std::stringstream t;
        t << "Iteration:" << iter << ", training " << names[k] << " : " << scores[k];
        Log::Info(t.str().c_str());
        if (early_stopping_round_ > 0) msg << t.str() << '\n';
      }
    }
  }
  if (need_output || early_stopping_round_ > 0) {
    for (size_t i = 0; i < valid_metrics_.size(); ++i) {
      for (size_t j = 0; j < valid_metrics_[i].size(); ++j) {
        auto scores = EvalValid(i, j);
        auto names = valid_metrics_[i][j]->GetName();
        for (size_t k = 0; k < names.size(); ++k) {
          std::stringstream t;
          t << "Iteration:" << iter << ", valid_" << i + 1 << " " << names[k] << " : " << scores[k];
          if (need_output) Log::Info(t.str().c_str());
          if (early_stopping_round_ > 0) msg << t.str() << '\n';
        }
        if (es_first_metric_only_ && j > 0) continue;
        if (ret.empty() && early_stopping_round_ > 0) {
          const double cur = valid_metrics_[i][j]->factor_to_bigger_better() * scores.back();
          if (cur > best_score_[i][j]) {
            best_score_[i][j] = cur;
            best_iter_[i][j] = iter;
            met_pairs.emplace_back(i, j);
          } else if (iter - best_iter_[i][j] >= early_stopping_round_) {
            ret = best_msg_[i][j];
          }
        }
      }
    }
  }
  for (auto& p : met_pairs) best_msg_[p.first][p.second] = msg.str();
  return ret;
}

std::vector<double> GBDT::GetEvalAt(int data_idx) {
  LGBM_CHECK(data_idx >= 0 && data_idx <= static_cast<int>(valid_score_updater_.size()));
  std::vector<double> ret;
  if (data_idx == 0) {
    for (auto* m : training_metrics_) {
      for (double v : EvalTrain(m)) ret.push_back(v);
    }
  } else {
    const int i = data_idx - 1;
    for (size_t j = 0; j < valid_metrics_[i].size(); ++j) {
      for (double v : EvalValid(i, static_cast<int>(j))) ret.push_back(v);  // device-resident scores when possible
    }
  }
  return ret;
}

int GBDT::GetEvalCounts() const {
  int n = 0;
  for (auto* m : training_metrics_) n += static_cast<int>(m->GetName().size());
  if (n == 0 && !valid_metrics_.empty()) {
    for (auto* m : valid_metrics_[0]) n += static_cast<int>(m->GetName().size());
  }
  return n;
}

std::vector<std::string> GBDT::GetEvalNames() const {
  std::vector<std::string> out;
  const std::vector<const Metric*>* ms = &training_metrics_;
  if (ms->empty() && !valid_metrics_.empty()) ms = &valid_metrics_[0];
  for (auto* m : *ms) {
    for (auto& n : m->GetName()) out.push_back(n);
  }
  return out;
}

int64_t GBDT::GetNumPredictAt(int data_idx) const {
  const data_size_t n = data_idx == 0 ? train_score_updater_->num_data() : valid_score_updater_[data_idx - 1]->num_data();
  return static_cast<int64_t>(n) * num_class_;
}

void GBDT::GetPredictAt(int data_idx, double* out, int64_t* out_len) {
  LGBM_CHECK(data_idx >= 0 && data_idx <= static_cast<int>(valid_score_updater_.size()));
  const double* raw;
  data_size_t n;
  if (data_idx == 0) {
    if (train_score_updater_ == nullptr) {
      Log::Fatal("GetPredictAt: the booster holds no training data (a booster loaded from a model, or one whose "
                 "dataset was freed)");
    }
    raw = HostTrainScore();
    n = num_data_;
  } else {
    raw = valid_score_updater_[data_idx - 1]->score();
    n = valid_score_updater_[data_idx - 1]->num_data();
  }
  *out_len = static_cast<int64_t>(n) * num_class_;
  if (objective_ != nullptr) {
#pragma omp parallel for schedule(static)
    for (data_size_t i = 0; i < n; ++i) {
      std::vector<double> tin(num_tree_per_iteration_), tout(num_class_);
      for (int k = 0; k < num_tree_per_iteration_; ++k) tin[k] = raw[static_cast<size_t>(k) * n + i];
      objective_->ConvertOutput(tin.data(), tout.data());
      for (int k = 0; k < num_class_; ++k) out[static_cast<size_t>(k) * n + i] = tout[k];
    }
  } else {
    std::copy(raw, raw + static_cast<size_t>(n) * num_tree_per_iteration_, out);
  }
}

void GBDT::MergeFrom(const GBDT* other) {
  // models of `other` first, then ours (reference gbdt.h:61-82)
  std::vector<std::unique_ptr<Tree>> old;
  for (auto& t : models_) old.push_back(std::move(t));
  models_.clear();
  for (auto& t : other->models_) models_.emplace_back(new Tree(*t));
  num_init_iteration_ = static_cast<int>(models_.size()) / num_tree_per_iteration_;
  for (auto& t : old) models_.push_back(std::move(t));
  num_iteration_for_pred_ = static_cast<int>(models_.size()) / num_tree_per_iteration_;
}

void GBDT::ShuffleModels(int start_iter, int end_iter) {
  const int total = static_cast<int>(models_.size()) / num_tree_per_iteration_;
  start_iter = std::max(0, start_iter);
  if (end_iter <= 0) end_iter = total;
  end_iter = std::min(total, end_iter);
  std::vector<std::unique_ptr<Tree>> orig;
  for (auto& t : models_) orig.push_back(std::move(t));
  std::vector<int> idx;
  for (int i = start_iter; i < end_iter; ++i) idx.push_back(i);
  Random rnd(0);
  for (int i = 0; i < static_cast<int>(idx.size()) - 1; ++i) {
    int j = rnd.NextShort(i + 1, static_cast<int>(idx.size()));
    std::swap(idx[i], idx[j]);
  }
  models_.clear();
  for (int i = 0; i < start_iter; ++i) {
    for (int k = 0; k < num_tree_per_iteration_; ++k) models_.push_back(std::move(orig[i * num_tree_per_iteration_ + k]));
  }
  for (int i : idx) {
    for (int k = 0; k < num_tree_per_iteration_; ++k) models_.push_back(std::move(orig[i * num_tree_per_iteration_ + k]));
  }
  for (int i = end_iter; i < total; ++i) {
    for (int k = 0; k < num_tree_per_iteration_; ++k) models_.push_back(std::move(orig[i * num_tree_per_iteration_ + k]));
  }
}

}  // namespace lgbm_amd
