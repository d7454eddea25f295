// Cost-effective gradient boosting: see cegb.h.
#include "cegb.h"

#include <omp.h>

#include "lgbm_amd/log.h"
#include "lgbm_amd/tree.h"

namespace lgbm_amd {

void CostEffectiveGB::Init(const Config* config, const Dataset* data) {
  config_ = config;
  data_ = data;
  const int total = data->num_total_features();
  if (!config->cegb_penalty_feature_coupled.empty() &&
      static_cast<int>(config->cegb_penalty_feature_coupled.size()) != total) {
    Log::Fatal("cegb_penalty_feature_coupled should be the same size as feature number.");
  }
  if (!config->cegb_penalty_feature_lazy.empty() &&
      static_cast<int>(config->cegb_penalty_feature_lazy.size()) != total) {
    Log::Fatal("cegb_penalty_feature_lazy should be the same size as feature number.");
  }
  if (init_) {  // the model-wide state survives config / data resets (reference Init)
    if (static_cast<int>(lazy_.size()) < config->num_leaves) {
      remembered_.resize(static_cast<size_t>(config->num_leaves) * num_features_);
      lazy_.resize(config->num_leaves, std::vector<double>(num_features_, 0.0));
    }
    if (!config->cegb_penalty_feature_lazy.empty() && paid_.empty()) {
      paid_.assign((static_cast<uint64_t>(num_features_) * num_data_ + 63) / 64, 0ull);
    }
    return;
  }
  num_features_ = data->num_features();
  num_data_ = data->num_data();
  remembered_.assign(static_cast<size_t>(config->num_leaves) * num_features_, SplitInfo());
  used_in_split_.assign(num_features_, 0);
  lazy_.assign(config->num_leaves, std::vector<double>(num_features_, 0.0));
  if (!config->cegb_penalty_feature_lazy.empty()) {
    paid_.assign((static_cast<uint64_t>(num_features_) * num_data_ + 63) / 64, 0ull);
  }
  init_ = true;
}

void CostEffectiveGB::PrepareLeaf(int leaf, const data_size_t* rows, data_size_t cnt) {
  if (config_->cegb_penalty_feature_lazy.empty() || leaf < 0) return;
  std::vector<double>& out = lazy_[leaf];
#pragma omp parallel for schedule(dynamic, 1)
  for (int f = 0; f < num_features_; ++f) {
    const double pen = config_->cegb_penalty_feature_lazy[data_->RealFeatureIndex(f)];
    data_size_t unpaid = 0;
    for (data_size_t i = 0; i < cnt; ++i) unpaid += RowPaid(f, rows[i]) ? 0 : 1;
    // the reference adds the penalty once per unpaid row (same rounding as a running sum)
    double total = 0.0;
    for (data_size_t i = 0; i < unpaid; ++i) total += pen;
    out[f] = total;
  }
}

double CostEffectiveGB::DeltaGain(int inner, int real, int leaf, data_size_t leaf_rows, const SplitInfo& raw) {
  const Config& c = *config_;
  double delta = c.cegb_tradeoff * c.cegb_penalty_split * leaf_rows;
  if (!c.cegb_penalty_feature_coupled.empty() && !used_in_split_[inner]) {
    delta += c.cegb_tradeoff * c.cegb_penalty_feature_coupled[real];
  }
  if (!c.cegb_penalty_feature_lazy.empty()) delta += c.cegb_tradeoff * lazy_[leaf][inner];
  remembered_[static_cast<size_t>(leaf) * num_features_ + inner] = raw;
  return delta;
}

void CostEffectiveGB::OnSplit(const Tree* tree, int best_leaf, const SplitInfo& split, const data_size_t* rows,
                              data_size_t cnt, std::vector<SplitInfo>* best_per_leaf) {
  const Config& c = *config_;
  const int inner = data_->InnerFeatureIndex(split.feature);
  if (!c.cegb_penalty_feature_coupled.empty() && !used_in_split_[inner]) {
    used_in_split_[inner] = 1;
    // refund the coupled penalty to the other leaves' remembered candidates on this feature
    const double refund = c.cegb_tradeoff * c.cegb_penalty_feature_coupled[split.feature];
    for (int i = 0; i < tree->num_leaves(); ++i) {
      if (i == best_leaf) continue;
      SplitInfo& cand = remembered_[static_cast<size_t>(i) * num_features_ + inner];
      cand.gain += refund;
      SplitInfo& cur = (*best_per_leaf)[i];
      if (cur.gain > kMinScore && cand > cur) cur = cand;
    }
  }
  if (!c.cegb_penalty_feature_lazy.empty()) {
    for (data_size_t i = 0; i < cnt; ++i) {
      const uint64_t bit = static_cast<uint64_t>(inner) * num_data_ + static_cast<uint64_t>(rows[i]);
      paid_[bit >> 6] |= 1ull << (bit & 63);
    }
  }
}

}  // namespace lgbm_amd
