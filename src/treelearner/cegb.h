// Cost-effective gradient boosting (reference
// src/treelearner/cost_effective_gradient_boosting.hpp:22-156; used from
// serial_tree_learner.cpp:66,111,144 (setup), :547 (split), :723 (gain)).
//
// A candidate split's gain is reduced by
//   tradeoff * (penalty_split * rows_in_leaf
//               + penalty_feature_coupled[f]      if f was never split on by this model
//               + penalty_feature_lazy[f] * rows of the leaf that never went through a
//                 split on f)
// The raw candidate of every (leaf, feature) is remembered: when a feature is split on for
// the first time its coupled penalty is refunded to the other leaves' remembered candidates
// (which may then become their best split), and a lazy feature's rows are marked as paid.
//
// Lazy costs are counted once per leaf and scan (PrepareLeaf, before the parallel feature
// loop) instead of per (feature, row) lookup inside it; the counts are the same because the
// paid-row bitset only changes at a split.
#pragma once

#include <cstdint>
#include <vector>

#include "lgbm_amd/config.h"
#include "lgbm_amd/dataset.h"
#include "lgbm_amd/split_info.h"

namespace lgbm_amd {

class Tree;

class CostEffectiveGB {
 public:
  static bool Enabled(const Config& c) {
    return c.cegb_tradeoff < 1.0 || c.cegb_penalty_split > 0.0 || !c.cegb_penalty_feature_coupled.empty() ||
           !c.cegb_penalty_feature_lazy.empty();
  }
  // first call allocates; later calls (config / data resets) keep the model-wide state
  void Init(const Config* config, const Dataset* data);
  // lazy penalties of `leaf` for every feature from its rows (no-op without lazy penalties)
  void PrepareLeaf(int leaf, const data_size_t* rows, data_size_t cnt);
  // penalty to subtract from `raw` (the feature's best threshold for `leaf`); remembers raw
  double DeltaGain(int inner, int real, int leaf, data_size_t leaf_rows, const SplitInfo& raw);
  // before `best_leaf` is split by `split`: refund coupled penalties, mark lazy rows paid
  void OnSplit(const Tree* tree, int best_leaf, const SplitInfo& split, const data_size_t* rows, data_size_t cnt,
               std::vector<SplitInfo>* best_per_leaf);
  // features the model has split on (coupled penalties paid); the device learner mirrors them
  const std::vector<char>& used_in_split() const { return used_in_split_; }
  void set_used_in_split(const std::vector<char>& u) { used_in_split_ = u; }

 private:
  bool RowPaid(int inner, data_size_t row) const {
    const uint64_t bit = static_cast<uint64_t>(inner) * num_data_ + static_cast<uint64_t>(row);
    return (paid_[bit >> 6] >> (bit & 63)) & 1ull;
  }

  const Config* config_ = nullptr;
  const Dataset* data_ = nullptr;
  bool init_ = false;
  int num_features_ = 0;
  data_size_t num_data_ = 0;
  std::vector<SplitInfo> remembered_;        // [num_leaves][num_features]
  std::vector<char> used_in_split_;          // [num_features] (coupled)
  std::vector<uint64_t> paid_;               // [num_features][num_data] bits (lazy)
  std::vector<std::vector<double>> lazy_;    // [num_leaves][num_features] current lazy cost
};

}  // namespace lgbm_amd
