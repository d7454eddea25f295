// Feature sub-sampling per tree (feature_fraction) and per node
// (feature_fraction_bynode) plus interaction constraints.  Same LCG stream and the same
// sampling calls as reference src/treelearner/col_sampler.hpp:20-202, so the sampled
// feature sets are identical for a given feature_fraction_seed.  Used by both the CPU
// and the device learners (masks are uploaded to HBM by the latter).
#pragma once

#include <cstring>
#include <unordered_set>
#include <vector>

#include "lgbm_amd/common.h"
#include "lgbm_amd/config.h"
#include "lgbm_amd/dataset.h"
#include "lgbm_amd/random.h"
#include "lgbm_amd/tree.h"

namespace lgbm_amd {

class ColSampler {
 public:
  explicit ColSampler(const Config* cfg)
      : frac_tree_(cfg->feature_fraction), frac_node_(cfg->feature_fraction_bynode),
        seed_(cfg->feature_fraction_seed), rnd_(cfg->feature_fraction_seed) {
    for (auto& c : cfg->interaction_constraints_vector) constraints_.emplace_back(c.begin(), c.end());
  }

  static int GetCnt(size_t total, double frac) {
    const int mn = std::min(1, static_cast<int>(total));
    return std::max(static_cast<int>(common::RoundInt(total * frac)), mn);
  }

  void SetTrainingData(const Dataset* data) {
    data_ = data;
    used_.assign(data->num_features(), 1);
    valid_.clear();
    for (int i = 0; i < data->num_total_features(); ++i) {
      if (data->InnerFeatureIndex(i) >= 0) valid_.push_back(i);
    }
    Refresh();
  }

  void SetConfig(const Config* cfg) {
    frac_tree_ = cfg->feature_fraction;
    frac_node_ = cfg->feature_fraction_bynode;
    if (seed_ != cfg->feature_fraction_seed) {
      seed_ = cfg->feature_fraction_seed;
      rnd_ = Random(seed_);
    }
    constraints_.clear();
    for (auto& c : cfg->interaction_constraints_vector) constraints_.emplace_back(c.begin(), c.end());
    used_.assign(data_->num_features(), 1);
    Refresh();
  }

  void ResetByTree() {
    if (!need_reset_tree_) return;
    std::fill(used_.begin(), used_.end(), 0);
    used_idx_ = rnd_.Sample(static_cast<int>(valid_.size()), used_cnt_tree_);
    for (int i : used_idx_) used_[data_->InnerFeatureIndex(valid_[i])] = 1;
  }

  std::vector<int8_t> GetByNode(const Tree* tree, int leaf) {
    std::unordered_set<int> allowed;
    if (!constraints_.empty()) {
      const std::vector<int> branch = tree->branch_features(leaf);
      allowed.insert(branch.begin(), branch.end());
      for (auto& c : constraints_) {
        if (branch.empty()) allowed.insert(c.begin(), c.end());
        int found = 0;
        for (int f : branch) {
          if (c.count(f) == 0) break;
          ++found;
          if (found == static_cast<int>(branch.size())) {
            allowed.insert(c.begin(), c.end());
            break;
          }
        }
      }
    }
    std::vector<int8_t> ret(data_->num_features(), 0);
    if (frac_node_ >= 1.0f) {
      if (constraints_.empty()) return std::vector<int8_t>(data_->num_features(), 1);
      for (int f : allowed) {
        int inner = data_->InnerFeatureIndex(f);
        if (inner >= 0) ret[inner] = 1;
      }
      return ret;
    }
    if (need_reset_tree_) {
      int cnt = GetCnt(used_idx_.size(), frac_node_);
      std::vector<int> filtered;
      const std::vector<int>* pool = &used_idx_;
      if (!constraints_.empty()) {
        for (int fi : used_idx_) {
          if (allowed.count(valid_[fi])) filtered.push_back(fi);
        }
        cnt = std::min(cnt, static_cast<int>(filtered.size()));
        pool = &filtered;
      }
      auto s = rnd_.Sample(static_cast<int>(pool->size()), cnt);
      for (int i : s) ret[data_->InnerFeatureIndex(valid_[(*pool)[i]])] = 1;
    } else {
      int cnt = GetCnt(valid_.size(), frac_node_);
      std::vector<int> filtered;
      const std::vector<int>* pool = &valid_;
      if (!constraints_.empty()) {
        for (int f : valid_) {
          if (allowed.count(f)) filtered.push_back(f);
        }
        pool = &filtered;
        cnt = std::min(cnt, static_cast<int>(filtered.size()));
      }
      auto s = rnd_.Sample(static_cast<int>(pool->size()), cnt);
      for (int i : s) ret[data_->InnerFeatureIndex((*pool)[i])] = 1;
    }
    return ret;
  }

  // per-node masks of the next `calls` GetByNode calls (no interaction constraints: the
  // draws do not depend on the tree), from a copy of the generator -- the device learner
  // uploads them before a tree and replays the calls the tree made (AdvanceByNode)
  std::vector<int8_t> PeekByNodeMasks(int calls) const {
    ColSampler copy(*this);
    std::vector<int8_t> out;
    out.reserve(static_cast<size_t>(calls) * data_->num_features());
    for (int c = 0; c < calls; ++c) {
      auto m = copy.GetByNode(nullptr, 0);
      out.insert(out.end(), m.begin(), m.end());
    }
    return out;
  }
  void AdvanceByNode(int calls) {
    for (int c = 0; c < calls; ++c) (void)GetByNode(nullptr, 0);
  }

  // the device's by-node sampling under interaction constraints (bynode_kernels.hip): the
  // tree's node pool as inner features in GetByNode's order, the sample size before the
  // constraint filter, and the generator state (read before, set after a device tree)
  std::vector<int32_t> NodePoolInner() const {
    std::vector<int32_t> out;
    if (need_reset_tree_) {
      for (int fi : used_idx_) out.push_back(data_->InnerFeatureIndex(valid_[fi]));
    } else {
      for (int f : valid_) out.push_back(data_->InnerFeatureIndex(f));
    }
    return out;
  }
  int NodeSampleCount() const {
    return GetCnt(need_reset_tree_ ? used_idx_.size() : valid_.size(), frac_node_);
  }
  uint32_t rng_state() const { return rnd_.state(); }
  void set_rng_state(uint32_t x) { rnd_ = Random(static_cast<int>(x)); }

  const std::vector<int8_t>& is_feature_used_bytree() const { return used_; }
  bool has_interaction_constraints() const { return !constraints_.empty(); }
  bool need_by_node() const { return frac_node_ < 1.0f || !constraints_.empty(); }

 private:
  void Refresh() {
    if (frac_tree_ >= 1.0f) {
      need_reset_tree_ = false;
      used_cnt_tree_ = static_cast<int>(valid_.size());
    } else {
      need_reset_tree_ = true;
      used_cnt_tree_ = GetCnt(valid_.size(), frac_tree_);
    }
    ResetByTree();
  }

  const Dataset* data_ = nullptr;
  double frac_tree_, frac_node_;
  bool need_reset_tree_ = false;
  int used_cnt_tree_ = 0;
  int seed_;
  Random rnd_;
  std::vector<int8_t> used_;
  std::vector<int> used_idx_;
  std::vector<int> valid_;
  std::vector<std::unordered_set<int>> constraints_;
};

}  // namespace lgbm_amd
