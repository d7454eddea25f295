// Per-leaf output bounds for monotone constraints (reference
// src/treelearner/monotone_constraints.hpp):
//  * basic: a monotone split bounds its two children by the midpoint of their outputs, and
//    the bounds are inherited down the subtree;
//  * intermediate: the children are bounded by each other's outputs, and a split inside a
//    monotone subtree also tightens the bounds of the leaves elsewhere in the tree that are
//    contiguous with the split leaves across a monotone split (found by walking up to each
//    monotone ancestor and down its other subtree).  Those leaves' best splits must then be
//    recomputed by the learner (Update returns them).
#pragma once

#include <limits>
#include <vector>

#include "lgbm_amd/config.h"
#include "lgbm_amd/split_info.h"
#include "lgbm_amd/split_math.h"
#include "lgbm_amd/tree.h"

namespace lgbm_amd {

class LeafConstraints {
 public:
  std::vector<ConstraintRange> entries;

  void Init(int num_leaves, const Config* cfg = nullptr);
  bool intermediate() const { return intermediate_; }
  // before tree->Split of `leaf` (whose right child becomes leaf `new_leaf`)
  void BeforeSplit(const Tree* tree, int leaf, int new_leaf, int8_t mono);
  // after the split; returns the leaves (other than the two children) whose bounds changed
  std::vector<int> Update(const Tree* tree, bool is_numerical, int leaf, int new_leaf, int8_t mono,
                          double right_out, double left_out, int split_inner, const SplitInfo& split,
                          const std::vector<SplitInfo>& best_split_per_leaf);

 private:
  struct Path {  // the splits met going up from the split leaf that matter going down
    std::vector<int> feature;
    std::vector<uint32_t> threshold;
    std::vector<bool> from_right;
  };
  void GoUp(const Tree* tree, int node, Path* path, int split_inner, const SplitInfo& split,
            const std::vector<SplitInfo>& best);
  void GoDown(const Tree* tree, int node, const Path& path, bool update_max, int split_inner, const SplitInfo& split,
              bool use_left, bool use_right, const std::vector<SplitInfo>& best);

  bool intermediate_ = false;
  const Config* cfg_ = nullptr;
  std::vector<char> in_monotone_subtree_;  // per leaf
  std::vector<int> node_parent_;           // per internal node
  std::vector<int> to_update_;
};

}  // namespace lgbm_amd
