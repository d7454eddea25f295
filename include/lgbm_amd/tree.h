// One regression tree (host representation + text/JSON/if-else serialisation).
// Node layout and the v3 text format are byte-compatible with the reference
// (include/LightGBM/tree.h:24-602, src/io/tree.cpp:223-260 ToString, :496 parser):
// internal nodes 0..num_leaves-2, children encoded as ~leaf for leaves, decision_type
// bit0 categorical, bit1 default-left, bits2-3 missing type.
#pragma once

#include <string>
#include <unordered_map>
#include <vector>

#include "lgbm_amd/common.h"
#include "lgbm_amd/meta.h"

namespace lgbm_amd {

class Dataset;

class Tree {
 public:
  Tree(int max_leaves, bool track_branch_features);
  // parse a "num_leaves=..." block; *used_len = consumed bytes
  Tree(const char* str, size_t* used_len);

  int Split(int leaf, int feature, int real_feature, uint32_t threshold_bin, double threshold_double,
            double left_value, double right_value, int left_cnt, int right_cnt, double left_weight,
            double right_weight, float gain, MissingType missing_type, bool default_left);
  int SplitCategorical(int leaf, int feature, int real_feature, const uint32_t* threshold_bin, int num_threshold_bin,
                       const uint32_t* threshold, int num_threshold, double left_value, double right_value,
                       int left_cnt, int right_cnt, double left_weight, double right_weight, float gain,
                       MissingType missing_type);

  double LeafOutput(int leaf) const { return leaf_value_[leaf]; }
  void SetLeafOutput(int leaf, double v) { leaf_value_[leaf] = MaybeRoundToZero(v); }
  int num_leaves() const { return num_leaves_; }
  int num_cat() const { return num_cat_; }
  int leaf_depth(int leaf) const { return leaf_depth_[leaf]; }
  int leaf_parent(int leaf) const { return leaf_parent_[leaf]; }
  int leaf_count(int leaf) const { return leaf_count_[leaf]; }
  double leaf_weight(int leaf) const { return leaf_weight_[leaf]; }
  int split_feature(int node) const { return split_feature_[node]; }
  int split_feature_inner(int node) const { return split_feature_inner_[node]; }
  double split_gain(int node) const { return split_gain_[node]; }
  double threshold(int node) const { return threshold_[node]; }
  uint32_t threshold_in_bin(int node) const { return threshold_in_bin_[node]; }
  int8_t decision_type(int node) const { return decision_type_[node]; }
  int left_child(int node) const { return left_child_[node]; }
  int right_child(int node) const { return right_child_[node]; }
  double internal_value(int node) const { return internal_value_[node]; }
  double internal_weight(int node) const { return internal_weight_[node]; }
  int internal_count(int node) const { return internal_count_[node]; }
  int data_count(int node) const { return node >= 0 ? internal_count_[node] : leaf_count_[~node]; }
  double shrinkage() const { return shrinkage_; }
  bool IsNumericalSplit(int node) const { return !(decision_type_[node] & kCategoricalMask); }
  const std::vector<int>& branch_features(int leaf) const { return branch_features_[leaf]; }
  const std::vector<int>& cat_boundaries_inner() const { return cat_boundaries_inner_; }
  const std::vector<uint32_t>& cat_threshold_inner() const { return cat_threshold_inner_; }
  const std::vector<int>& cat_boundaries() const { return cat_boundaries_; }
  const std::vector<uint32_t>& cat_threshold() const { return cat_threshold_; }
  int NextLeafId() const { return num_leaves_; }

  void Shrinkage(double rate);
  void AddBias(double v);
  void AsConstantTree(double v) {
    num_leaves_ = 1;
    shrinkage_ = 1.0;
    leaf_value_[0] = v;
  }
  double GetUpperBoundValue() const;
  double GetLowerBoundValue() const;

  // prediction on raw feature values (dense row indexed by real feature id)
  double Predict(const double* x) const { return num_leaves_ > 1 ? leaf_value_[GetLeaf(x)] : leaf_value_[0]; }
  int PredictLeafIndex(const double* x) const { return num_leaves_ > 1 ? GetLeaf(x) : 0; }
  double PredictByMap(const std::unordered_map<int, double>& x) const;
  int PredictLeafIndexByMap(const std::unordered_map<int, double>& x) const;
  // TreeSHAP (Lundberg et al., arXiv:1706.06060); output has num_features+1 entries
  void PredictContrib(const double* x, int num_features, double* out);
  void PredictContribByMap(const std::unordered_map<int, double>& x, int num_features,
                           std::unordered_map<int, double>* out);
  // add this tree's output to `score` for binned rows (host path)
  void AddPredictionToScore(const Dataset* data, data_size_t num_data, double* score) const;
  void AddPredictionToScore(const Dataset* data, const data_size_t* idx, data_size_t n, double* score) const;

  std::string ToString() const;
  std::string ToJSON() const;
  std::string ToIfElse(int index, bool predict_leaf_index) const;

  void RecomputeMaxDepth();
  int max_depth() const { return max_depth_; }

  static bool IsZero(double v) { return v >= -kZeroThreshold && v <= kZeroThreshold; }
  static double MaybeRoundToZero(double v) { return IsZero(v) ? 0.0 : v; }
  static int8_t GetMissingType(int8_t dt) { return (dt >> 2) & 3; }

  // decision on a raw value at `node`; returns child index (>=0 internal, <0 ~leaf)
  int NumericalDecision(double fval, int node) const;
  int CategoricalDecision(double fval, int node) const;
  int Decision(double fval, int node) const {
    return (decision_type_[node] & kCategoricalMask) ? CategoricalDecision(fval, node) : NumericalDecision(fval, node);
  }
  // decision on a feature bin (binned data)
  int DecisionInner(uint32_t fbin, int node, uint32_t default_bin, uint32_t max_bin) const;

 private:
  void SplitCommon(int leaf, int feature, int real_feature, double left_value, double right_value, int left_cnt,
                   int right_cnt, double left_weight, double right_weight, float gain);
  int GetLeaf(const double* x) const;
  void RecomputeLeafDepths(int node, int depth);
  std::string NodeToJSON(int index) const;
  std::string NodeToIfElse(int index, bool predict_leaf_index) const;
  std::string NodeToIfElseByMap(int index, bool predict_leaf_index) const;
  std::string NumericalDecisionIfElse(int node) const;
  std::string CategoricalDecisionIfElse(int node) const;
  double ExpectedValue() const;

  struct PathElement {
    int feature_index;
    double zero_fraction;
    double one_fraction;
    double pweight;
  };
  static void ExtendPath(PathElement* path, int depth, double zero_fraction, double one_fraction, int feature);
  static void UnwindPath(PathElement* path, int depth, int path_index);
  static double UnwoundPathSum(const PathElement* path, int depth, int path_index);
  template <typename GetValue, typename Phi>
  void TreeShapRec(const GetValue& get, Phi& phi, int node, int depth, PathElement* parent_path,
                   double parent_zero, double parent_one, int parent_feature) const;

  int max_leaves_;
  int num_leaves_;
  std::vector<int> left_child_, right_child_;
  std::vector<int> split_feature_inner_, split_feature_;
  std::vector<uint32_t> threshold_in_bin_;
  std::vector<double> threshold_;
  int num_cat_ = 0;
  std::vector<int> cat_boundaries_inner_;
  std::vector<uint32_t> cat_threshold_inner_;
  std::vector<int> cat_boundaries_;
  std::vector<uint32_t> cat_threshold_;
  std::vector<int8_t> decision_type_;
  std::vector<float> split_gain_;
  std::vector<int> leaf_parent_;
  std::vector<double> leaf_value_, leaf_weight_;
  std::vector<int> leaf_count_;
  std::vector<double> internal_value_, internal_weight_;
  std::vector<int> internal_count_;
  std::vector<int> leaf_depth_;
  bool track_branch_features_ = false;
  std::vector<std::vector<int>> branch_features_;
  double shrinkage_ = 1.0;
  int max_depth_ = -1;
};

}  // namespace lgbm_amd
