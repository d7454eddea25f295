// Tree growth bookkeeping, prediction, TreeSHAP and (de)serialisation.
// Text format byte-compatible with the reference (src/io/tree.cpp:223-260 ToString,
// :262-335 ToJSON, :376-494 if-else codegen, :496-620 parser).
#include "lgbm_amd/tree.h"

#include <omp.h>

#include <cmath>
#include <functional>
#include <iomanip>
#include <sstream>

#include "lgbm_amd/dataset.h"
#include "lgbm_amd/log.h"

namespace lgbm_amd {

Tree::Tree(int max_leaves, bool track_branch_features)
    : max_leaves_(max_leaves), num_leaves_(1), track_branch_features_(track_branch_features) {
  const int ni = std::max(max_leaves - 1, 1);
  left_child_.assign(ni, 0);
  right_child_.assign(ni, 0);
  split_feature_inner_.assign(ni, 0);
  split_feature_.assign(ni, 0);
  threshold_in_bin_.assign(ni, 0);
  threshold_.assign(ni, 0.0);
  decision_type_.assign(ni, 0);
  split_gain_.assign(ni, 0.0f);
  internal_value_.assign(ni, 0.0);
  internal_weight_.assign(ni, 0.0);
  internal_count_.assign(ni, 0);
  leaf_parent_.assign(max_leaves, -1);
  leaf_value_.assign(max_leaves, 0.0);
  leaf_weight_.assign(max_leaves, 0.0);
  leaf_count_.assign(max_leaves, 0);
  leaf_depth_.assign(max_leaves, 0);
  if (track_branch_features_) branch_features_.assign(max_leaves, {});
  cat_boundaries_.push_back(0);
  cat_boundaries_inner_.push_back(0);
}

void Tree::SplitCommon(int leaf, int feature, int real_feature, double left_value, double right_value,
                       int left_cnt, int right_cnt, double left_weight, double right_weight, float gain) {
  const int node = num_leaves_ - 1;
  const int parent = leaf_parent_[leaf];
  if (parent >= 0) {
    if (left_child_[parent] == ~leaf) left_child_[parent] = node;
    else right_child_[parent] = node;
  }
  split_feature_inner_[node] = feature;
  split_feature_[node] = real_feature;
  split_gain_[node] = gain;
  left_child_[node] = ~leaf;
  right_child_[node] = ~num_leaves_;
  leaf_parent_[leaf] = node;
  leaf_parent_[num_leaves_] = node;
  internal_weight_[node] = leaf_weight_[leaf];
  internal_value_[node] = leaf_value_[leaf];
  internal_count_[node] = left_cnt + right_cnt;
  leaf_value_[leaf] = std::isnan(left_value) ? 0.0 : left_value;
  leaf_weight_[leaf] = left_weight;
  leaf_count_[leaf] = left_cnt;
  leaf_value_[num_leaves_] = std::isnan(right_value) ? 0.0 : right_value;
  leaf_weight_[num_leaves_] = right_weight;
  leaf_count_[num_leaves_] = right_cnt;
  leaf_depth_[num_leaves_] = leaf_depth_[leaf] + 1;
  leaf_depth_[leaf]++;
  if (track_branch_features_) {
    branch_features_[num_leaves_] = branch_features_[leaf];
    branch_features_[num_leaves_].push_back(real_feature);
    branch_features_[leaf].push_back(real_feature);
  }
}

int Tree::Split(int leaf, int feature, int real_feature, uint32_t threshold_bin, double threshold_double,
                double left_value, double right_value, int left_cnt, int right_cnt, double left_weight,
                double right_weight, float gain, MissingType missing_type, bool default_left) {
  SplitCommon(leaf, feature, real_feature, left_value, right_value, left_cnt, right_cnt, left_weight, right_weight,
              gain);
  const int node = num_leaves_ - 1;
  int8_t dt = 0;
  if (default_left) dt |= kDefaultLeftMask;
  dt |= static_cast<int8_t>(static_cast<int8_t>(missing_type) << 2);
  decision_type_[node] = dt;
  threshold_in_bin_[node] = threshold_bin;
  threshold_[node] = threshold_double;
  ++num_leaves_;
  return num_leaves_ - 1;
}

int Tree::SplitCategorical(int leaf, int feature, int real_feature, const uint32_t* threshold_bin,
                           int num_threshold_bin, const uint32_t* threshold, int num_threshold, double left_value,
                           double right_value, int left_cnt, int right_cnt, double left_weight, double right_weight,
                           float gain, MissingType missing_type) {
  SplitCommon(leaf, feature, real_feature, left_value, right_value, left_cnt, right_cnt, left_weight, right_weight,
              gain);
  const int node = num_leaves_ - 1;
  int8_t dt = kCategoricalMask;
  dt |= static_cast<int8_t>(static_cast<int8_t>(missing_type) << 2);
  decision_type_[node] = dt;
  threshold_in_bin_[node] = static_cast<uint32_t>(num_cat_);
  threshold_[node] = num_cat_;
  ++num_cat_;
  cat_boundaries_.push_back(cat_boundaries_.back() + num_threshold);
  for (int i = 0; i < num_threshold; ++i) cat_threshold_.push_back(threshold[i]);
  cat_boundaries_inner_.push_back(cat_boundaries_inner_.back() + num_threshold_bin);
  for (int i = 0; i < num_threshold_bin; ++i) cat_threshold_inner_.push_back(threshold_bin[i]);
  ++num_leaves_;
  return num_leaves_ - 1;
}

void Tree::Shrinkage(double rate) {
  for (int i = 0; i < num_leaves_ - 1; ++i) {
    leaf_value_[i] = MaybeRoundToZero(leaf_value_[i] * rate);
    internal_value_[i] = MaybeRoundToZero(internal_value_[i] * rate);
  }
  leaf_value_[num_leaves_ - 1] = MaybeRoundToZero(leaf_value_[num_leaves_ - 1] * rate);
  shrinkage_ *= rate;
}

void Tree::AddBias(double v) {
  for (int i = 0; i < num_leaves_ - 1; ++i) {
    leaf_value_[i] = MaybeRoundToZero(leaf_value_[i] + v);
    internal_value_[i] = MaybeRoundToZero(internal_value_[i] + v);
  }
  leaf_value_[num_leaves_ - 1] = MaybeRoundToZero(leaf_value_[num_leaves_ - 1] + v);
  shrinkage_ = 1.0;
}

double Tree::GetUpperBoundValue() const {
  double v = leaf_value_[0];
  for (int i = 1; i < num_leaves_; ++i) v = std::max(v, leaf_value_[i]);
  return v;
}

double Tree::GetLowerBoundValue() const {
  double v = leaf_value_[0];
  for (int i = 1; i < num_leaves_; ++i) v = std::min(v, leaf_value_[i]);
  return v;
}

int Tree::NumericalDecision(double fval, int node) const {
  const int8_t mt = GetMissingType(decision_type_[node]);
  if (std::isnan(fval) && mt != static_cast<int8_t>(MissingType::NaN)) fval = 0.0;
  if ((mt == static_cast<int8_t>(MissingType::Zero) && IsZero(fval)) ||
      (mt == static_cast<int8_t>(MissingType::NaN) && std::isnan(fval))) {
    return (decision_type_[node] & kDefaultLeftMask) ? left_child_[node] : right_child_[node];
  }
  return fval <= threshold_[node] ? left_child_[node] : right_child_[node];
}

int Tree::CategoricalDecision(double fval, int node) const {
  const int8_t mt = GetMissingType(decision_type_[node]);
  int iv = static_cast<int>(fval);
  if (iv < 0) {
    return right_child_[node];
  } else if (std::isnan(fval)) {
    if (mt == static_cast<int8_t>(MissingType::NaN)) return right_child_[node];
    iv = 0;
  }
  const int ci = static_cast<int>(threshold_[node]);
  if (common::FindInBitset(cat_threshold_.data() + cat_boundaries_[ci], cat_boundaries_[ci + 1] - cat_boundaries_[ci],
                           iv)) {
    return left_child_[node];
  }
  return right_child_[node];
}

int Tree::DecisionInner(uint32_t fbin, int node, uint32_t default_bin, uint32_t max_bin) const {
  const int8_t dt = decision_type_[node];
  if (dt & kCategoricalMask) {
    const int ci = static_cast<int>(threshold_in_bin_[node]);
    if (common::FindInBitset(cat_threshold_inner_.data() + cat_boundaries_inner_[ci],
                             cat_boundaries_inner_[ci + 1] - cat_boundaries_inner_[ci], fbin)) {
      return left_child_[node];
    }
    return right_child_[node];
  }
  const int8_t mt = GetMissingType(dt);
  if ((mt == static_cast<int8_t>(MissingType::Zero) && fbin == default_bin) ||
      (mt == static_cast<int8_t>(MissingType::NaN) && fbin == max_bin)) {
    return (dt & kDefaultLeftMask) ? left_child_[node] : right_child_[node];
  }
  return fbin <= threshold_in_bin_[node] ? left_child_[node] : right_child_[node];
}

int Tree::GetLeaf(const double* x) const {
  int node = 0;
  if (num_cat_ > 0) {
    while (node >= 0) node = Decision(x[split_feature_[node]], node);
  } else {
    while (node >= 0) node = NumericalDecision(x[split_feature_[node]], node);
  }
  return ~node;
}

double Tree::PredictByMap(const std::unordered_map<int, double>& x) const {
  return leaf_value_[PredictLeafIndexByMap(x)];
}

int Tree::PredictLeafIndexByMap(const std::unordered_map<int, double>& x) const {
  if (num_leaves_ <= 1) return 0;
  int node = 0;
  while (node >= 0) {
    auto it = x.find(split_feature_[node]);
    node = Decision(it == x.end() ? 0.0 : it->second, node);
  }
  return ~node;
}

void Tree::AddPredictionToScore(const Dataset* data, data_size_t n, double* score) const {
  AddPredictionToScore(data, nullptr, n, score);
}

void Tree::AddPredictionToScore(const Dataset* data, const data_size_t* idx, data_size_t n, double* score) const {
  if (num_leaves_ <= 1) {
    if (leaf_value_[0] != 0.0) {
#pragma omp parallel for schedule(static, 512) if (n >= 1024)
      for (data_size_t i = 0; i < n; ++i) score[idx ? idx[i] : i] += leaf_value_[0];
    }
    return;
  }
  std::vector<uint32_t> default_bins(num_leaves_ - 1), max_bins(num_leaves_ - 1);
  for (int i = 0; i < num_leaves_ - 1; ++i) {
    const BinMapper* m = data->FeatureBinMapper(split_feature_inner_[i]);
    default_bins[i] = m->GetDefaultBin();
    max_bins[i] = static_cast<uint32_t>(m->num_bin() - 1);
  }
  // (one bin reader per node and thread: each thread's rows ascend within its chunks)
#pragma omp parallel if (n >= 1024)
  {
    std::vector<Dataset::BinReader> rd(num_leaves_ - 1);
    for (int i = 0; i < num_leaves_ - 1; ++i) rd[i] = data->FeatureBinReader(split_feature_inner_[i]);
#pragma omp for schedule(static, 512)
    for (data_size_t i = 0; i < n; ++i) {
      const data_size_t r = idx ? idx[i] : i;
      int node = 0;
      while (node >= 0) {
        const uint32_t b = rd[node].Get(r);
        node = DecisionInner(b, node, default_bins[node], max_bins[node]);
      }
      score[r] += leaf_value_[~node];
    }
  }
}

// ------------------------------------------------------------------------- TreeSHAP
void Tree::ExtendPath(PathElement* path, int depth, double zero_fraction, double one_fraction, int feature) {
  path[depth].feature_index = feature;
  path[depth].zero_fraction = zero_fraction;
  path[depth].one_fraction = one_fraction;
  path[depth].pweight = depth == 0 ? 1.0 : 0.0;
  for (int i = depth - 1; i >= 0; --i) {
    path[i + 1].pweight += one_fraction * path[i].pweight * (i + 1) / static_cast<double>(depth + 1);
    path[i].pweight = zero_fraction * path[i].pweight * (depth - i) / static_cast<double>(depth + 1);
  }
}

void Tree::UnwindPath(PathElement* path, int depth, int path_index) {
  const double one = path[path_index].one_fraction;
  const double zero = path[path_index].zero_fraction;
  double next_one = path[depth].pweight;
  for (int i = depth - 1; i >= 0; --i) {
    if (one != 0) {
      const double tmp = path[i].pweight;
      path[i].pweight = next_one * (depth + 1) / static_cast<double>((i + 1) * one);
      next_one = tmp - path[i].pweight * zero * (depth - i) / static_cast<double>(depth + 1);
    } else {
      path[i].pweight = (path[i].pweight * (depth + 1)) / static_cast<double>(zero * (depth - i));
    }
  }
  for (int i = path_index; i < depth; ++i) {
    path[i].feature_index = path[i + 1].feature_index;
    path[i].zero_fraction = path[i + 1].zero_fraction;
    path[i].one_fraction = path[i + 1].one_fraction;
  }
}

double Tree::UnwoundPathSum(const PathElement* path, int depth, int path_index) {
  const double one = path[path_index].one_fraction;
  const double zero = path[path_index].zero_fraction;
  double next_one = path[depth].pweight;
  double total = 0;
  for (int i = depth - 1; i >= 0; --i) {
    if (one != 0) {
      const double tmp = next_one * (depth + 1) / static_cast<double>((i + 1) * one);
      total += tmp;
      next_one = path[i].pweight - tmp * zero * ((depth - i) / static_cast<double>(depth + 1));
    } else {
      total += (path[i].pweight / zero) / ((depth - i) / static_cast<double>(depth + 1));
    }
  }
  return total;
}

template <typename GetValue, typename Phi>
void Tree::TreeShapRec(const GetValue& get, Phi& phi, int node, int depth, PathElement* parent_path,
                       double parent_zero, double parent_one, int parent_feature) const {
  PathElement* path = parent_path + depth;
  if (depth > 0) std::copy(parent_path, parent_path + depth, path);
  ExtendPath(path, depth, parent_zero, parent_one, parent_feature);
  if (node < 0) {
    for (int i = 1; i <= depth; ++i) {
      const double w = UnwoundPathSum(path, depth, i);
      phi(path[i].feature_index) += w * (path[i].one_fraction - path[i].zero_fraction) * leaf_value_[~node];
    }
    return;
  }
  const int hot = Decision(get(split_feature_[node]), node);
  const int cold = hot == left_child_[node] ? right_child_[node] : left_child_[node];
  const double w = data_count(node);
  const double hot_zero = data_count(hot) / w;
  const double cold_zero = data_count(cold) / w;
  double in_zero = 1, in_one = 1;
  int pi = 0;
  for (; pi <= depth; ++pi) {
    if (path[pi].feature_index == split_feature_[node]) break;
  }
  if (pi != depth + 1) {
    in_zero = path[pi].zero_fraction;
    in_one = path[pi].one_fraction;
    UnwindPath(path, depth, pi);
    depth -= 1;
  }
  TreeShapRec(get, phi, hot, depth + 1, path, hot_zero * in_zero, in_one, split_feature_[node]);
  TreeShapRec(get, phi, cold, depth + 1, path, cold_zero * in_zero, 0, split_feature_[node]);
}

double Tree::ExpectedValue() const {
  if (num_leaves_ == 1) return leaf_value_[0];
  const double total = internal_count_[0];
  double v = 0;
  for (int i = 0; i < num_leaves_; ++i) v += (leaf_count_[i] / total) * leaf_value_[i];
  return v;
}

void Tree::RecomputeLeafDepths(int node, int depth) {
  if (node == 0) leaf_depth_.resize(num_leaves_);
  if (node < 0) {
    leaf_depth_[~node] = depth;
  } else {
    RecomputeLeafDepths(left_child_[node], depth + 1);
    RecomputeLeafDepths(right_child_[node], depth + 1);
  }
}

void Tree::RecomputeMaxDepth() {
  if (num_leaves_ == 1) {
    max_depth_ = 0;
    return;
  }
  if (leaf_depth_.empty()) RecomputeLeafDepths(0, 0);
  max_depth_ = leaf_depth_[0];
  for (int i = 1; i < num_leaves_; ++i) max_depth_ = std::max(max_depth_, leaf_depth_[i]);
}

void Tree::PredictContrib(const double* x, int num_features, double* out) {
  out[num_features] += ExpectedValue();
  if (num_leaves_ > 1) {
    if (max_depth_ < 0) RecomputeMaxDepth();
    const int L = max_depth_ + 1;
    std::vector<PathElement> buf(static_cast<size_t>(L) * (L + 1) / 2);
    auto get = [x](int f) { return x[f]; };
    auto phi = [out](int f) -> double& { return out[f]; };
    TreeShapRec(get, phi, 0, 0, buf.data(), 1, 1, -1);
  }
}

void Tree::PredictContribByMap(const std::unordered_map<int, double>& x, int num_features,
                               std::unordered_map<int, double>* out) {
  (*out)[num_features] += ExpectedValue();
  if (num_leaves_ > 1) {
    if (max_depth_ < 0) RecomputeMaxDepth();
    const int L = max_depth_ + 1;
    std::vector<PathElement> buf(static_cast<size_t>(L) * (L + 1) / 2);
    auto get = [&x](int f) {
      auto it = x.find(f);
      return it == x.end() ? 0.0 : it->second;
    };
    auto phi = [out](int f) -> double& { return (*out)[f]; };
    TreeShapRec(get, phi, 0, 0, buf.data(), 1, 1, -1);
  }
}

// ------------------------------------------------------------------------- text IO
std::string Tree::ToString() const {
  std::stringstream s;
  const size_t ni = static_cast<size_t>(num_leaves_ - 1);
  s << "num_leaves=" << num_leaves_ << '\n';
  s << "num_cat=" << num_cat_ << '\n';
  s << "split_feature=" << common::ArrayToStringFast(split_feature_, ni) << '\n';
  s << "split_gain=" << common::ArrayToStringFast(split_gain_, ni) << '\n';
  s << "threshold=" << common::ArrayToString(threshold_, ni) << '\n';
  std::vector<int> dt(decision_type_.begin(), decision_type_.end());
  s << "decision_type=" << common::ArrayToStringFast(dt, ni) << '\n';
  s << "left_child=" << common::ArrayToStringFast(left_child_, ni) << '\n';
  s << "right_child=" << common::ArrayToStringFast(right_child_, ni) << '\n';
  s << "leaf_value=" << common::ArrayToString(leaf_value_, num_leaves_) << '\n';
  s << "leaf_weight=" << common::ArrayToString(leaf_weight_, num_leaves_) << '\n';
  s << "leaf_count=" << common::ArrayToStringFast(leaf_count_, num_leaves_) << '\n';
  s << "internal_value=" << common::ArrayToStringFast(internal_value_, ni) << '\n';
  s << "internal_weight=" << common::ArrayToStringFast(internal_weight_, ni) << '\n';
  s << "internal_count=" << common::ArrayToStringFast(internal_count_, ni) << '\n';
  if (num_cat_ > 0) {
    s << "cat_boundaries=" << common::ArrayToStringFast(cat_boundaries_, num_cat_ + 1) << '\n';
    s << "cat_threshold=" << common::ArrayToStringFast(cat_threshold_, cat_threshold_.size()) << '\n';
  }
  s << "shrinkage=" << shrinkage_ << '\n';
  s << '\n';
  return s.str();
}

namespace {
template <typename T>
std::vector<T> ParseFast(const std::string& s, int n) {
  std::vector<T> out;
  out.reserve(n);
  const char* p = s.c_str();
  for (int i = 0; i < n; ++i) {
    while (*p == ' ') ++p;
    if (*p == '\0') break;
    if constexpr (std::is_floating_point<T>::value) {
      double v;
      p = common::Atof(p, &v);
      out.push_back(static_cast<T>(v));
    } else {
      long long v;
      p = common::Atoi(p, &v);
      out.push_back(static_cast<T>(v));
    }
  }
  if (static_cast<int>(out.size()) != n) Log::Fatal("Model format error: expected %d values, got %d", n, static_cast<int>(out.size()));
  return out;
}

std::vector<double> ParsePrecise(const std::string& s, int n) {
  auto toks = common::Split(s.c_str(), ' ');
  if (static_cast<int>(toks.size()) != n) Log::Fatal("Model format error: expected %d values, got %d", n, static_cast<int>(toks.size()));
  std::vector<double> out(n);
  for (int i = 0; i < n; ++i) out[i] = common::ParseDoublePrecise(toks[i]);
  return out;
}
}  // namespace

Tree::Tree(const char* str, size_t* used_len) {
  const char* p = str;
  std::unordered_map<std::string, std::string> kv;
  for (int line = 0; line < 17; ++line) {
    if (*p == '\r' || *p == '\n' || *p == '\0') break;
    const char* b = p;
    while (*p != '=' && *p != '\0') ++p;
    std::string key(b, p - b);
    if (*p == '=') ++p;
    b = p;
    while (*p != '\r' && *p != '\n' && *p != '\0') ++p;
    kv[key] = std::string(b, p - b);
    if (*p == '\r') ++p;
    if (*p == '\n') ++p;
  }
  *used_len = static_cast<size_t>(p - str);
  if (!kv.count("num_leaves")) Log::Fatal("Tree model should contain num_leaves field");
  common::Atoi(kv["num_leaves"].c_str(), &num_leaves_);
  max_leaves_ = num_leaves_;
  if (!kv.count("num_cat")) Log::Fatal("Tree model should contain num_cat field");
  common::Atoi(kv["num_cat"].c_str(), &num_cat_);
  if (!kv.count("leaf_value")) Log::Fatal("Tree model string format error, should contain leaf_value field");
  leaf_value_ = ParsePrecise(kv["leaf_value"], num_leaves_);
  shrinkage_ = 1.0;
  if (kv.count("shrinkage")) common::Atof(kv["shrinkage"].c_str(), &shrinkage_);
  cat_boundaries_.assign(1, 0);
  cat_boundaries_inner_.assign(1, 0);
  leaf_depth_.clear();
  if (num_leaves_ <= 1) {
    leaf_weight_.assign(1, 0.0);
    leaf_count_.assign(1, 0);
    leaf_parent_.assign(1, -1);
    return;
  }
  const int ni = num_leaves_ - 1;
  auto need = [&](const char* k) {
    if (!kv.count(k)) Log::Fatal("Tree model string format error, should contain %s field", k);
    return kv[k];
  };
  left_child_ = ParseFast<int>(need("left_child"), ni);
  right_child_ = ParseFast<int>(need("right_child"), ni);
  split_feature_ = ParseFast<int>(need("split_feature"), ni);
  split_feature_inner_ = split_feature_;
  threshold_ = ParsePrecise(need("threshold"), ni);
  threshold_in_bin_.assign(ni, 0);
  split_gain_ = kv.count("split_gain") ? ParseFast<float>(kv["split_gain"], ni) : std::vector<float>(ni, 0.0f);
  internal_count_ = kv.count("internal_count") ? ParseFast<int>(kv["internal_count"], ni) : std::vector<int>(ni, 0);
  internal_value_ = kv.count("internal_value") ? ParseFast<double>(kv["internal_value"], ni) : std::vector<double>(ni, 0.0);
  internal_weight_ =
      kv.count("internal_weight") ? ParseFast<double>(kv["internal_weight"], ni) : std::vector<double>(ni, 0.0);
  leaf_weight_ = kv.count("leaf_weight") ? ParsePrecise(kv["leaf_weight"], num_leaves_) : std::vector<double>(num_leaves_, 0.0);
  leaf_count_ = kv.count("leaf_count") ? ParseFast<int>(kv["leaf_count"], num_leaves_) : std::vector<int>(num_leaves_, 0);
  if (kv.count("decision_type")) {
    auto d = ParseFast<int>(kv["decision_type"], ni);
    decision_type_.assign(d.begin(), d.end());
  } else {
    decision_type_.assign(ni, 0);
  }
  if (num_cat_ > 0) {
    cat_boundaries_ = ParseFast<int>(need("cat_boundaries"), num_cat_ + 1);
    cat_threshold_ = ParseFast<uint32_t>(need("cat_threshold"), cat_boundaries_.back());
  }
  leaf_parent_.assign(num_leaves_, -1);
  for (int i = 0; i < ni; ++i) {
    if (left_child_[i] < 0) leaf_parent_[~left_child_[i]] = i;
    if (right_child_[i] < 0) leaf_parent_[~right_child_[i]] = i;
  }
  RecomputeLeafDepths(0, 0);
  max_depth_ = -1;
}

std::string Tree::ToJSON() const {
  std::stringstream s;
  s << std::setprecision(std::numeric_limits<double>::digits10 + 2);
  s << "\"num_leaves\":" << num_leaves_ << "," << '\n';
  s << "\"num_cat\":" << num_cat_ << "," << '\n';
  s << "\"shrinkage\":" << shrinkage_ << "," << '\n';
  if (num_leaves_ == 1) {
    s << "\"tree_structure\":{" << "\"leaf_value\":" << leaf_value_[0] << "}" << '\n';
  } else {
    s << "\"tree_structure\":" << NodeToJSON(0) << '\n';
  }
  return s.str();
}

std::string Tree::NodeToJSON(int index) const {
  std::stringstream s;
  s << std::setprecision(std::numeric_limits<double>::digits10 + 2);
  if (index >= 0) {
    s << "{" << '\n';
    s << "\"split_index\":" << index << "," << '\n';
    s << "\"split_feature\":" << split_feature_[index] << "," << '\n';
    s << "\"split_gain\":" << common::AvoidInf(split_gain_[index]) << "," << '\n';
    if (decision_type_[index] & kCategoricalMask) {
      const int ci = static_cast<int>(threshold_[index]);
      std::vector<int> cats;
      for (int i = cat_boundaries_[ci]; i < cat_boundaries_[ci + 1]; ++i) {
        for (int j = 0; j < 32; ++j) {
          int cat = (i - cat_boundaries_[ci]) * 32 + j;
          if (common::FindInBitset(cat_threshold_.data() + cat_boundaries_[ci], cat_boundaries_[ci + 1] - cat_boundaries_[ci], cat)) {
            cats.push_back(cat);
          }
        }
      }
      s << "\"threshold\":\"" << common::Join(cats, "||") << "\"," << '\n';
      s << "\"decision_type\":\"==\"," << '\n';
    } else {
      s << "\"threshold\":" << common::AvoidInf(threshold_[index]) << "," << '\n';
      s << "\"decision_type\":\"<=\"," << '\n';
    }
    s << "\"default_left\":" << ((decision_type_[index] & kDefaultLeftMask) ? "true" : "false") << "," << '\n';
    const int8_t mt = GetMissingType(decision_type_[index]);
    s << "\"missing_type\":\"" << (mt == 0 ? "None" : (mt == 1 ? "Zero" : "NaN")) << "\"," << '\n';
    s << "\"internal_value\":" << internal_value_[index] << "," << '\n';
    s << "\"internal_weight\":" << internal_weight_[index] << "," << '\n';
    s << "\"internal_count\":" << internal_count_[index] << "," << '\n';
    s << "\"left_child\":" << NodeToJSON(left_child_[index]) << "," << '\n';
    s << "\"right_child\":" << NodeToJSON(right_child_[index]) << '\n';
    s << "}";
  } else {
    const int leaf = ~index;
    s << "{" << '\n';
    s << "\"leaf_index\":" << leaf << "," << '\n';
    s << "\"leaf_value\":" << leaf_value_[leaf] << "," << '\n';
    s << "\"leaf_weight\":" << leaf_weight_[leaf] << "," << '\n';
    s << "\"leaf_count\":" << leaf_count_[leaf] << '\n';
    s << "}";
  }
  return s.str();
}

std::string Tree::NumericalDecisionIfElse(int node) const {
  std::stringstream s;
  s << std::setprecision(std::numeric_limits<double>::digits10 + 2);
  const int8_t mt = GetMissingType(decision_type_[node]);
  const bool dl = decision_type_[node] & kDefaultLeftMask;
  if (mt == 0 || (mt == 1 && dl && kZeroThreshold < threshold_[node])) {
    s << "if (fval <= " << threshold_[node] << ") {";
  } else if (mt == 1) {
    if (dl) s << "if (fval <= " << threshold_[node] << " || Tree::IsZero(fval)" << " || std::isnan(fval)) {";
    else s << "if (fval <= " << threshold_[node] << " && !Tree::IsZero(fval)" << " && !std::isnan(fval)) {";
  } else {
    if (dl) s << "if (fval <= " << threshold_[node] << " || std::isnan(fval)) {";
    else s << "if (fval <= " << threshold_[node] << " && !std::isnan(fval)) {";
  }
  return s.str();
}

std::string Tree::CategoricalDecisionIfElse(int node) const {
  const int8_t mt = GetMissingType(decision_type_[node]);
  std::stringstream s;
  if (mt == 2) s << "if (std::isnan(fval)) { int_fval = -1; } else { int_fval = static_cast<int>(fval); }";
  else s << "if (std::isnan(fval)) { int_fval = 0; } else { int_fval = static_cast<int>(fval); }";
  const int ci = static_cast<int>(threshold_[node]);
  s << "if (int_fval >= 0 && int_fval < 32 * (" << cat_boundaries_[ci + 1] - cat_boundaries_[ci]
    << ") && (((cat_threshold[" << cat_boundaries_[ci] << " + int_fval / 32] >> (int_fval & 31)) & 1))) {";
  return s.str();
}

std::string Tree::NodeToIfElse(int index, bool leaf_idx) const {
  std::stringstream s;
  s << std::setprecision(std::numeric_limits<double>::digits10 + 2);
  if (index >= 0) {
    s << "fval = arr[" << split_feature_[index] << "];";
    s << ((decision_type_[index] & kCategoricalMask) ? CategoricalDecisionIfElse(index) : NumericalDecisionIfElse(index));
    s << NodeToIfElse(left_child_[index], leaf_idx) << " } else { " << NodeToIfElse(right_child_[index], leaf_idx) << " }";
  } else {
    s << "return ";
    if (leaf_idx) s << ~index;
    else s << leaf_value_[~index];
    s << ";";
  }
  return s.str();
}

std::string Tree::NodeToIfElseByMap(int index, bool leaf_idx) const {
  std::stringstream s;
  s << std::setprecision(std::numeric_limits<double>::digits10 + 2);
  if (index >= 0) {
    s << "fval = arr.count(" << split_feature_[index] << ") > 0 ? arr.at(" << split_feature_[index] << ") : 0.0f;";
    s << ((decision_type_[index] & kCategoricalMask) ? CategoricalDecisionIfElse(index) : NumericalDecisionIfElse(index));
    s << NodeToIfElseByMap(left_child_[index], leaf_idx) << " } else { "
      << NodeToIfElseByMap(right_child_[index], leaf_idx) << " }";
  } else {
    s << "return ";
    if (leaf_idx) s << ~index;
    else s << leaf_value_[~index];
    s << ";";
  }
  return s.str();
}

std::string Tree::ToIfElse(int index, bool leaf_idx) const {
  std::stringstream s;
  s << std::setprecision(std::numeric_limits<double>::digits10 + 2);
  auto body = [&](bool by_map) {
    if (num_leaves_ <= 1) {
      s << "return " << leaf_value_[0] << ";";
      return;
    }
    s << "const std::vector<uint32_t> cat_threshold = {";
    for (size_t i = 0; i < cat_threshold_.size(); ++i) s << (i ? "," : "") << cat_threshold_[i];
    s << "};";
    s << "double fval = 0.0f; ";
    if (num_cat_ > 0) s << "int int_fval = 0; ";
    s << (by_map ? NodeToIfElseByMap(0, leaf_idx) : NodeToIfElse(0, leaf_idx));
  };
  s << "double PredictTree" << index << (leaf_idx ? "Leaf" : "") << "(const double* arr) { ";
  body(false);
  s << " }" << '\n';
  s << "double PredictTree" << index << (leaf_idx ? "LeafByMap" : "ByMap")
    << "(const std::unordered_map<int, double>& arr) { ";
  body(true);
  s << " }" << '\n';
  return s.str();
}

}  // namespace lgbm_amd
