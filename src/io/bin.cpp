// BinMapper implementation.  Algorithmic parity with reference src/io/bin.cpp:54-521:
//   * distinct values are collected from the sample with near-equal doubles merged
//     (keeping the larger), zeros re-inserted at the sign change;
//   * numerical bins: negative and positive halves are binned separately around a
//     dedicated zero bin ([-kZeroThreshold, kZeroThreshold]), each half by the greedy
//     equal-frequency rule that isolates values heavier than the mean bin size;
//   * NaN gets the last bin when present (missing_type NaN); zero_as_missing -> Zero;
//   * categorical: categories sorted by count, keep until 99% of mass and max_bin,
//     bin 0 reserved for NaN/negative/rare categories.
#include "lgbm_amd/bin.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <sstream>
#include <iomanip>

#include "lgbm_amd/common.h"
#include "lgbm_amd/log.h"

namespace lgbm_amd {

namespace {

constexpr double kInf = std::numeric_limits<double>::infinity();

// true when no threshold can leave >= filter_cnt samples on both sides
bool CannotSplit(const std::vector<int>& cnt_in_bin, int total_cnt, int filter_cnt, BinType type) {
  if (type == BinType::Numerical) {
    int left = 0;
    for (size_t i = 0; i + 1 < cnt_in_bin.size(); ++i) {
      left += cnt_in_bin[i];
      if (left >= filter_cnt && total_cnt - left >= filter_cnt) return false;
    }
    return true;
  }
  if (cnt_in_bin.size() <= 2) {
    for (size_t i = 0; i + 1 < cnt_in_bin.size(); ++i) {
      int left = cnt_in_bin[i];
      if (left >= filter_cnt && total_cnt - left >= filter_cnt) return false;
    }
    return true;
  }
  return false;
}

// Greedy equal-frequency boundaries over sorted distinct values.
std::vector<double> GreedyBounds(const double* vals, const int* cnts, int n, int max_bin, size_t total_cnt,
                                 int min_data_in_bin) {
  std::vector<double> bounds;
  LGBM_CHECK_GT(max_bin, 0);
  if (n <= max_bin) {
    int acc = 0;
    for (int i = 0; i + 1 < n; ++i) {
      acc += cnts[i];
      if (acc >= min_data_in_bin) {
        double ub = common::GetDoubleUpperBound((vals[i] + vals[i + 1]) / 2.0);
        if (bounds.empty() || !common::CheckDoubleEqualOrdered(bounds.back(), ub)) {
          bounds.push_back(ub);
          acc = 0;
        }
      }
    }
    bounds.push_back(kInf);
    return bounds;
  }
  if (min_data_in_bin > 0) {
    max_bin = std::min(max_bin, static_cast<int>(total_cnt / min_data_in_bin));
    max_bin = std::max(max_bin, 1);
  }
  double mean_bin = static_cast<double>(total_cnt) / max_bin;
  int rest_bins = max_bin;
  int rest_samples = static_cast<int>(total_cnt);
  std::vector<char> heavy(n, 0);
  for (int i = 0; i < n; ++i) {
    if (cnts[i] >= mean_bin) {
      heavy[i] = 1;
      --rest_bins;
      rest_samples -= cnts[i];
    }
  }
  mean_bin = static_cast<double>(rest_samples) / rest_bins;
  std::vector<double> upper(max_bin, kInf), lower(max_bin, kInf);
  int nb = 0;
  lower[0] = vals[0];
  int acc = 0;
  for (int i = 0; i + 1 < n; ++i) {
    if (!heavy[i]) rest_samples -= cnts[i];
    acc += cnts[i];
    bool cut = heavy[i] || acc >= mean_bin || (heavy[i + 1] && acc >= std::max(1.0, mean_bin * 0.5f));
    if (cut) {
      upper[nb] = vals[i];
      ++nb;
      lower[nb] = vals[i + 1];
      if (nb >= max_bin - 1) break;
      acc = 0;
      if (!heavy[i]) {
        --rest_bins;
        mean_bin = rest_samples / static_cast<double>(rest_bins);
      }
    }
  }
  ++nb;
  for (int i = 0; i + 1 < nb; ++i) {
    double ub = common::GetDoubleUpperBound((upper[i] + lower[i + 1]) / 2.0);
    if (bounds.empty() || !common::CheckDoubleEqualOrdered(bounds.back(), ub)) bounds.push_back(ub);
  }
  bounds.push_back(kInf);
  return bounds;
}

struct ZeroSplit {
  int left_cnt_data = 0, zero_cnt = 0, right_cnt_data = 0;
  int left_cnt = 0;     // number of distinct values < -kZeroThreshold
  int right_start = -1; // first distinct value > kZeroThreshold
};

ZeroSplit AnalyzeAroundZero(const double* vals, const int* cnts, int n) {
  ZeroSplit z;
  for (int i = 0; i < n; ++i) {
    if (vals[i] <= -kZeroThreshold) z.left_cnt_data += cnts[i];
    else if (vals[i] > kZeroThreshold) z.right_cnt_data += cnts[i];
    else z.zero_cnt += cnts[i];
  }
  z.left_cnt = -1;
  for (int i = 0; i < n; ++i) {
    if (vals[i] > -kZeroThreshold) { z.left_cnt = i; break; }
  }
  if (z.left_cnt < 0) z.left_cnt = n;
  for (int i = z.left_cnt; i < n; ++i) {
    if (vals[i] > kZeroThreshold) { z.right_start = i; break; }
  }
  return z;
}

std::vector<double> BoundsWithForced(const double* vals, const int* cnts, int n, int max_bin, size_t total_cnt,
                                     int min_data_in_bin, const std::vector<double>& forced) {
  ZeroSplit z = AnalyzeAroundZero(vals, cnts, n);
  std::vector<double> bounds;
  if (max_bin == 2) {
    bounds.push_back(z.left_cnt == 0 ? kZeroThreshold : -kZeroThreshold);
  } else if (max_bin >= 3) {
    if (z.left_cnt > 0) bounds.push_back(-kZeroThreshold);
    if (z.right_start >= 0) bounds.push_back(kZeroThreshold);
  }
  bounds.push_back(kInf);
  int room = max_bin - static_cast<int>(bounds.size());
  int added = 0;
  for (double f : forced) {
    if (added >= room) break;
    if (std::fabs(f) > kZeroThreshold) { bounds.push_back(f); ++added; }
  }
  std::stable_sort(bounds.begin(), bounds.end());
  int free_bins = max_bin - static_cast<int>(bounds.size());
  std::vector<double> extra;
  int vi = 0;
  for (size_t i = 0; i < bounds.size(); ++i) {
    int cnt_in = 0, distinct_in = 0, start = vi;
    while (vi < n && vals[vi] < bounds[i]) { cnt_in += cnts[vi]; ++distinct_in; ++vi; }
    int remaining = max_bin - static_cast<int>(bounds.size()) - static_cast<int>(extra.size());
    int sub = static_cast<int>(std::lround(static_cast<double>(cnt_in) * free_bins / total_cnt));
    sub = std::min(sub, remaining) + 1;
    if (i == bounds.size() - 1) sub = remaining + 1;
    auto nb = GreedyBounds(vals + start, cnts + start, distinct_in, sub, cnt_in, min_data_in_bin);
    extra.insert(extra.end(), nb.begin(), nb.end() - 1);
  }
  bounds.insert(bounds.end(), extra.begin(), extra.end());
  std::stable_sort(bounds.begin(), bounds.end());
  LGBM_CHECK_LE(bounds.size(), static_cast<size_t>(max_bin));
  return bounds;
}

std::vector<double> BoundsZeroAsBin(const double* vals, const int* cnts, int n, int max_bin, size_t total_cnt,
                                    int min_data_in_bin) {
  ZeroSplit z = AnalyzeAroundZero(vals, cnts, n);
  std::vector<double> bounds;
  if (z.left_cnt > 0 && max_bin > 1) {
    int left_max =
        static_cast<int>(static_cast<double>(z.left_cnt_data) / (total_cnt - z.zero_cnt) * (max_bin - 1));
    left_max = std::max(1, left_max);
    bounds = GreedyBounds(vals, cnts, z.left_cnt, left_max, z.left_cnt_data, min_data_in_bin);
    if (!bounds.empty()) bounds.back() = -kZeroThreshold;
  }
  int right_max = max_bin - 1 - static_cast<int>(bounds.size());
  if (z.right_start >= 0 && right_max > 0) {
    auto rb = GreedyBounds(vals + z.right_start, cnts + z.right_start, n - z.right_start, right_max,
                           z.right_cnt_data, min_data_in_bin);
    bounds.push_back(kZeroThreshold);
    bounds.insert(bounds.end(), rb.begin(), rb.end());
  } else {
    bounds.push_back(kInf);
  }
  LGBM_CHECK_LE(bounds.size(), static_cast<size_t>(max_bin));
  return bounds;
}

std::vector<double> NumericalBounds(const double* vals, const int* cnts, int n, int max_bin, size_t total_cnt,
                                    int min_data_in_bin, const std::vector<double>& forced) {
  if (forced.empty()) return BoundsZeroAsBin(vals, cnts, n, max_bin, total_cnt, min_data_in_bin);
  return BoundsWithForced(vals, cnts, n, max_bin, total_cnt, min_data_in_bin, forced);
}

}  // namespace

BinMapper::BinMapper()
    : num_bin_(1), missing_type_(MissingType::None), is_trivial_(true), sparse_rate_(1.0),
      bin_type_(BinType::Numerical), min_val_(0), max_val_(0), default_bin_(0), most_freq_bin_(0) {
  bin_upper_bound_.push_back(kInf);
}

void BinMapper::FindBin(double* values, int num_values, size_t total_sample_cnt, int max_bin, int min_data_in_bin,
                        int min_split_data, bool pre_filter, BinType bin_type, bool use_missing,
                        bool zero_as_missing, const std::vector<double>& forced_upper_bounds) {
  // drop NaNs (counted separately)
  int kept = 0;
  for (int i = 0; i < num_values; ++i) {
    if (!std::isnan(values[i])) values[kept++] = values[i];
  }
  int na_cnt = 0;
  if (!use_missing) {
    missing_type_ = MissingType::None;
  } else if (zero_as_missing) {
    missing_type_ = MissingType::Zero;
  } else if (kept == num_values) {
    missing_type_ = MissingType::None;
  } else {
    missing_type_ = MissingType::NaN;
    na_cnt = num_values - kept;
  }
  num_values = kept;
  bin_type_ = bin_type;
  default_bin_ = 0;
  const int zero_cnt = static_cast<int>(total_sample_cnt - num_values - na_cnt);

  std::stable_sort(values, values + num_values);
  std::vector<double> distinct;
  std::vector<int> counts;
  if (num_values == 0 || (values[0] > 0.0 && zero_cnt > 0)) {
    distinct.push_back(0.0);
    counts.push_back(zero_cnt);
  }
  if (num_values > 0) {
    distinct.push_back(values[0]);
    counts.push_back(1);
  }
  for (int i = 1; i < num_values; ++i) {
    if (!common::CheckDoubleEqualOrdered(values[i - 1], values[i])) {
      if (values[i - 1] < 0.0 && values[i] > 0.0) {
        distinct.push_back(0.0);
        counts.push_back(zero_cnt);
      }
      distinct.push_back(values[i]);
      counts.push_back(1);
    } else {
      distinct.back() = values[i];  // keep the larger of near-equal values
      ++counts.back();
    }
  }
  if (num_values > 0 && values[num_values - 1] < 0.0 && zero_cnt > 0) {
    distinct.push_back(0.0);
    counts.push_back(zero_cnt);
  }
  min_val_ = distinct.front();
  max_val_ = distinct.back();
  const int nd = static_cast<int>(distinct.size());
  std::vector<int> cnt_in_bin;

  if (bin_type_ == BinType::Numerical) {
    if (missing_type_ == MissingType::Zero) {
      bin_upper_bound_ = NumericalBounds(distinct.data(), counts.data(), nd, max_bin, total_sample_cnt,
                                         min_data_in_bin, forced_upper_bounds);
      if (bin_upper_bound_.size() == 2) missing_type_ = MissingType::None;
    } else if (missing_type_ == MissingType::None) {
      bin_upper_bound_ = NumericalBounds(distinct.data(), counts.data(), nd, max_bin, total_sample_cnt,
                                         min_data_in_bin, forced_upper_bounds);
    } else {
      bin_upper_bound_ = NumericalBounds(distinct.data(), counts.data(), nd, max_bin - 1, total_sample_cnt - na_cnt,
                                         min_data_in_bin, forced_upper_bounds);
      // the reference pushes its unscoped enumerator MissingType::NaN here (bin.cpp:407), so
      // the NaN bin's (never consulted) upper bound is 2.0; keeping the value makes
      // CheckAlign (NaN != NaN) and binary dataset files agree with it
      bin_upper_bound_.push_back(static_cast<double>(MissingType::NaN));
    }
    num_bin_ = static_cast<int>(bin_upper_bound_.size());
    cnt_in_bin.assign(num_bin_, 0);
    int b = 0;
    for (int i = 0; i < nd; ++i) {
      if (distinct[i] > bin_upper_bound_[b]) ++b;
      cnt_in_bin[b] += counts[i];
    }
    if (missing_type_ == MissingType::NaN) cnt_in_bin[num_bin_ - 1] = na_cnt;
    LGBM_CHECK_LE(num_bin_, max_bin);
  } else {
    std::vector<int> cats, cat_cnts;
    for (int i = 0; i < nd; ++i) {
      int v = static_cast<int>(distinct[i]);
      if (v < 0) {
        na_cnt += counts[i];
        Log::Warning("Met negative value in categorical features, will convert it to NaN");
      } else if (cats.empty() || v != cats.back()) {
        cats.push_back(v);
        cat_cnts.push_back(counts[i]);
      } else {
        cat_cnts.back() += counts[i];
      }
    }
    int rest_cnt = static_cast<int>(total_sample_cnt - na_cnt);
    if (rest_cnt > 0) {
      const int kSparseRatio = 100;
      if (cats.back() / kSparseRatio > static_cast<int>(cats.size())) {
        Log::Warning("Met categorical feature which contains sparse values. "
                     "Consider renumbering to consecutive integers started from zero");
      }
      common::SortPairsByKey(&cat_cnts, &cats, true);
      int cut_cnt = static_cast<int>(common::RoundInt((total_sample_cnt - na_cnt) * 0.99f));
      categorical_2_bin_.clear();
      bin_2_categorical_.clear();
      int used_cnt = 0;
      int distinct_cnt = static_cast<int>(cats.size()) + (na_cnt > 0 ? 1 : 0);
      max_bin = std::min(distinct_cnt, max_bin);
      cnt_in_bin.clear();
      // bin 0 is the NaN / other bucket
      bin_2_categorical_.push_back(-1);
      categorical_2_bin_[-1] = 0;
      cnt_in_bin.push_back(0);
      num_bin_ = 1;
      size_t cur = 0;
      while (cur < cats.size() && (used_cnt < cut_cnt || num_bin_ < max_bin)) {
        if (cat_cnts[cur] < min_data_in_bin && cur > 1) break;
        bin_2_categorical_.push_back(cats[cur]);
        categorical_2_bin_[cats[cur]] = static_cast<unsigned>(num_bin_);
        used_cnt += cat_cnts[cur];
        cnt_in_bin.push_back(cat_cnts[cur]);
        ++num_bin_;
        ++cur;
      }
      missing_type_ = (cur == cats.size() && na_cnt == 0) ? MissingType::None : MissingType::NaN;
      cnt_in_bin[0] = static_cast<int>(total_sample_cnt - used_cnt);
    }
  }

  is_trivial_ = num_bin_ <= 1;
  if (!is_trivial_ && pre_filter &&
      CannotSplit(cnt_in_bin, static_cast<int>(total_sample_cnt), min_split_data, bin_type_)) {
    is_trivial_ = true;
  }
  if (!is_trivial_) {
    default_bin_ = ValueToBin(0);
    most_freq_bin_ = static_cast<uint32_t>(std::max_element(cnt_in_bin.begin(), cnt_in_bin.end()) - cnt_in_bin.begin());
    double max_sparse = static_cast<double>(cnt_in_bin[most_freq_bin_]) / total_sample_cnt;
    // a non-default most-frequent bin only pays off when it is really dominant
    if (most_freq_bin_ != default_bin_ && max_sparse < kSparseThreshold) most_freq_bin_ = default_bin_;
    sparse_rate_ = static_cast<double>(cnt_in_bin[most_freq_bin_]) / total_sample_cnt;
  } else {
    sparse_rate_ = 1.0;
  }
}

uint32_t BinMapper::ValueToBin(double value) const {
  if (std::isnan(value)) {
    if (bin_type_ == BinType::Categorical) return 0;
    if (missing_type_ == MissingType::NaN) return static_cast<uint32_t>(num_bin_ - 1);
    value = 0.0;
  }
  if (bin_type_ == BinType::Numerical) {
    int lo = 0;
    int hi = num_bin_ - 1;
    if (missing_type_ == MissingType::NaN) hi -= 1;
    while (lo < hi) {
      int mid = (lo + hi - 1) / 2;
      if (value <= bin_upper_bound_[mid]) hi = mid;
      else lo = mid + 1;
    }
    return static_cast<uint32_t>(lo);
  }
  int iv = static_cast<int>(value);
  if (iv < 0) return 0;
  auto it = categorical_2_bin_.find(iv);
  return it == categorical_2_bin_.end() ? 0u : it->second;
}

bool BinMapper::CheckAlign(const BinMapper& o) const {
  if (num_bin_ != o.num_bin_ || missing_type_ != o.missing_type_) return false;
  if (bin_type_ == BinType::Numerical) {
    for (int i = 0; i < num_bin_; ++i) {
      if (bin_upper_bound_[i] != o.bin_upper_bound_[i]) return false;
    }
  } else {
    for (int i = 0; i < num_bin_; ++i) {
      if (bin_2_categorical_[i] != o.bin_2_categorical_[i]) return false;
    }
  }
  return true;
}

std::string BinMapper::bin_info_string() const {
  if (bin_type_ == BinType::Categorical) return common::Join(bin_2_categorical_, ":");
  std::stringstream ss;
  ss << std::setprecision(std::numeric_limits<double>::digits10 + 2);
  ss << '[' << min_val_ << ':' << max_val_ << ']';
  return ss.str();
}

// layout: num_bin i32 | missing i8 | trivial u8 | sparse f64 | type i8 | min f64 | max f64 | default u32 |
//         most_freq u32 | bounds f64[num_bin] or cats i32[num_bin]
// the reference's layout (bin.cpp:562-620: enums as 4-byte ints, bool as one byte, no padding),
// shared by the distributed bin-mapper exchange and the dataset binary file
size_t BinMapper::SizesInByte() const {
  size_t s = 4 + 4 + 1 + 8 + 4 + 8 + 8 + 4 + 4;
  s += bin_type_ == BinType::Numerical ? 8 * num_bin_ : 4 * num_bin_;
  return s;
}

void BinMapper::CopyTo(char* b) const {
  auto put = [&b](const void* p, size_t n) { std::memcpy(b, p, n); b += n; };
  const int32_t mt = static_cast<int32_t>(missing_type_), bt = static_cast<int32_t>(bin_type_);
  const uint8_t tr = is_trivial_ ? 1 : 0;
  put(&num_bin_, 4); put(&mt, 4); put(&tr, 1); put(&sparse_rate_, 8); put(&bt, 4);
  put(&min_val_, 8); put(&max_val_, 8); put(&default_bin_, 4); put(&most_freq_bin_, 4);
  if (bin_type_ == BinType::Numerical) put(bin_upper_bound_.data(), 8 * num_bin_);
  else put(bin_2_categorical_.data(), 4 * num_bin_);
}

void BinMapper::CopyFrom(const char* b) {
  auto get = [&b](void* p, size_t n) { std::memcpy(p, b, n); b += n; };
  int32_t mt, bt;
  uint8_t tr;
  get(&num_bin_, 4); get(&mt, 4); get(&tr, 1); get(&sparse_rate_, 8); get(&bt, 4);
  get(&min_val_, 8); get(&max_val_, 8); get(&default_bin_, 4); get(&most_freq_bin_, 4);
  if (mt < 0 || mt > 2 || bt < 0 || bt > 1 || num_bin_ < 0) Log::Fatal("Binary file error: corrupt bin mapper");
  missing_type_ = static_cast<MissingType>(mt);
  bin_type_ = static_cast<BinType>(bt);
  is_trivial_ = tr != 0;
  if (bin_type_ == BinType::Numerical) {
    bin_upper_bound_.resize(num_bin_);
    get(bin_upper_bound_.data(), 8 * num_bin_);
    bin_2_categorical_.clear();
  } else {
    bin_2_categorical_.resize(num_bin_);
    get(bin_2_categorical_.data(), 4 * num_bin_);
    categorical_2_bin_.clear();
    for (int i = 0; i < num_bin_; ++i) categorical_2_bin_[bin_2_categorical_[i]] = static_cast<unsigned>(i);
  }
}

}  // namespace lgbm_amd
