// Best-split record for one leaf.  Ordering (higher gain wins; equal gain -> smaller
// real feature index; -1 features last) matches reference
// src/treelearner/split_info.hpp:126-153.  `DeviceSplit` is the fixed-size POD that
// HIP kernels and collectives exchange (the reference serialises SplitInfo into a
// byte buffer for its argmax allreduce, split_info.hpp:51-98).
#pragma once

#include <cstdint>
#include <cstring>
#include <vector>

#include "lgbm_amd/meta.h"

namespace lgbm_amd {

constexpr int kMaxCatWords = 128;  // categorical bitset capacity: 4096 bins

struct DeviceSplit {
  double gain;
  double left_sum_gradient;
  double left_sum_hessian;
  double right_sum_gradient;
  double right_sum_hessian;
  double left_output;
  double right_output;
  int32_t feature;      // inner feature index (-1: none)
  int32_t real_feature;  // real feature index (tie-breaking)
  int32_t threshold;
  int32_t left_count;
  int32_t right_count;
  int8_t default_left;
  int8_t monotone_type;
  int8_t is_categorical;
  int8_t pad0;
  int32_t num_cat_threshold;  // number of categories on the left
  uint32_t cat_bits[kMaxCatWords];
};

struct SplitInfo {
  int feature = -1;  // real feature index
  int inner_feature = -1;
  uint32_t threshold = 0;
  data_size_t left_count = 0;
  data_size_t right_count = 0;
  int num_cat_threshold = 0;
  double left_output = 0.0;
  double right_output = 0.0;
  double gain = kMinScore;
  double left_sum_gradient = 0;
  double left_sum_hessian = 0;
  double right_sum_gradient = 0;
  double right_sum_hessian = 0;
  std::vector<uint32_t> cat_threshold;
  bool default_left = true;
  int8_t monotone_type = 0;

  void Reset() {
    feature = -1;
    inner_feature = -1;
    gain = kMinScore;
  }

  bool operator>(const SplitInfo& o) const {
    double a = gain, b = o.gain;
    if (a != a) a = kMinScore;
    if (b != b) b = kMinScore;
    int fa = feature == -1 ? INT32_MAX : feature;
    int fb = o.feature == -1 ? INT32_MAX : o.feature;
    if (a != b) return a > b;
    return fa < fb;
  }

  void FromDevice(const DeviceSplit& d) {
    gain = d.gain;
    inner_feature = d.feature;
    feature = d.feature < 0 ? -1 : d.real_feature;
    threshold = static_cast<uint32_t>(d.threshold);
    left_count = d.left_count;
    right_count = d.right_count;
    left_output = d.left_output;
    right_output = d.right_output;
    left_sum_gradient = d.left_sum_gradient;
    left_sum_hessian = d.left_sum_hessian;
    right_sum_gradient = d.right_sum_gradient;
    right_sum_hessian = d.right_sum_hessian;
    default_left = d.default_left != 0;
    monotone_type = d.monotone_type;
    cat_threshold.clear();
    num_cat_threshold = 0;
    if (d.is_categorical) {
      for (int w = 0; w < kMaxCatWords; ++w) {
        for (int b = 0; b < 32; ++b) {
          if ((d.cat_bits[w] >> b) & 1u) cat_threshold.push_back(static_cast<uint32_t>(w * 32 + b));
        }
      }
      num_cat_threshold = static_cast<int>(cat_threshold.size());
    }
  }

  void ToDevice(DeviceSplit* d, bool is_cat) const {
    std::memset(d, 0, sizeof(*d));
    d->gain = gain;
    d->feature = inner_feature;
    d->real_feature = feature;
    d->threshold = static_cast<int32_t>(threshold);
    d->left_count = left_count;
    d->right_count = right_count;
    d->left_output = left_output;
    d->right_output = right_output;
    d->left_sum_gradient = left_sum_gradient;
    d->left_sum_hessian = left_sum_hessian;
    d->right_sum_gradient = right_sum_gradient;
    d->right_sum_hessian = right_sum_hessian;
    d->default_left = default_left ? 1 : 0;
    d->monotone_type = monotone_type;
    d->is_categorical = is_cat ? 1 : 0;
    d->num_cat_threshold = num_cat_threshold;
    for (uint32_t t : cat_threshold) {
      if (t < 32u * kMaxCatWords) d->cat_bits[t / 32] |= (1u << (t % 32));
    }
  }
};

// light record for voting-parallel top-k exchange (reference split_info.hpp:185-280)
struct LightSplitInfo {
  int feature = -1;
  double gain = kMinScore;
  data_size_t left_count = 0;
  data_size_t right_count = 0;
  bool operator>(const LightSplitInfo& o) const {
    double a = gain, b = o.gain;
    int fa = feature == -1 ? INT32_MAX : feature;
    int fb = o.feature == -1 ? INT32_MAX : o.feature;
    if (a != b) return a > b;
    return fa < fb;
  }
};

}  // namespace lgbm_amd
