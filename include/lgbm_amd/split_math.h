// Leaf-output / split-gain formulas shared by the CPU split finder and the HIP
// split-scan kernels (compiled as __host__ __device__ under hipcc).
// Formulas and the kEpsilon placements are those of reference
// src/treelearner/feature_histogram.hpp:734-851 (L1 soft-thresholding, max_delta_step
// clipping, path smoothing towards the parent output, monotone-constraint clamping).
// The reference selects template instantiations from config flags; here the same flags
// are runtime values (uniform across a wave on device).
#pragma once

#include <cmath>

#include "lgbm_amd/meta.h"

namespace lgbm_amd {

struct SplitParams {
  double lambda_l1 = 0;
  double lambda_l2 = 0;
  double max_delta_step = 0;
  double path_smooth = 0;
  double min_gain_to_split = 0;
  double min_sum_hessian_in_leaf = 1e-3;
  int min_data_in_leaf = 20;
  double cat_l2 = 10;
  double cat_smooth = 10;
  int max_cat_threshold = 32;
  int min_data_per_group = 100;
  int max_cat_to_onehot = 4;
  int use_l1 = 0;
  int use_max_output = 0;
  int use_smoothing = 0;
  int use_mc = 0;
};

struct ConstraintRange {
  double min = -INFINITY;
  double max = INFINITY;
};

LGBM_HD double SignD(double x) { return (x > 0.0) - (x < 0.0); }

LGBM_HD double ThresholdL1(double s, double l1) {
  const double reg = fmax(0.0, fabs(s) - l1);
  return SignD(s) * reg;
}

// CalculateSplittedLeafOutput<USE_L1, USE_MAX_OUTPUT, USE_SMOOTHING>
LGBM_HD double LeafOutputRaw(double sg, double sh, double l1, double l2, double max_delta_step, double smoothing,
                             data_size_t num_data, double parent_output, int use_l1, int use_max_output,
                             int use_smoothing) {
  double r = use_l1 ? -ThresholdL1(sg, l1) / (sh + l2) : -sg / (sh + l2);
  if (use_max_output && max_delta_step > 0 && fabs(r) > max_delta_step) r = SignD(r) * max_delta_step;
  if (use_smoothing) {
    const double n = num_data / smoothing;
    r = r * n / (n + 1) + parent_output / (n + 1);
  }
  return r;
}

LGBM_HD double LeafOutputConstrained(double sg, double sh, double l2, const SplitParams& p, ConstraintRange c,
                                     data_size_t num_data, double parent_output) {
  double r = LeafOutputRaw(sg, sh, p.lambda_l1, l2, p.max_delta_step, p.path_smooth, num_data, parent_output,
                           p.use_l1, p.use_max_output, p.use_smoothing);
  if (p.use_mc) {
    if (r < c.min) r = c.min;
    else if (r > c.max) r = c.max;
  }
  return r;
}

LGBM_HD double LeafGainGivenOutput(double sg, double sh, double l1, double l2, double output, int use_l1) {
  const double g = use_l1 ? ThresholdL1(sg, l1) : sg;
  return -(2.0 * g * output + (sh + l2) * output * output);
}

// GetLeafGain<USE_L1, USE_MAX_OUTPUT, USE_SMOOTHING>
LGBM_HD double LeafGain(double sg, double sh, double l1, double l2, double max_delta_step, double smoothing,
                        data_size_t num_data, double parent_output, int use_l1, int use_max_output,
                        int use_smoothing) {
  if (!use_max_output && !use_smoothing) {
    const double g = use_l1 ? ThresholdL1(sg, l1) : sg;
    return (g * g) / (sh + l2);
  }
  const double out = LeafOutputRaw(sg, sh, l1, l2, max_delta_step, smoothing, num_data, parent_output, use_l1,
                                   use_max_output, use_smoothing);
  return LeafGainGivenOutput(sg, sh, l1, l2, out, use_l1);
}

// GetSplitGains<USE_MC, USE_L1, USE_MAX_OUTPUT, USE_SMOOTHING>
LGBM_HD double SplitGain(double lg, double lh, double rg, double rh, double l2, const SplitParams& p,
                         ConstraintRange c, int8_t monotone, data_size_t lcnt, data_size_t rcnt,
                         double parent_output) {
  if (!p.use_mc) {
    return LeafGain(lg, lh, p.lambda_l1, l2, p.max_delta_step, p.path_smooth, lcnt, parent_output, p.use_l1,
                    p.use_max_output, p.use_smoothing) +
           LeafGain(rg, rh, p.lambda_l1, l2, p.max_delta_step, p.path_smooth, rcnt, parent_output, p.use_l1,
                    p.use_max_output, p.use_smoothing);
  }
  const double lo = LeafOutputConstrained(lg, lh, l2, p, c, lcnt, parent_output);
  const double ro = LeafOutputConstrained(rg, rh, l2, p, c, rcnt, parent_output);
  if ((monotone > 0 && lo > ro) || (monotone < 0 && lo < ro)) return 0;
  return LeafGainGivenOutput(lg, lh, p.lambda_l1, l2, lo, p.use_l1) +
         LeafGainGivenOutput(rg, rh, p.lambda_l1, l2, ro, p.use_l1);
}

}  // namespace lgbm_amd
