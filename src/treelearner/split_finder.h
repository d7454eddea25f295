// Host (CPU) best-threshold search over one feature histogram.  This is the exact,
// sequential formulation of reference src/treelearner/feature_histogram.hpp:85-1049
// (forward/reverse scans with missing-value routing, count estimation from hessians,
// extra_trees random thresholds, categorical one-hot and sorted-ratio scans); the HIP
// split-scan kernel (src/device/split_kernels.hip) evaluates the same candidates in
// parallel and is differential-tested against this code.
#pragma once

#include <vector>

#include "lgbm_amd/bin.h"
#include "lgbm_amd/config.h"
#include "lgbm_amd/random.h"
#include "lgbm_amd/split_info.h"
#include "lgbm_amd/split_math.h"

namespace lgbm_amd {

struct FeatureMeta {
  int num_bin = 0;
  MissingType missing_type = MissingType::None;
  int8_t offset = 0;  // 1 when the most frequent bin is 0 (bin 0 not stored)
  uint32_t default_bin = 0;
  int8_t monotone_type = 0;
  double penalty = 1.0;
  BinType bin_type = BinType::Numerical;
  mutable Random rand;
};

SplitParams MakeSplitParams(const Config& cfg);

// hist: (num_bin - offset) pairs (grad, hess) in double
void FindBestThreshold(const FeatureMeta& meta, const SplitParams& p, bool extra_trees, const hist_t* hist,
                       double sum_gradient, double sum_hessian, data_size_t num_data, ConstraintRange c,
                       double parent_output, SplitInfo* out, bool* is_splittable);

// gather the split info for a given threshold (forced splits)
void GatherInfoForThreshold(const FeatureMeta& meta, const SplitParams& p, const hist_t* hist, double sum_gradient,
                            double sum_hessian, uint32_t threshold, data_size_t num_data, double parent_output,
                            SplitInfo* out);

}  // namespace lgbm_amd
