// Core scalar types and numeric constants shared by host and device code.
// The constants must match the reference bit-for-bit because they change split
// decisions (reference: include/LightGBM/meta.h:28-80, include/LightGBM/bin.h:32-39).
#pragma once

#include <cstdint>
#include <cstddef>
#include <limits>

#if defined(__HIPCC__)
#define LGBM_HD __host__ __device__ __forceinline__
#else
#define LGBM_HD inline
#endif

namespace lgbm_amd {

using data_size_t = int32_t;   // row index type (<= 2^31-1 rows per rank)
using score_t = float;         // gradient / hessian storage
using label_t = float;         // label / weight storage
using comm_size_t = int32_t;   // collective message sizes
using hist_t = double;         // host histogram accumulator

constexpr double kZeroThreshold = 1e-35f;
constexpr double kEpsilon = 1e-15f;
constexpr double kMinScore = -std::numeric_limits<double>::infinity();
constexpr double kMaxScore = std::numeric_limits<double>::infinity();
constexpr double kSparseThreshold = 0.7;
constexpr int kDefaultNumLeaves = 31;

enum class MissingType : int8_t { None = 0, Zero = 1, NaN = 2 };
enum class BinType : int8_t { Numerical = 0, Categorical = 1 };

// decision_type bit layout of tree nodes (reference: include/LightGBM/tree.h:19-20,235-254)
constexpr int8_t kCategoricalMask = 1;
constexpr int8_t kDefaultLeftMask = 2;

}  // namespace lgbm_amd
