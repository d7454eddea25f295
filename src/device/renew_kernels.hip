// Leaf-output renewal for the percentile objectives on the device (reference
// src/objective/regression_objective.hpp:18-60 PercentileFun / WeightedPercentileFun, and
// RenewTreeOutput of L1 :238, quantile, MAPE): each leaf's output becomes the alpha-percentile
// of its in-bag rows' residuals (label - score), optionally weighted.
//   k_renew_gather      the leaves' rows (from the partition) -> residual keys and weights,
//                       leaf after leaf (the partition's row order inside a leaf)
//   segmented radix sort (hipCUB, stable) of the keys by leaf, ascending
//   k_renew_percentile  one workgroup per leaf: the reference's interpolated percentile of the
//                       sorted segment (weighted: the cumulative weights in sorted order)
#include <hipcub/hipcub.hpp>

#include "device_common.h"

namespace lgbm_amd {
namespace dev {

namespace {

constexpr int kRenewThreads = 256;
constexpr int kRenewBlocksPerLeaf = 64;

template <typename T>
T* CarveR(char** p, size_t n) {
  const uintptr_t a = (reinterpret_cast<uintptr_t>(*p) + 255) & ~static_cast<uintptr_t>(255);
  T* out = reinterpret_cast<T*>(a);
  *p = reinterpret_cast<char*>(a + sizeof(T) * n);
  return out;
}

__global__ __launch_bounds__(kRenewThreads) void k_renew_gather(RenewArgs r) {
  const int l = blockIdx.y;
  const Leaf lf = r.leaves[l];
  const int32_t* rows = RowBuf(r.idx, r.tmp, r.buf_stride, lf.buf) + lf.begin;
  const int64_t out0 = r.offsets[l];
  for (int i = blockIdx.x * kRenewThreads + threadIdx.x; i < lf.count; i += gridDim.x * kRenewThreads) {
    const int row = rows[i];
    r.keys[out0 + i] = static_cast<double>(r.label[row]) - r.score[row];
    if (r.weights != nullptr) r.vals[out0 + i] = static_cast<double>(r.weights[row]);
  }
}

// one workgroup per leaf
__global__ __launch_bounds__(kRenewThreads) void k_renew_percentile(RenewArgs r, const double* keys,
                                                                    const double* vals, double* cdf) {
  __shared__ int s_pos;
  const int l = blockIdx.x;
  const int64_t b = r.offsets[l];
  const int n = static_cast<int>(r.offsets[l + 1] - b);
  const double* v = keys + b;  // ascending
  if (n <= 0) {
    if (threadIdx.x == 0) r.out[l] = 0.0;
    return;
  }
  if (n == 1) {
    if (threadIdx.x == 0) r.out[l] = v[0];
    return;
  }
  if (vals == nullptr) {
    // pos-th and (pos+1)-th largest, pos = floor((1 - alpha) * n), linear interpolation
    if (threadIdx.x != 0) return;
    const double fpos = __dmul_rn(1.0f - r.alpha, static_cast<double>(n));
    const int pos = static_cast<int>(fpos);
    double out;
    if (pos < 1) {
      out = v[n - 1];
    } else if (pos >= n) {
      out = v[0];
    } else {
      const double bias = fpos - pos;
      const double v1 = v[n - pos], v2 = v[n - pos - 1];
      // separately rounded products and sums (no fused multiply-add): the host's arithmetic
      out = __dsub_rn(v1, __dmul_rn(__dsub_rn(v1, v2), bias));
    }
    r.out[l] = out;
    return;
  }
  // weighted: cumulative weights in sorted order, summed sequentially as the reference does
  // (the threshold comparisons below see bit-identical partial sums)
  const double* w = vals + b;
  double* c = cdf + b;
  if (threadIdx.x == 0) {
    double acc = 0.0;
    for (int i = 0; i < n; ++i) {
      acc = i == 0 ? w[0] : __dadd_rn(acc, w[i]);
      c[i] = acc;
    }
  }
  __syncthreads();
  const double thr = __dmul_rn(c[n - 1], r.alpha);
  // first position whose cumulative weight exceeds thr (upper_bound)
  if (threadIdx.x == 0) s_pos = n;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += kRenewThreads) {
    if (c[i] > thr && (i == 0 || c[i - 1] <= thr)) atomicMin(&s_pos, i);
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  int pos = min(s_pos, n - 1);
  double out;
  if (pos == 0 || pos == n - 1) {
    out = v[pos];
  } else {
    const double v1 = v[pos - 1], v2 = v[pos];
    if (c[pos + 1] - c[pos] >= 1.0f) {
      out = __dadd_rn(__dmul_rn((thr - c[pos]) / (c[pos + 1] - c[pos]), __dsub_rn(v2, v1)), v1);
    } else {
      out = v2;
    }
  }
  r.out[l] = out;
}

size_t SortTempBytes(int64_t n, int leaves, bool weighted) {
  size_t bytes = 0;
  if (weighted) {
    (void)hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, bytes, static_cast<const double*>(nullptr),
                                                      static_cast<double*>(nullptr), static_cast<const double*>(nullptr),
                                                      static_cast<double*>(nullptr), static_cast<int>(n), leaves,
                                                      static_cast<const int64_t*>(nullptr),
                                                      static_cast<const int64_t*>(nullptr) + 1);
  } else {
    (void)hipcub::DeviceSegmentedRadixSort::SortKeys(nullptr, bytes, static_cast<const double*>(nullptr),
                                                     static_cast<double*>(nullptr), static_cast<int>(n), leaves,
                                                     static_cast<const int64_t*>(nullptr),
                                                     static_cast<const int64_t*>(nullptr) + 1);
  }
  return bytes;
}

}  // namespace

size_t RenewScratchBytes(int64_t n, int leaves) {
  const size_t un = static_cast<size_t>(std::max<int64_t>(1, n));
  return 8 * 256 + 5 * un * sizeof(double) + std::max(SortTempBytes(n, leaves, true), SortTempBytes(n, leaves, false));
}

void RenewLeafOutputs(RenewArgs r, int64_t n, hipStream_t s) {
  const size_t un = static_cast<size_t>(std::max<int64_t>(1, n));
  char* p = static_cast<char*>(r.scratch);
  r.keys = CarveR<double>(&p, un);
  r.vals = CarveR<double>(&p, un);
  double* keys_sorted = CarveR<double>(&p, un);
  double* vals_sorted = CarveR<double>(&p, un);
  double* cdf = CarveR<double>(&p, un);
  const bool weighted = r.weights != nullptr;
  size_t temp_bytes = SortTempBytes(n, r.num_leaves, weighted);
  void* temp = CarveR<char>(&p, temp_bytes);
  hipLaunchKernelGGL(k_renew_gather, dim3(kRenewBlocksPerLeaf, r.num_leaves), dim3(kRenewThreads), 0, s, r);
  if (n > 0) {
    if (weighted) {
      (void)hipcub::DeviceSegmentedRadixSort::SortPairs(temp, temp_bytes, r.keys, keys_sorted, r.vals, vals_sorted,
                                                        static_cast<int>(n), r.num_leaves, r.offsets, r.offsets + 1, 0,
                                                        sizeof(double) * 8, s);
    } else {
      (void)hipcub::DeviceSegmentedRadixSort::SortKeys(temp, temp_bytes, r.keys, keys_sorted, static_cast<int>(n),
                                                       r.num_leaves, r.offsets, r.offsets + 1, 0, sizeof(double) * 8,
                                                       s);
    }
  }
  hipLaunchKernelGGL(k_renew_percentile, dim3(r.num_leaves), dim3(kRenewThreads), 0, s, r, keys_sorted,
                     weighted ? vals_sorted : nullptr, cdf);
}

}  // namespace dev
}  // namespace lgbm_amd
