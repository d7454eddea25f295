// Validation metrics on device-resident scores (reference src/metric/regression_metric.hpp,
// binary_metric.hpp: point-wise losses and AUC with tied scores sharing half credit).
//
// Point-wise losses: per-workgroup double partial sums, then a fixed-order final sum (the
// result does not depend on scheduling).  AUC: the scores are radix-sorted descending
// (hipCUB), runs of equal scores are reduced to (positive, negative) weight pairs, and
//   accum = sum over runs of neg_run * (positives before the run + 0.5 * pos_run),
// which is the reference's sequential tie-aware sweep (binary_metric.hpp:194-262).
#include <hipcub/hipcub.hpp>

#include "device_common.h"

namespace lgbm_amd {
namespace dev {

namespace {

constexpr int kMetricThreads = 256;
constexpr int kMetricBlocks = 1024;
constexpr double kEps = 1e-15f;  // kEpsilon

__device__ __forceinline__ double ConvertScore(const MetricArgs& m, double s) {
  if (m.convert == 1) return 1.0f / (1.0f + exp(-m.sigmoid * s));
  if (m.convert == 2) return (s > 0.0 ? 1.0 : (s < 0.0 ? -1.0 : 0.0)) * s * s;
  return s;
}

__device__ __forceinline__ double PointLoss(int kind, double y, double p) {
  switch (kind) {
    case kMetricL2:
    case kMetricRMSE:
      return (p - y) * (p - y);
    case kMetricL1:
      return fabs(p - y);
    case kMetricBinLogloss:
      if (y <= 0) return 1.0f - p > kEps ? -log(1.0f - p) : -log(kEps);
      return p > kEps ? -log(p) : -log(kEps);
    case kMetricBinError:
      return p <= 0.5f ? (y > 0 ? 1.0 : 0.0) : (y <= 0 ? 1.0 : 0.0);
    default:
      return 0.0;
  }
}

__global__ __launch_bounds__(kMetricThreads) void k_point_loss(MetricArgs m, double* partials) {
  __shared__ double sh[kMetricThreads / kWave];
  double acc = 0.0;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(kMetricThreads) + threadIdx.x; i < m.n;
       i += static_cast<int64_t>(gridDim.x) * kMetricThreads) {
    const double l = PointLoss(m.kind, m.label[i], ConvertScore(m, m.score[i]));
    acc += m.weights ? l * m.weights[i] : l;
  }
  acc = BlockSum(acc, sh);
  if (threadIdx.x == 0) partials[blockIdx.x] = acc;
}

// one workgroup: fixed-order sum of `n` partials into out[slot]
__global__ __launch_bounds__(kMetricThreads) void k_sum_partials(const double* partials, int n, double* out, int slot) {
  __shared__ double sh[kMetricThreads / kWave];
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += kMetricThreads) acc += partials[i];
  acc = BlockSum(acc, sh);
  if (threadIdx.x == 0) out[slot] = acc;
}

__global__ __launch_bounds__(kMetricThreads) void k_auc_keys(MetricArgs m, double* keys, int32_t* idx) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(kMetricThreads) + threadIdx.x; i < m.n;
       i += static_cast<int64_t>(gridDim.x) * kMetricThreads) {
    keys[i] = m.score[i];
    idx[i] = static_cast<int32_t>(i);
  }
}

struct PosNeg {
  double pos, neg;
};
struct PosNegSum {
  __device__ __forceinline__ PosNeg operator()(const PosNeg& a, const PosNeg& b) const {
    return PosNeg{a.pos + b.pos, a.neg + b.neg};
  }
};

__global__ __launch_bounds__(kMetricThreads) void k_auc_weights(MetricArgs m, const int32_t* idx, PosNeg* pn) {
  for (int64_t k = blockIdx.x * static_cast<int64_t>(kMetricThreads) + threadIdx.x; k < m.n;
       k += static_cast<int64_t>(gridDim.x) * kMetricThreads) {
    const int32_t i = idx[k];
    const double w = m.weights ? m.weights[i] : 1.0;
    const bool pos = m.label[i] > 0;
    pn[k] = PosNeg{pos ? w : 0.0, pos ? 0.0 : w};
  }
}

__global__ __launch_bounds__(kMetricThreads) void k_auc_pos(const PosNeg* agg, const int* num_runs, double* pos) {
  const int n = *num_runs;
  for (int g = blockIdx.x * kMetricThreads + threadIdx.x; g < n; g += gridDim.x * kMetricThreads) pos[g] = agg[g].pos;
}

// accum partials: neg_run * (positives before the run + 0.5 * pos_run); the last workgroup
// slot also records the total positive weight
__global__ __launch_bounds__(kMetricThreads) void k_auc_accum(const PosNeg* agg, const double* pos_before,
                                                              const int* num_runs, double* partials, double* out) {
  __shared__ double sh[kMetricThreads / kWave];
  const int n = *num_runs;
  double acc = 0.0;
  for (int g = blockIdx.x * kMetricThreads + threadIdx.x; g < n; g += gridDim.x * kMetricThreads) {
    acc += agg[g].neg * (agg[g].pos * 0.5f + pos_before[g]);
  }
  acc = BlockSum(acc, sh);
  if (threadIdx.x == 0) partials[blockIdx.x] = acc;
  if (blockIdx.x == 0 && threadIdx.x == 0) out[1] = n > 0 ? pos_before[n - 1] + agg[n - 1].pos : 0.0;
}

template <typename T>
T* Carve(char** p, size_t count) {
  const size_t a = 256;
  char* q = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(*p) + a - 1) / a * a);
  *p = q + count * sizeof(T);
  return reinterpret_cast<T*>(q);
}

size_t CubTempBytes(int64_t n) {
  const int nn = static_cast<int>(n);
  size_t a = 0, b = 0, c = 0;
  (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, a, static_cast<double*>(nullptr),
                                                     static_cast<double*>(nullptr), static_cast<int32_t*>(nullptr),
                                                     static_cast<int32_t*>(nullptr), nn);
  (void)hipcub::DeviceReduce::ReduceByKey(nullptr, b, static_cast<double*>(nullptr), static_cast<double*>(nullptr),
                                          static_cast<PosNeg*>(nullptr), static_cast<PosNeg*>(nullptr),
                                          static_cast<int*>(nullptr), PosNegSum(), nn);
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, c, static_cast<double*>(nullptr), static_cast<double*>(nullptr),
                                         nn);
  return std::max(a, std::max(b, c));
}

}  // namespace

size_t MetricScratchBytes(int64_t n) {
  const size_t un = static_cast<size_t>(std::max<int64_t>(1, n));
  return 16 * 256 + sizeof(double) * kMetricBlocks + un * (4 * sizeof(double) + 2 * sizeof(int32_t)) +
         2 * un * sizeof(PosNeg) + 2 * un * sizeof(double) + sizeof(int) + CubTempBytes(n);
}

void EvalMetric(const MetricArgs& m, hipStream_t s) {
  char* p = static_cast<char*>(m.scratch);
  double* partials = Carve<double>(&p, kMetricBlocks);
  const int blocks = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>((m.n + kMetricThreads - 1) / kMetricThreads,
                                                                             kMetricBlocks)));
  if (m.kind != kMetricAUC) {
    hipLaunchKernelGGL(k_point_loss, dim3(blocks), dim3(kMetricThreads), 0, s, m, partials);
    hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(kMetricThreads), 0, s, partials, blocks, m.out, 0);
    return;
  }
  const size_t un = static_cast<size_t>(std::max<int64_t>(1, m.n));
  double* keys = Carve<double>(&p, un);
  double* keys_sorted = Carve<double>(&p, un);
  int32_t* idx = Carve<int32_t>(&p, un);
  int32_t* idx_sorted = Carve<int32_t>(&p, un);
  PosNeg* pn = Carve<PosNeg>(&p, un);
  PosNeg* agg = Carve<PosNeg>(&p, un);
  double* uniq = Carve<double>(&p, un);
  double* runpos = Carve<double>(&p, un);
  double* pos_before = Carve<double>(&p, un);
  int* num_runs = Carve<int>(&p, 1);
  size_t temp_bytes = CubTempBytes(m.n);
  void* temp = Carve<char>(&p, temp_bytes);
  const int nn = static_cast<int>(m.n);
  hipLaunchKernelGGL(k_auc_keys, dim3(blocks), dim3(kMetricThreads), 0, s, m, keys, idx);
  (void)hipcub::DeviceRadixSort::SortPairsDescending(temp, temp_bytes, keys, keys_sorted, idx, idx_sorted, nn, 0,
                                                     sizeof(double) * 8, s);
  hipLaunchKernelGGL(k_auc_weights, dim3(blocks), dim3(kMetricThreads), 0, s, m, idx_sorted, pn);
  temp_bytes = CubTempBytes(m.n);
  (void)hipcub::DeviceReduce::ReduceByKey(temp, temp_bytes, keys_sorted, uniq, pn, agg, num_runs, PosNegSum(), nn, s);
  hipLaunchKernelGGL(k_auc_pos, dim3(blocks), dim3(kMetricThreads), 0, s, agg, num_runs, runpos);
  temp_bytes = CubTempBytes(m.n);
  // runs beyond num_runs hold stale values; the exclusive sum of the first num_runs is all that is read
  (void)hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, runpos, pos_before, nn, s);
  hipLaunchKernelGGL(k_auc_accum, dim3(blocks), dim3(kMetricThreads), 0, s, agg, pos_before, num_runs, partials, m.out);
  hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(kMetricThreads), 0, s, partials, blocks, m.out, 0);
}

}  // namespace dev
}  // namespace lgbm_amd
