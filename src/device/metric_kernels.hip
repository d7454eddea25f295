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
  if (m.convert == 3) return exp(s);
  return s;
}

__device__ __forceinline__ double SafeLog(double x) { return x > 0 ? log(x) : -INFINITY; }

// the per-row losses of src/metric/metrics.cpp (reference regression_metric.hpp,
// binary_metric.hpp, xentropy_metric.hpp), with their float-literal constants
__device__ __forceinline__ double PointLoss(const MetricArgs& m, double y, double p) {
  switch (m.kind) {
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
    case kMetricQuantile: {
      const double d = y - p;
      return d < 0 ? (m.param - 1.0f) * d : m.param * d;
    }
    case kMetricHuber: {
      const double d = p - y;
      return fabs(d) <= m.param ? 0.5f * d * d : m.param * (fabs(d) - 0.5f * m.param);
    }
    case kMetricFair: {
      const double x = fabs(p - y), c = m.param;
      return c * x - c * c * log(1.0f + x / c);
    }
    case kMetricPoisson: {
      const double e = 1e-10f;
      const double s = p < e ? e : p;
      return s - y * log(s);
    }
    case kMetricMape:
      return fabs(y - p) / fmax(1.0f, fabs(y));
    case kMetricGamma: {
      const double theta = -1.0 / p;
      const double b = -SafeLog(-theta);
      const double c = SafeLog(y) - SafeLog(y);  // 1/psi * log(y/psi) - log(y), psi = 1
      return -((y * theta - b) + c);
    }
    case kMetricGammaDeviance: {
      const double t = y / (p + 1.0e-9);
      return t - SafeLog(t) - 1;
    }
    case kMetricTweedie: {
      const double rho = m.param, e = 1e-10f;
      const double s = p < e ? e : p;
      return -y * exp((1 - rho) * log(s)) / (1 - rho) + exp((2 - rho) * log(s)) / (2 - rho);
    }
    case kMetricXent: {
      const double e = 1.0e-12;
      const double a = y * (p > e ? log(p) : log(e));
      const double b = (1.0f - y) * (1.0f - p > e ? log(1.0f - p) : log(e));
      return -(a + b);
    }
    default:
      return 0.0;
  }
}

// multiclass row loss: converted class scores (softmax / per-class sigmoid / raw), then
// -log p[label] or the top-k error (a class counts as larger when it is >= the label's)
__device__ __forceinline__ double MulticlassLoss(const MetricArgs& m, int64_t i) {
  const int K = m.num_class;
  const int y = static_cast<int>(m.label[i]);
  double mx = -INFINITY;
  if (m.convert == 4) {
    for (int k = 0; k < K; ++k) mx = fmax(mx, m.score[static_cast<int64_t>(k) * m.n + i]);
  }
  double denom = 0.0;
  if (m.convert == 4) {
    for (int k = 0; k < K; ++k) denom += exp(m.score[static_cast<int64_t>(k) * m.n + i] - mx);
  }
  auto rec = [&](int k) {
    const double s = m.score[static_cast<int64_t>(k) * m.n + i];
    if (m.convert == 4) return exp(s - mx) / denom;
    if (m.convert == 5) return 1.0f / (1.0f + exp(-m.sigmoid * s));
    return s;
  };
  const double ry = rec(y);
  if (m.kind == kMetricMultiLogloss) return ry > kEps ? -log(ry) : -log(kEps);
  int larger = 0;
  for (int k = 0; k < K; ++k) {
    if (rec(k) >= ry) ++larger;
    if (larger > m.top_k) return 1.0;
  }
  return 0.0;
}

__global__ __launch_bounds__(kMetricThreads) void k_point_loss(MetricArgs m, double* partials) {
  __shared__ double sh[kMetricThreads / kWave];
  double acc = 0.0;
  const bool multi = m.kind == kMetricMultiLogloss || m.kind == kMetricMultiError;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(kMetricThreads) + threadIdx.x; i < m.n;
       i += static_cast<int64_t>(gridDim.x) * kMetricThreads) {
    const double l = multi ? MulticlassLoss(m, i) : PointLoss(m, m.label[i], ConvertScore(m, m.score[i]));
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

struct PosNeg {
  double pos, neg;
};
struct PosNegSum {
  __device__ __forceinline__ PosNeg operator()(const PosNeg& a, const PosNeg& b) const {
    return PosNeg{a.pos + b.pos, a.neg + b.neg};
  }
};

// AUC: each row's weight with its class in the sign (negative rows -w; w = 0 either way adds
// nothing), sorted along with the scores, so the (positive, negative) pairs are read in order
// instead of gathered through a sorted row index
__global__ __launch_bounds__(kMetricThreads) void k_auc_signed(MetricArgs m, float* v) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(kMetricThreads) + threadIdx.x; i < m.n;
       i += static_cast<int64_t>(gridDim.x) * kMetricThreads) {
    const float w = m.weights ? static_cast<float>(m.weights[i]) : 1.0f;
    v[i] = m.label[i] > 0 ? w : -w;
  }
}

__global__ __launch_bounds__(kMetricThreads) void k_auc_unsign(const float* v, int64_t n, PosNeg* pn) {
  for (int64_t k = blockIdx.x * static_cast<int64_t>(kMetricThreads) + threadIdx.x; k < n;
       k += static_cast<int64_t>(gridDim.x) * kMetricThreads) {
    const float x = v[k];
    pn[k] = signbit(x) ? PosNeg{0.0, static_cast<double>(-x)} : PosNeg{static_cast<double>(x), 0.0};
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

// AUC-mu (reference multiclass_metric.hpp AucMuMetric): the pair (i, j)'s binary AUC with
// class j as positives over the keys -t1 * (v . score), v = W[i] - W[j], t1 = v[i] - v[j];
// rows of other classes weigh nothing.  Products and sums are rounded one by one (no fused
// multiply-add) as on the host.
__global__ __launch_bounds__(kMetricThreads) void k_aucmu_keys(MetricArgs m, int ci, int cj, double* keys,
                                                               int32_t* idx) {
  const int K = m.num_class;
  const double* wi = m.qconst + static_cast<int64_t>(ci) * K;
  const double* wj = m.qconst + static_cast<int64_t>(cj) * K;
  const double t1 = __dadd_rn(wi[ci] - wj[ci], -(wi[cj] - wj[cj]));
  for (int64_t r = blockIdx.x * static_cast<int64_t>(kMetricThreads) + threadIdx.x; r < m.n;
       r += static_cast<int64_t>(gridDim.x) * kMetricThreads) {
    const int lab = static_cast<int>(m.label[r]);
    double key = 0.0;
    if (lab == ci || lab == cj) {
      double va = 0.0;
      for (int k = 0; k < K; ++k) va = __dadd_rn(va, __dmul_rn(wi[k] - wj[k], m.score[static_cast<int64_t>(k) * m.n + r]));
      key = -__dmul_rn(t1, va) + 0.0;  // (+0.0: no negative zero key apart from 0.0)
    }
    keys[r] = key;
    idx[r] = static_cast<int32_t>(r);
  }
}

__global__ __launch_bounds__(kMetricThreads) void k_aucmu_weights(MetricArgs m, int ci, int cj, const int32_t* idx,
                                                                  PosNeg* pn) {
  for (int64_t k = blockIdx.x * static_cast<int64_t>(kMetricThreads) + threadIdx.x; k < m.n;
       k += static_cast<int64_t>(gridDim.x) * kMetricThreads) {
    const int lab = static_cast<int>(m.label[idx[k]]);
    pn[k] = PosNeg{lab == cj ? 1.0 : 0.0, lab == ci ? 1.0 : 0.0};
  }
}

template <typename T>
T* Carve(char** p, size_t count) {
  const size_t a = 256;
  char* q = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(*p) + a - 1) / a * a);
  *p = q + count * sizeof(T);
  return reinterpret_cast<T*>(q);
}

// ---------------------------------------------------------------- query metrics
// one workgroup per query: the documents' stable descending score order as ranks (as in
// rank_kernels.hip), then the query's NDCG@k / MAP@k for every k into partials[q][nk]
constexpr int kQueryThreads = 128;

template <int NT>
__device__ __forceinline__ double QBlockSum(double v, double* red) {
  for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  const int w = threadIdx.x / kWave;
  __syncthreads();
  if ((threadIdx.x & (kWave - 1)) == 0) red[w] = v;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < NT / kWave; ++i) t += red[i];
  return t;
}

template <int NT>
__device__ void QueryMetricBody(const MetricArgs& m, int q, double* partials, double* s_score, int* s_pos,
                                char* s_rel, int* s_label, double* red) {
  const int b = m.qb[q], cnt = m.qb[q + 1] - b;
  for (int i = threadIdx.x; i < cnt; i += NT) {
    s_score[i] = m.score[b + i];
    s_label[i] = static_cast<int>(m.label[b + i]);
    s_rel[i] = m.label[b + i] > 0.5f ? 1 : 0;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < cnt; i += NT) {
    const double si = s_score[i];
    int p = 0;
    for (int j = 0; j < cnt; ++j) p += (s_score[j] > si) || (s_score[j] == si && j < i);
    s_pos[i] = p;
  }
  __syncthreads();
  const double w = m.qw != nullptr ? m.qw[q] : 1.0;
  for (int kk = 0; kk < m.nk; ++kk) {
    const int k = min(m.eval_at[kk], cnt);
    double v = 0.0;
    if (m.kind == kMetricNDCG) {
      const double inv = m.qconst[static_cast<int64_t>(q) * m.nk + kk];
      if (m.qconst[static_cast<int64_t>(q) * m.nk] <= 0.0) {
        v = threadIdx.x == 0 ? 1.0 : 0.0;  // no relevant document: NDCG 1
      } else {
        for (int i = threadIdx.x; i < cnt; i += NT) {
          if (s_pos[i] < k) v += m.label_gain[s_label[i]] * m.discount[s_pos[i]];
        }
        v *= inv;
      }
    } else {
      const int npos = static_cast<int>(m.qconst[q]);
      // precision at every relevant document ranked within k: (relevant ranked above + 1) / (rank + 1)
      for (int i = threadIdx.x; i < cnt; i += NT) {
        if (!s_rel[i] || s_pos[i] >= k) continue;
        int hits = 0;
        for (int j = 0; j < cnt; ++j) hits += s_rel[j] && s_pos[j] < s_pos[i];
        v += static_cast<double>(hits + 1) / (s_pos[i] + 1.0f);
      }
      v = npos > 0 ? v / min(npos, k) : (threadIdx.x == 0 ? 1.0 : 0.0);
    }
    const double t = QBlockSum<NT>(v, red);
    if (threadIdx.x == 0) partials[static_cast<int64_t>(q) * m.nk + kk] = t * w;
  }
}

__global__ __launch_bounds__(kQueryThreads) void k_query_metric(MetricArgs m, double* partials) {
  __shared__ double s_score[kRankMaxDocs];
  __shared__ int s_pos[kRankMaxDocs];
  __shared__ char s_rel[kRankMaxDocs];
  __shared__ int s_label[kRankMaxDocs];
  __shared__ double red[kQueryThreads / kWave];
  const int q = blockIdx.x;
  if (m.qb[q + 1] - m.qb[q] > kRankMaxDocs) return;  // (k_query_metric_big)
  QueryMetricBody<kQueryThreads>(m, q, partials, s_score, s_pos, s_rel, s_label, red);
}

// queries of more than kRankMaxDocs documents (MetricArgs::big): the same body over the query's
// rows of a global scratch, one 1024-thread workgroup each
constexpr int kQueryBigThreads = 1024;
__global__ __launch_bounds__(kQueryBigThreads) void k_query_metric_big(MetricArgs m, double* partials, double* g_score,
                                                                        int* g_pos, char* g_rel, int* g_label) {
  __shared__ double red[kQueryBigThreads / kWave];
  const int q = blockIdx.x;
  const int b = m.qb[q];
  if (m.qb[q + 1] - b <= kRankMaxDocs) return;
  QueryMetricBody<kQueryBigThreads>(m, q, partials, g_score + b, g_pos + b, g_rel + b, g_label + b, red);
}

// one workgroup per k: the queries' values summed in query order (block-strided, then a
// fixed-shape block sum)
__global__ __launch_bounds__(kMetricThreads) void k_query_sum(const double* partials, int nq, int nk, double* out) {
  __shared__ double sh[kMetricThreads / kWave];
  double acc = 0.0;
  for (int q = threadIdx.x; q < nq; q += kMetricThreads) acc += partials[static_cast<int64_t>(q) * nk + blockIdx.x];
  acc = BlockSum(acc, sh);
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
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
  size_t d = 0;
  (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, d, static_cast<const double*>(nullptr),
                                                     static_cast<double*>(nullptr), static_cast<float*>(nullptr),
                                                     static_cast<float*>(nullptr), nn);
  return std::max(std::max(a, d), std::max(b, c));
}

}  // namespace

size_t MetricScratchBytes(int64_t n, int64_t query_values) {
  const size_t un = static_cast<size_t>(std::max<int64_t>(1, n));
  return 16 * 256 + sizeof(double) * std::max<int64_t>(kMetricBlocks, query_values) +
         un * (4 * sizeof(double) + 2 * sizeof(int32_t)) + 2 * un * sizeof(PosNeg) + 2 * un * sizeof(double) +
         sizeof(int) + CubTempBytes(n);
}

void EvalMetric(const MetricArgs& m, hipStream_t s) {
  char* p = static_cast<char*>(m.scratch);
  if (m.kind == kMetricNDCG || m.kind == kMetricMAP) {
    double* qpart = Carve<double>(&p, static_cast<size_t>(std::max(1, m.nq * m.nk)));
    hipLaunchKernelGGL(k_query_metric, dim3(m.nq), dim3(kQueryThreads), 0, s, m, qpart);
    if (m.big) {
      const size_t n = static_cast<size_t>(std::max<int64_t>(1, m.n));
      double* gs = Carve<double>(&p, n);
      int* gp = Carve<int>(&p, n);
      int* gl = Carve<int>(&p, n);
      char* gr = Carve<char>(&p, n);
      hipLaunchKernelGGL(k_query_metric_big, dim3(m.nq), dim3(kQueryBigThreads), 0, s, m, qpart, gs, gp, gr, gl);
    }
    hipLaunchKernelGGL(k_query_sum, dim3(m.nk), dim3(kMetricThreads), 0, s, qpart, m.nq, m.nk, m.out);
    return;
  }
  double* partials = Carve<double>(&p, kMetricBlocks);
  const int blocks = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>((m.n + kMetricThreads - 1) / kMetricThreads,
                                                                             kMetricBlocks)));
  if (m.kind != kMetricAUC && m.kind != kMetricAucMu) {
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
  // one binary AUC: keys (descending), the rows' (positive, negative) weights in that order,
  // tie runs, positives before each run, accumulated into out[0] / out[1]
  auto auc = [&](int ci, int cj, double* out) {
    size_t tb = temp_bytes;
    if (m.kind == kMetricAucMu) {
      hipLaunchKernelGGL(k_aucmu_keys, dim3(blocks), dim3(kMetricThreads), 0, s, m, ci, cj, keys, idx);
      (void)hipcub::DeviceRadixSort::SortPairsDescending(temp, tb, keys, keys_sorted, idx, idx_sorted, nn, 0,
                                                         sizeof(double) * 8, s);
      hipLaunchKernelGGL(k_aucmu_weights, dim3(blocks), dim3(kMetricThreads), 0, s, m, ci, cj, idx_sorted, pn);
    } else {
      // the scores sorted in place of a copy, the signed weights as the values (stable: ties
      // keep the row order, as the row-index sort did)
      float* sv = reinterpret_cast<float*>(idx);
      float* sv_sorted = reinterpret_cast<float*>(idx_sorted);
      hipLaunchKernelGGL(k_auc_signed, dim3(blocks), dim3(kMetricThreads), 0, s, m, sv);
      (void)hipcub::DeviceRadixSort::SortPairsDescending(temp, tb, m.score, keys_sorted, sv, sv_sorted, nn, 0,
                                                         sizeof(double) * 8, s);
      hipLaunchKernelGGL(k_auc_unsign, dim3(blocks), dim3(kMetricThreads), 0, s, sv_sorted, m.n, pn);
    }
    tb = temp_bytes;
    (void)hipcub::DeviceReduce::ReduceByKey(temp, tb, keys_sorted, uniq, pn, agg, num_runs, PosNegSum(), nn, s);
    hipLaunchKernelGGL(k_auc_pos, dim3(blocks), dim3(kMetricThreads), 0, s, agg, num_runs, runpos);
    tb = temp_bytes;
    // runs beyond num_runs hold stale values; the exclusive sum of the first num_runs is all that is read
    (void)hipcub::DeviceScan::ExclusiveSum(temp, tb, runpos, pos_before, nn, s);
    hipLaunchKernelGGL(k_auc_accum, dim3(blocks), dim3(kMetricThreads), 0, s, agg, pos_before, num_runs, partials, out);
    hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(kMetricThreads), 0, s, partials, blocks, out, 0);
  };
  if (m.kind == kMetricAUC) {
    auc(0, 0, m.out);
    return;
  }
  int pair = 0;
  for (int ci = 0; ci < m.num_class; ++ci) {
    for (int cj = ci + 1; cj < m.num_class; ++cj) auc(ci, cj, m.out + 2 * pair++);
  }
}

}  // namespace dev
}  // namespace lgbm_amd
