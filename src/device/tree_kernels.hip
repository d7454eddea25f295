// MI355X (gfx950) kernels of the device-resident leaf-wise tree learner.
//
// One boosting tree is grown without any host round trip:
//   TreeBegin -> RootSum -> HistRoot -> FindRoot, then num_leaves-1 times
//   SelectSplit -> PartitionCount -> PartitionScatter -> HistStep -> FindStep
// Every kernel reads the current step from HBM (dev::Step), so the sequence can be
// enqueued blindly or captured into a hipGraph; once a step finds no positive gain the
// remaining kernels of the tree exit immediately.
//
// Semantics follow the reference serial learner (reference
// src/treelearner/serial_tree_learner.cpp:152-776, feature_histogram.hpp:85-1049,
// data_partition.hpp:20-190):
//  * histograms: per-workgroup LDS-privatised fp32 (grad, hess) histograms over the
//    rows of the smaller child, 64-wide waves, then one global fp32 atomic per
//    non-empty bin; the larger child is parent - smaller (histogram subtraction).
//  * split scan: one wave per feature, forward / reverse scans with the reference's
//    missing-value routing, min_data / min_hessian filters, hessian-estimated counts,
//    L1 / max_delta_step / path smoothing / monotone-constraint gain, evaluated for all
//    thresholds in parallel (wave prefix scans) instead of sequentially.
//  * partition: stable two-pass (count, scatter) split of the leaf's index range.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>

#include "kernels.h"

namespace lgbm_amd {
namespace dev {

namespace {

int g_num_cus = 256;

constexpr int kWave = 64;
constexpr int kFindThreads = 1024;
constexpr int kMinRowsPerHistBlock = 2048;
constexpr int kPartThreads = 256;

__device__ __forceinline__ double NegInf() { return -INFINITY; }

__device__ __forceinline__ int RoundIntD(double x) { return static_cast<int>(x + 0.5f); }

__device__ __forceinline__ uint32_t GroupBin(const KArgs& a, int64_t row, int group) {
  if (a.bin_bytes == 1) {
    return static_cast<const uint8_t*>(a.bins)[row * (4 * a.words_per_row) + group];
  }
  return static_cast<const uint16_t*>(a.bins)[row * (2 * a.words_per_row) + group];
}

__device__ __forceinline__ uint32_t FeatureBinOf(const Feature& f, uint32_t gb) {
  if (gb < static_cast<uint32_t>(f.sub_lo) || gb >= static_cast<uint32_t>(f.sub_hi)) return f.mfb;
  return gb - f.sub_lo + f.offset;
}

// split decision on a feature bin (DataPartition::Split / Tree::DecisionInner semantics)
struct SplitRule {
  int32_t threshold;
  int32_t default_left;
  int32_t is_cat;
  int32_t missing_type;
  int32_t default_bin;
  int32_t max_bin;  // num_bin - 1
};

__device__ __forceinline__ bool GoesLeft(const SplitRule& r, const uint32_t* cat_bits, uint32_t bin) {
  if (r.is_cat) {
    return bin < 32u * kMaxCatWords && ((cat_bits[bin >> 5] >> (bin & 31u)) & 1u);
  }
  if ((r.missing_type == 1 && bin == static_cast<uint32_t>(r.default_bin)) ||
      (r.missing_type == 2 && bin == static_cast<uint32_t>(r.max_bin))) {
    return r.default_left != 0;
  }
  return bin <= static_cast<uint32_t>(r.threshold);
}

// ---- wave / block reductions ---------------------------------------------------
template <typename T>
__device__ __forceinline__ T WaveSum(T v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

template <typename T>
__device__ T BlockSum(T v, T* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = WaveSum(v);
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  T r = 0;
  for (int i = 0; i < nw; ++i) r += sh[i];
  return r;
}

// SplitInfo ordering: larger gain first, then smaller real feature index
__device__ __forceinline__ bool SplitBetter(double ga, int fa, double gb, int fb) {
  if (ga != ga) ga = -INFINITY;
  if (gb != gb) gb = -INFINITY;
  if (fa < 0) fa = 0x7fffffff;
  if (fb < 0) fb = 0x7fffffff;
  if (ga != gb) return ga > gb;
  return fa < fb;
}

}  // namespace

int HistGridBlocks() { return 2 * g_num_cus; }

// ==================================================================== gradients
__global__ void k_pack_gh(const float* __restrict__ g, const float* __restrict__ h, float2* __restrict__ gh,
                          int64_t n) {
  static_assert(sizeof(GH) == sizeof(float2), "GH layout");
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    gh[i] = make_float2(g[i], h[i]);
  }
}

void PackGH(const float* g, const float* h, GH* gh, int64_t n, hipStream_t s) {
  const int blocks = static_cast<int>(std::min<int64_t>((n + 255) / 256, 8 * g_num_cus));
  hipLaunchKernelGGL(k_pack_gh, dim3(std::max(blocks, 1)), dim3(256), 0, s, g, h, reinterpret_cast<float2*>(gh), n);
}

// ==================================================================== tree begin
__global__ void k_tree_begin(KArgs a) {
  const int L = a.p.num_leaves;
  for (int l = threadIdx.x; l < L; l += blockDim.x) {
    Leaf lf;
    lf.begin = 0;
    lf.count = l == 0 ? a.num_rows : 0;
    lf.global_count = lf.count;
    lf.depth = 0;
    lf.slot = l;
    lf.pad = 0;
    lf.sum_g = lf.sum_h = lf.output = 0.0;
    lf.cmin = -DBL_MAX;
    lf.cmax = DBL_MAX;
    a.leaves[l] = lf;
    a.best[l].gain = NegInf();
    a.best[l].feature = -1;
    a.best[l].real_feature = -1;
  }
  if (threadIdx.x == 0) {
    Step* st = a.st;
    st->done = 0;
    st->step = 0;
    st->leaf = 0;
    st->new_leaf = 0;
    st->smaller = 0;
    st->larger = -1;
    st->skip_find = 0;
    st->total_left = 0;
    a.root[0] = a.root[1] = a.root[2] = 0.0;
  }
}

void TreeBegin(const KArgs& a, hipStream_t s) { hipLaunchKernelGGL(k_tree_begin, dim3(1), dim3(256), 0, s, a); }

// root statistics (sum of gradients / hessians over the root rows)
__global__ __launch_bounds__(256) void k_root_sum(KArgs a) {
  __shared__ double sh[8];
  double sg = 0.0, shh = 0.0;
  const int n = a.num_rows;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int r = a.root_identity ? i : a.idx[i];
    const float2 v = reinterpret_cast<const float2*>(a.gh)[r];
    sg += v.x;
    shh += v.y;
  }
  sg = BlockSum(sg, sh);
  shh = BlockSum(shh, sh);
  if (threadIdx.x == 0) {
    atomicAdd(&a.root[0], sg);
    atomicAdd(&a.root[1], shh);
    if (blockIdx.x == 0) atomicAdd(&a.root[2], static_cast<double>(n));
  }
}

void RootSum(const KArgs& a, hipStream_t s) {
  const int blocks = std::max(1, std::min((a.num_rows + 255) / 256, 2 * g_num_cus));
  hipLaunchKernelGGL(k_root_sum, dim3(blocks), dim3(256), 0, s, a);
}

// ==================================================================== histograms
// grid: (row blocks, column tiles); each block owns one column tile (a run of 32-bit
// words of the row) and a contiguous chunk of the leaf's rows.
template <int MODE>  // 0 root, 1 split step, 2 explicit range
__global__ __launch_bounds__(kHistBlockThreads) void k_hist(KArgs a) {
  extern __shared__ float lds[];
  constexpr bool ROOT = MODE == 0;
  int begin, count;
  const int32_t* src;
  const float2* gh = reinterpret_cast<const float2*>(a.gh);
  if (MODE == 0) {
    begin = 0;
    count = a.num_rows;
    src = a.root_identity ? nullptr : a.idx;
  } else if (MODE == 2) {
    begin = a.range_begin;
    count = a.num_rows;
    src = a.idx;
  } else {
    const Step* st = a.st;
    if (st->done) return;
    // copy the partitioned range of the split leaf back into the index array
    const int pb = st->part_begin, pc = st->part_count;
    const int nthreads = gridDim.x * gridDim.y * blockDim.x;
    const int gtid = (blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x;
    for (int i = gtid; i < pc; i += nthreads) a.idx[pb + i] = a.tmp[pb + i];
    if (st->skip_find) return;
    const Leaf& sm = a.leaves[st->smaller];
    begin = sm.begin;
    count = sm.count;
    src = a.tmp;
  }
  if (count <= 0) return;
  const int active = min(static_cast<int>(gridDim.x), max(1, count / kMinRowsPerHistBlock));
  if (static_cast<int>(blockIdx.x) >= active) return;
  const int chunk = (count + active - 1) / active;
  const int r0 = begin + blockIdx.x * chunk;
  const int r1 = min(begin + count, r0 + chunk);

  // column tile of this block
  const int gpw = a.bin_bytes == 1 ? 4 : 2;  // groups per 32-bit word
  const int w0 = blockIdx.y * a.tile_words;
  const int w1 = min(a.words_per_row, w0 + a.tile_words);
  const int g0 = w0 * gpw;
  const int g_end = min(a.p.num_groups, w1 * gpw);
  const int lo_bin = a.group_off[g0];
  const int hi_bin = g_end < a.p.num_groups ? a.group_off[g_end] : a.p.total_bins;
  const int nbins2 = 2 * (hi_bin - lo_bin);
  for (int i = threadIdx.x; i < nbins2; i += blockDim.x) lds[i] = 0.f;
  __syncthreads();

  const int tpr = w1 - w0;  // threads per row
  const int rpp = blockDim.x / tpr;
  const int q = threadIdx.x % tpr;
  const int rs = threadIdx.x / tpr;
  if (rs < rpp) {
    const int w = w0 + q;
    int goff[4];
    for (int j = 0; j < 4; ++j) {
      const int g = w * gpw + j;
      goff[j] = (j < gpw && g < a.p.num_groups) ? 2 * (a.group_off[g] - lo_bin) : -1;
    }
    const uint32_t* bins32 = static_cast<const uint32_t*>(a.bins);
    const int64_t wpr = a.words_per_row;
    const bool write_iota = ROOT && src == nullptr && q == 0 && blockIdx.y == 0;
    int i = r0 + rs;
    // 2 rows in flight per thread
    for (; i + rpp < r1; i += 2 * rpp) {
      const int ra = src ? src[i] : i;
      const int rb = src ? src[i + rpp] : i + rpp;
      if (write_iota) {
        a.idx[i] = i;
        a.idx[i + rpp] = i + rpp;
      }
      const float2 va = gh[ra];
      const float2 vb = gh[rb];
      const uint32_t wa = bins32[ra * wpr + w];
      const uint32_t wb = bins32[rb * wpr + w];
      if (gpw == 4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (goff[j] >= 0) {
            const int ba = goff[j] + 2 * ((wa >> (8 * j)) & 0xffu);
            const int bb = goff[j] + 2 * ((wb >> (8 * j)) & 0xffu);
            atomicAdd(&lds[ba], va.x);
            atomicAdd(&lds[ba + 1], va.y);
            atomicAdd(&lds[bb], vb.x);
            atomicAdd(&lds[bb + 1], vb.y);
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if (goff[j] >= 0) {
            const int ba = goff[j] + 2 * ((wa >> (16 * j)) & 0xffffu);
            const int bb = goff[j] + 2 * ((wb >> (16 * j)) & 0xffffu);
            atomicAdd(&lds[ba], va.x);
            atomicAdd(&lds[ba + 1], va.y);
            atomicAdd(&lds[bb], vb.x);
            atomicAdd(&lds[bb + 1], vb.y);
          }
        }
      }
    }
    for (; i < r1; i += rpp) {
      const int ra = src ? src[i] : i;
      if (write_iota) a.idx[i] = i;
      const float2 va = gh[ra];
      const uint32_t wa = bins32[ra * wpr + w];
      for (int j = 0; j < gpw; ++j) {
        if (goff[j] >= 0) {
          const uint32_t b = gpw == 4 ? ((wa >> (8 * j)) & 0xffu) : ((wa >> (16 * j)) & 0xffffu);
          const int ba = goff[j] + 2 * static_cast<int>(b);
          atomicAdd(&lds[ba], va.x);
          atomicAdd(&lds[ba + 1], va.y);
        }
      }
    }
  }
  __syncthreads();
  float* out = a.scratch + 2 * lo_bin;
  for (int i = threadIdx.x; i < nbins2; i += blockDim.x) {
    const float v = lds[i];
    if (v != 0.f) atomicAdd(&out[i], v);
  }
}

static void LaunchHist(const KArgs& a, hipStream_t s, int mode) {
  const size_t lds_bytes = sizeof(float) * 2 * static_cast<size_t>(a.tile_bins);
  dim3 grid(HistGridBlocks(), a.hist_tiles);
  if (mode == 0) {
    hipLaunchKernelGGL(k_hist<0>, grid, dim3(kHistBlockThreads), lds_bytes, s, a);
  } else if (mode == 1) {
    hipLaunchKernelGGL(k_hist<1>, grid, dim3(kHistBlockThreads), lds_bytes, s, a);
  } else {
    hipLaunchKernelGGL(k_hist<2>, grid, dim3(kHistBlockThreads), lds_bytes, s, a);
  }
}

void HistRoot(const KArgs& a, hipStream_t s) { LaunchHist(a, s, 0); }
void HistStep(const KArgs& a, hipStream_t s) { LaunchHist(a, s, 1); }
void HistRange(const KArgs& a, hipStream_t s) { LaunchHist(a, s, 2); }

// ==================================================================== split scan
namespace {

struct Cand {
  double gain;
  int thr;
  double lg, lh;
  int lc;
};

// better for the reverse scan: higher gain, ties -> higher threshold (first met scanning down)
__device__ __forceinline__ bool CandBetter(const Cand& x, const Cand& y, bool reverse) {
  if (x.gain > y.gain) return true;
  if (x.gain < y.gain || x.gain != x.gain) return false;
  if (y.gain != y.gain) return true;
  return reverse ? x.thr > y.thr : x.thr < y.thr;
}

__device__ __forceinline__ Cand WaveBestCand(Cand c, bool reverse) {
  for (int o = 32; o > 0; o >>= 1) {
    Cand o2;
    o2.gain = __shfl_xor(c.gain, o, kWave);
    o2.thr = __shfl_xor(c.thr, o, kWave);
    o2.lg = __shfl_xor(c.lg, o, kWave);
    o2.lh = __shfl_xor(c.lh, o, kWave);
    o2.lc = __shfl_xor(c.lc, o, kWave);
    if (CandBetter(o2, c, reverse)) c = o2;
  }
  return c;
}

struct LeafCtx {
  double sg, sh;  // sh already includes + 2*kEpsilon
  int n;
  double cnt_factor;
  double parent_out;
  double min_gain_shift;
  ConstraintRange c;
};

// inclusive suffix (down) / prefix (up) scans across the wave
template <typename T>
__device__ __forceinline__ T WaveSuffixIncl(T v) {
  const int lane = threadIdx.x & 63;
  for (int o = 1; o < 64; o <<= 1) {
    T t = __shfl_down(v, o, kWave);
    if (lane + o < 64) v += t;
  }
  return v;
}
template <typename T>
__device__ __forceinline__ T WavePrefixIncl(T v) {
  const int lane = threadIdx.x & 63;
  for (int o = 1; o < 64; o <<= 1) {
    T t = __shfl_up(v, o, kWave);
    if (lane >= o) v += t;
  }
  return v;
}

// a feature's histogram with its most-frequent bin restored (Dataset::FixHistogram)
struct HistView {
  const float* h;
  int fix_t;  // bin whose value is reconstructed from the leaf totals (-1: none)
  double fix_g, fix_h;
  __device__ __forceinline__ double G(int t) const { return t == fix_t ? fix_g : static_cast<double>(h[2 * t]); }
  __device__ __forceinline__ double H(int t) const { return t == fix_t ? fix_h : static_cast<double>(h[2 * t + 1]); }
};

// one numerical scan of one feature by one wave (reference FindBestThresholdSequentially)
__device__ Cand ScanNumericalWave(const HistView& hv, int nb, int offset, int default_bin, bool reverse,
                                  bool skip_def, bool na, const LeafCtx& L, const SplitParams& p, int mono,
                                  bool* splittable) {
  const int lane = threadIdx.x & 63;
  const int K = (nb + 63) / 64;
  const int b0 = lane * K;
  const int b1 = min(nb, b0 + K);
  const int t_start_r = nb - 1 - (na ? 1 : 0);
  const int t_end_r = 1 - offset;
  const int t_end_f = nb - 2;
  auto acc = [&](int t) -> bool {
    if (skip_def && t + offset == default_bin) return false;
    if (reverse) return t >= t_end_r && t <= t_start_r;
    return t >= 0 && t <= t_end_f;
  };
  // lane totals
  double tg = 0.0, th = 0.0;
  int tc = 0;
  for (int t = b0; t < b1; ++t) {
    if (!acc(t)) continue;
    const double g = hv.G(t), hh = hv.H(t);
    tg += g;
    th += hh;
    tc += RoundIntD(hh * L.cnt_factor);
  }
  Cand best;
  best.gain = -INFINITY;
  best.thr = reverse ? -1 : 0x7fffffff;
  best.lg = best.lh = 0.0;
  best.lc = 0;
  bool any = false;
  const double min_h = p.min_sum_hessian_in_leaf;
  const int min_n = p.min_data_in_leaf;
  if (reverse) {
    const double ig = WaveSuffixIncl(tg), ih = WaveSuffixIncl(th);
    const int ic = WaveSuffixIncl(tc);
    double rg = ig - tg, rh = ih - th;  // exclusive suffix (bins above this lane)
    int rc = ic - tc;
    rh += kEpsilon;
    for (int t = b1 - 1; t >= b0; --t) {
      if (!acc(t)) continue;
      const double g = hv.G(t), hh = hv.H(t);
      rg += g;
      rh += hh;
      rc += RoundIntD(hh * L.cnt_factor);
      if (rc < min_n || rh < min_h) continue;
      const int lc = L.n - rc;
      if (lc < min_n) continue;
      const double lh = L.sh - rh;
      if (lh < min_h) continue;
      const double lg = L.sg - rg;
      const double gain = SplitGain(lg, lh, rg, rh, p.lambda_l2, p, L.c, static_cast<int8_t>(mono), lc, rc, L.parent_out);
      if (gain <= L.min_gain_shift) continue;
      any = true;
      if (gain > best.gain) {
        best.gain = gain;
        best.thr = t - 1 + offset;
        best.lg = lg;
        best.lh = lh;
        best.lc = lc;
      }
    }
  } else {
    double lg0 = 0.0, lh0 = kEpsilon;
    int lc0 = 0;
    const bool minus_one = na && offset == 1;
    if (minus_one) {
      // left starts with everything outside the stored bins (the most frequent bin 0)
      double ag = 0.0, ah = 0.0;
      int ac = 0;
      for (int t = b0; t < b1; ++t) {
        const double hh = hv.H(t);
        ag += hv.G(t);
        ah += hh;
        ac += RoundIntD(hh * L.cnt_factor);
      }
      ag = WaveSum(ag);
      ah = WaveSum(ah);
      ac = WaveSum(ac);
      lg0 = L.sg - ag;
      lh0 = L.sh - kEpsilon - ah;
      lc0 = L.n - ac;
    }
    const double ig = WavePrefixIncl(tg), ih = WavePrefixIncl(th);
    const int ic = WavePrefixIncl(tc);
    double lg = lg0 + (ig - tg), lh = lh0 + (ih - th);
    int lc = lc0 + (ic - tc);
    auto eval = [&](int t, double xg, double xh, int xc) {
      if (xc < min_n || xh < min_h) return;
      const int rc = L.n - xc;
      if (rc < min_n) return;
      const double rh = L.sh - xh;
      if (rh < min_h) return;
      const double rg = L.sg - xg;
      const double gain = SplitGain(xg, xh, rg, rh, p.lambda_l2, p, L.c, static_cast<int8_t>(mono), xc, rc, L.parent_out);
      if (gain <= L.min_gain_shift) return;
      any = true;
      if (gain > best.gain) {
        best.gain = gain;
        best.thr = t + offset;
        best.lg = xg;
        best.lh = xh;
        best.lc = xc;
      }
    };
    if (minus_one && lane == 0 && !(skip_def && offset - 1 == default_bin)) eval(-1, lg0, lh0, lc0);
    for (int t = b0; t < b1; ++t) {
      if (!acc(t)) continue;
      const double g = hv.G(t), hh = hv.H(t);
      lg += g;
      lh += hh;
      lc += RoundIntD(hh * L.cnt_factor);
      eval(t, lg, lh, lc);
    }
  }
  if (__any(any)) *splittable = true;
  return WaveBestCand(best, reverse);
}

struct FeatOut {
  double gain;
  int feature, real_feature, thr, default_left, lc, rc, mono;
  double lg, lh, rg, rh, lo, ro;
};

__device__ void FindNumericalWave(const Feature& F, float* __restrict__ h, const LeafCtx& L,
                                  const SplitParams& p, int depth, double mono_penalty, FeatOut* out) {
  const int nb = F.num_bin - F.offset;
  HistView hv;
  hv.h = h;
  hv.fix_t = -1;
  hv.fix_g = hv.fix_h = 0.0;
  if (F.mfb > 0) {
    // FixHistogram: the most frequent bin is not accumulated; rebuild it from the leaf totals
    double sg = 0.0, sh = 0.0;
    const int lane = threadIdx.x & 63;
    for (int t = lane; t < nb; t += 64) {
      if (t == F.mfb) continue;
      sg += h[2 * t];
      sh += h[2 * t + 1];
    }
    sg = WaveSum(sg);
    sh = WaveSum(sh);
    hv.fix_t = F.mfb;
    hv.fix_g = L.sg - sg;
    hv.fix_h = (L.sh - 2 * kEpsilon) - sh;
    if (lane == 0) {
      h[2 * F.mfb] = static_cast<float>(hv.fix_g);
      h[2 * F.mfb + 1] = static_cast<float>(hv.fix_h);
    }
  }
  out->gain = -INFINITY;
  out->default_left = 1;
  out->mono = F.monotone;
  bool splittable = false;
  auto apply = [&](const Cand& b, bool reverse) {
    if (splittable && b.gain > out->gain + L.min_gain_shift) {
      out->thr = b.thr;
      out->lo = LeafOutputConstrained(b.lg, b.lh, p.lambda_l2, p, L.c, b.lc, L.parent_out);
      out->lc = b.lc;
      out->lg = b.lg;
      out->lh = b.lh - kEpsilon;
      out->ro = LeafOutputConstrained(L.sg - b.lg, L.sh - b.lh, p.lambda_l2, p, L.c, L.n - b.lc, L.parent_out);
      out->rc = L.n - b.lc;
      out->rg = L.sg - b.lg;
      out->rh = L.sh - b.lh - kEpsilon;
      out->gain = b.gain - L.min_gain_shift;
      out->default_left = reverse ? 1 : 0;
    }
  };
  if (F.num_bin > 2 && F.missing_type != 0) {
    if (F.missing_type == 1) {
      apply(ScanNumericalWave(hv, nb, F.offset, F.default_bin, true, true, false, L, p, F.monotone, &splittable), true);
      apply(ScanNumericalWave(hv, nb, F.offset, F.default_bin, false, true, false, L, p, F.monotone, &splittable), false);
    } else {
      apply(ScanNumericalWave(hv, nb, F.offset, F.default_bin, true, false, true, L, p, F.monotone, &splittable), true);
      apply(ScanNumericalWave(hv, nb, F.offset, F.default_bin, false, false, true, L, p, F.monotone, &splittable), false);
    }
  } else {
    apply(ScanNumericalWave(hv, nb, F.offset, F.default_bin, true, false, false, L, p, F.monotone, &splittable), true);
    if (F.missing_type == 2) out->default_left = 0;
  }
  out->gain *= F.penalty;
  if (F.monotone != 0) {
    // MonotoneSplitPenalty(depth, penalization)
    double pen;
    if (mono_penalty >= depth + 1.) pen = kEpsilon;
    else if (mono_penalty <= 1.) pen = 1. - mono_penalty / pow(2., depth) + kEpsilon;
    else pen = 1. - pow(2., mono_penalty - 1. - depth) + kEpsilon;
    out->gain *= pen;
  }
}

}  // namespace

template <bool ROOT>
__global__ __launch_bounds__(kFindThreads) void k_find(KArgs a) {
  __shared__ FeatOut wbest[kFindThreads / kWave];
  int leaf;
  bool is_smaller = true;
  if (ROOT) {
    if (blockIdx.x != 0) return;
    leaf = 0;
  } else {
    const Step* st = a.st;
    if (st->done || st->skip_find) return;
    is_smaller = blockIdx.x == 0;
    leaf = is_smaller ? st->smaller : st->larger;
  }
  const SplitParams& p = a.p.sp;
  LeafCtx L;
  int depth;
  int slot;
  if (ROOT) {
    const double sg = a.root[0], sh = a.root[1];
    const int n = static_cast<int>(a.root[2]);
    ConstraintRange c;
    c.min = -DBL_MAX;
    c.max = DBL_MAX;
    SplitParams rp = p;
    rp.use_l1 = 1;
    rp.use_max_output = 1;
    rp.use_smoothing = 0;
    rp.use_mc = 1;
    const double out0 = LeafOutputConstrained(sg, sh, p.lambda_l2, rp, c, n, 0);
    if (threadIdx.x == 0) {
      Leaf& lf = a.leaves[0];
      lf.sum_g = sg;
      lf.sum_h = sh;
      lf.global_count = n;
      lf.output = out0;
    }
    L.sg = sg;
    L.sh = sh + 2 * kEpsilon;
    L.n = n;
    L.parent_out = out0;
    L.c = c;
    depth = 0;
    slot = 0;
  } else {
    const Leaf lf = a.leaves[leaf];
    L.sg = lf.sum_g;
    L.sh = lf.sum_h + 2 * kEpsilon;
    L.n = lf.global_count;
    L.parent_out = lf.output;
    L.c.min = lf.cmin;
    L.c.max = lf.cmax;
    depth = lf.depth;
    slot = lf.slot;
  }
  L.cnt_factor = L.n / L.sh;
  const double gain_shift = LeafGain(L.sg, L.sh, p.lambda_l1, p.lambda_l2, p.max_delta_step, p.path_smooth, L.n,
                                     L.parent_out, p.use_l1, p.use_max_output, p.use_smoothing);
  L.min_gain_shift = gain_shift + p.min_gain_to_split;

  // materialise this leaf's histogram in its slot: smaller = built one, larger = parent - built
  const int nh = 2 * a.p.total_bins;
  float* dst = a.hist + static_cast<size_t>(slot) * nh;
  if (is_smaller) {
    for (int i = threadIdx.x; i < nh; i += blockDim.x) dst[i] = a.scratch[i];
  } else {
    for (int i = threadIdx.x; i < nh; i += blockDim.x) dst[i] -= a.scratch[i];
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  FeatOut mine;
  mine.gain = -INFINITY;
  mine.feature = -1;
  mine.real_feature = -1;
  for (int f = w; f < a.p.num_features; f += nw) {
    if (!a.tree_mask[f]) continue;
    const Feature F = a.feat[f];
    if (F.is_cat) continue;  // categorical splits are searched by the host-assisted path
    FeatOut o;
    o.feature = f;
    o.real_feature = F.real_index;
    o.thr = 0;
    o.lc = o.rc = 0;
    o.lg = o.lh = o.rg = o.rh = o.lo = o.ro = 0.0;
    FindNumericalWave(F, dst + 2 * F.hist_offset, L, p, depth, a.p.monotone_penalty, &o);
    if (SplitBetter(o.gain, o.real_feature, mine.gain, mine.real_feature)) mine = o;
  }
  if (lane == 0) wbest[w] = mine;
  __syncthreads();
  if (threadIdx.x == 0) {
    FeatOut b = wbest[0];
    for (int i = 1; i < nw; ++i) {
      if (SplitBetter(wbest[i].gain, wbest[i].real_feature, b.gain, b.real_feature)) b = wbest[i];
    }
    DeviceSplit& d = a.best[leaf];
    d.gain = b.gain;
    d.feature = b.feature;
    d.real_feature = b.real_feature;
    if (b.feature >= 0) {
      d.threshold = b.thr;
      d.left_count = b.lc;
      d.right_count = b.rc;
      d.left_output = b.lo;
      d.right_output = b.ro;
      d.left_sum_gradient = b.lg;
      d.left_sum_hessian = b.lh;
      d.right_sum_gradient = b.rg;
      d.right_sum_hessian = b.rh;
      d.default_left = static_cast<int8_t>(b.default_left);
      d.monotone_type = static_cast<int8_t>(b.mono);
      d.is_categorical = 0;
      d.num_cat_threshold = 0;
    }
  }
}

void FindRoot(const KArgs& a, hipStream_t s) { hipLaunchKernelGGL(k_find<true>, dim3(1), dim3(kFindThreads), 0, s, a); }
void FindStep(const KArgs& a, hipStream_t s) { hipLaunchKernelGGL(k_find<false>, dim3(2), dim3(kFindThreads), 0, s, a); }

// ==================================================================== select + apply
__global__ __launch_bounds__(256) void k_select(KArgs a) {
  __shared__ double sg[256];
  __shared__ int sf[256], sl[256];
  Step* st = a.st;
  if (st->done) return;
  const int s = st->step;
  const int L = a.p.num_leaves;
  if (s >= L - 1) {
    if (threadIdx.x == 0) st->done = 1;
    return;
  }
  double bg = -INFINITY;
  int bf = -1, bl = 0x7fffffff;
  for (int l = threadIdx.x; l <= s; l += blockDim.x) {
    const DeviceSplit& d = a.best[l];
    if (bl == 0x7fffffff || SplitBetter(d.gain, d.real_feature, bg, bf)) {
      bg = d.gain;
      bf = d.real_feature;
      bl = l;
    }
  }
  sg[threadIdx.x] = bg;
  sf[threadIdx.x] = bf;
  sl[threadIdx.x] = bl;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const int j = threadIdx.x + o;
      const bool take = sl[j] != 0x7fffffff &&
                        (sl[threadIdx.x] == 0x7fffffff || SplitBetter(sg[j], sf[j], sg[threadIdx.x], sf[threadIdx.x]) ||
                         (!SplitBetter(sg[threadIdx.x], sf[threadIdx.x], sg[j], sf[j]) && sl[j] < sl[threadIdx.x]));
      if (take) {
        sg[threadIdx.x] = sg[j];
        sf[threadIdx.x] = sf[j];
        sl[threadIdx.x] = sl[j];
      }
    }
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  const int leaf = sl[0];
  const DeviceSplit sp = a.best[leaf];
  if (!(sp.gain > 0.0) || sp.feature < 0) {
    st->done = 1;
    return;
  }
  const int nl = s + 1;
  Leaf P = a.leaves[leaf];
  st->leaf = leaf;
  st->new_leaf = nl;
  st->split = sp;
  st->part_begin = P.begin;
  st->part_count = P.count;
  int nb = (P.count + 4095) / 4096;
  nb = max(1, min(kMaxPartBlocks, nb));
  int rpb = (P.count + nb - 1) / nb;
  rpb = ((rpb + kPartThreads - 1) / kPartThreads) * kPartThreads;
  if (rpb == 0) rpb = kPartThreads;
  nb = max(1, (P.count + rpb - 1) / rpb);
  st->num_blocks = nb;
  st->rows_per_block = rpb;
  SplitRecord& r = a.rec[s];
  r.leaf = leaf;
  r.split = sp;
  r.left_count = sp.left_count;
  r.right_count = sp.right_count;
  // children (left keeps the leaf id)
  Leaf R = P;
  P.depth += 1;
  R.depth = P.depth;
  P.sum_g = sp.left_sum_gradient;
  P.sum_h = sp.left_sum_hessian;
  P.output = sp.left_output;
  R.sum_g = sp.right_sum_gradient;
  R.sum_h = sp.right_sum_hessian;
  R.output = sp.right_output;
  P.global_count = sp.left_count;
  R.global_count = sp.right_count;
  R.slot = a.leaves[nl].slot;
  if (!sp.is_categorical) {
    // basic monotone constraints (LeafConstraints::Update)
    const double mid = (sp.left_output + sp.right_output) / 2.0f;
    if (sp.monotone_type < 0) {
      P.cmin = fmax(P.cmin, mid);
      R.cmax = fmin(R.cmax, mid);
    } else if (sp.monotone_type > 0) {
      P.cmax = fmin(P.cmax, mid);
      R.cmin = fmax(R.cmin, mid);
    }
  }
  a.leaves[leaf] = P;
  a.leaves[nl] = R;
  a.best[leaf].gain = -INFINITY;
  a.best[leaf].feature = -1;
  a.best[leaf].real_feature = -1;
  a.best[nl].gain = -INFINITY;
  a.best[nl].feature = -1;
  a.best[nl].real_feature = -1;
}

void SelectSplit(const KArgs& a, hipStream_t s) { hipLaunchKernelGGL(k_select, dim3(1), dim3(256), 0, s, a); }

// ==================================================================== partition
namespace {
__device__ __forceinline__ void LoadRule(const KArgs& a, SplitRule* r, Feature* f, uint32_t* cat_bits_lds) {
  const DeviceSplit& sp = a.st->split;
  *f = a.feat[sp.feature];
  r->threshold = sp.threshold;
  r->default_left = sp.default_left;
  r->is_cat = sp.is_categorical;
  r->missing_type = f->missing_type;
  r->default_bin = f->default_bin;
  r->max_bin = f->num_bin - 1;
  if (sp.is_categorical) {
    for (int i = threadIdx.x; i < kMaxCatWords; i += blockDim.x) cat_bits_lds[i] = sp.cat_bits[i];
  }
}
}  // namespace

__global__ __launch_bounds__(kPartThreads) void k_part_count(KArgs a) {
  __shared__ uint32_t cat_bits[kMaxCatWords];
  __shared__ int red[8];
  const Step* st = a.st;
  if (st->done) return;
  const int b = blockIdx.x;
  if (b >= st->num_blocks) return;
  SplitRule r;
  Feature F;
  LoadRule(a, &r, &F, cat_bits);
  __syncthreads();
  const int pb = st->part_begin, pc = st->part_count, rpb = st->rows_per_block;
  const int s0 = b * rpb, s1 = min(pc, s0 + rpb);
  int cnt = 0;
  for (int i = s0 + threadIdx.x; i < s1; i += blockDim.x) {
    const int row = a.idx[pb + i];
    const uint32_t bin = FeatureBinOf(F, GroupBin(a, row, F.group));
    cnt += GoesLeft(r, cat_bits, bin) ? 1 : 0;
  }
  cnt = BlockSum(cnt, red);
  if (threadIdx.x == 0) a.blk[b] = cnt;
}

void PartitionCount(const KArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_part_count, dim3(kMaxPartBlocks), dim3(kPartThreads), 0, s, a);
}

__global__ __launch_bounds__(kPartThreads) void k_part_scatter(KArgs a) {
  __shared__ uint32_t cat_bits[kMaxCatWords];
  __shared__ int red[8];
  __shared__ int wl[kPartThreads / kWave];
  Step* st = a.st;
  if (st->done) return;
  const int b = blockIdx.x;
  const int nb = st->num_blocks;
  if (b >= nb) return;
  SplitRule r;
  Feature F;
  LoadRule(a, &r, &F, cat_bits);
  // left rows before this block and in total
  int before = 0, total = 0;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) {
    const int c = a.blk[i];
    total += c;
    if (i < b) before += c;
  }
  before = BlockSum(before, red);
  total = BlockSum(total, red);
  const int pb = st->part_begin, pc = st->part_count, rpb = st->rows_per_block;
  const int s0 = b * rpb, s1 = min(pc, s0 + rpb);
  int run_l = 0, run_r = 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int left_base = pb + before;
  const int right_base = pb + total + (s0 - before);
  for (int t0 = s0; t0 < s1; t0 += blockDim.x) {
    const int i = t0 + threadIdx.x;
    int row = 0;
    bool left = false;
    const bool valid = i < s1;
    if (valid) {
      row = a.idx[pb + i];
      left = GoesLeft(r, cat_bits, FeatureBinOf(F, GroupBin(a, row, F.group)));
    }
    const unsigned long long m = __ballot(valid && left);
    const unsigned long long mv = __ballot(valid);
    const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int pl = __popcll(m & lt);
    const int pv = __popcll(mv & lt);
    __syncthreads();
    if (lane == 0) wl[w] = __popcll(m);
    __syncthreads();
    int wbefore_l = 0, tile_l = 0;
    for (int k = 0; k < nw; ++k) {
      if (k < w) wbefore_l += wl[k];
      tile_l += wl[k];
    }
    // rows of this wave before this lane: w*64 + pv (all valid rows precede invalid ones)
    const int pos_in_tile = w * 64 + pv;
    if (valid) {
      if (left) {
        a.tmp[left_base + run_l + wbefore_l + pl] = row;
      } else {
        const int lpos = wbefore_l + pl;  // lefts before me in the tile
        a.tmp[right_base + run_r + (pos_in_tile - lpos)] = row;
      }
    }
    const int tile_valid = min(static_cast<int>(blockDim.x), s1 - t0);
    run_l += tile_l;
    run_r += tile_valid - tile_l;
  }
  if (b == 0 && threadIdx.x == 0) {
    // bookkeeping of the two children
    const int leaf = st->leaf, nl = st->new_leaf;
    Leaf P = a.leaves[leaf];
    Leaf R = a.leaves[nl];
    P.begin = pb;
    P.count = total;
    R.begin = pb + total;
    R.count = pc - total;
    SplitRecord& rec = a.rec[st->step];
    if (!a.p.data_parallel) {
      P.global_count = P.count;
      R.global_count = R.count;
      rec.left_count = P.count;
      rec.right_count = R.count;
    }
    const int nlft = P.global_count, nrgt = R.global_count;
    bool skip = (a.p.max_depth > 0 && P.depth >= a.p.max_depth) ||
                (nrgt < 2 * a.p.sp.min_data_in_leaf && nlft < 2 * a.p.sp.min_data_in_leaf) ||
                (st->step + 1 >= a.p.num_leaves - 1);
    if (!skip) {
      if (nlft < nrgt) {
        // parent histogram moves to the (larger) right child
        const int t = P.slot;
        P.slot = R.slot;
        R.slot = t;
        st->smaller = leaf;
        st->larger = nl;
      } else {
        st->smaller = nl;
        st->larger = leaf;
      }
    }
    a.leaves[leaf] = P;
    a.leaves[nl] = R;
    st->skip_find = skip ? 1 : 0;
    st->total_left = total;
    st->step = st->step + 1;
  }
}

void PartitionScatter(const KArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_part_scatter, dim3(kMaxPartBlocks), dim3(kPartThreads), 0, s, a);
}

// ==================================================================== score updates
__global__ void k_add_leaf_score(KArgs a, const double* __restrict__ vals, int num_leaves, double* __restrict__ score) {
  const int leaf = blockIdx.y;
  if (leaf >= num_leaves) return;
  const Leaf lf = a.leaves[leaf];
  const double v = vals[leaf];
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < lf.count; i += gridDim.x * blockDim.x) {
    score[a.idx[lf.begin + i]] += v;
  }
}

void AddLeafScore(const KArgs& a, const double* leaf_values, int num_leaves, double* score, hipStream_t s) {
  const int bx = std::max(1, std::min(64, (a.num_rows / std::max(1, num_leaves) + 255) / 256));
  hipLaunchKernelGGL(k_add_leaf_score, dim3(bx, num_leaves), dim3(256), 0, s, a, leaf_values, num_leaves, score);
}

__global__ void k_add_tree_score(KArgs a, DevTree t, const int32_t* __restrict__ rows, int64_t n,
                                 double* __restrict__ score) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int row = rows ? rows[i] : static_cast<int>(i);
    int node = 0;
    if (t.num_leaves > 1) {
      while (node >= 0) {
        const int f = t.split_feature_inner[node];
        const Feature F = a.feat[f];
        const uint32_t bin = FeatureBinOf(F, GroupBin(a, row, F.group));
        const int8_t dt = t.decision_type[node];
        bool left;
        if (dt & 1) {
          const int ci = static_cast<int>(t.threshold_in_bin[node]);
          const int lo = t.cat_boundaries_inner[ci], hi = t.cat_boundaries_inner[ci + 1];
          const int word = static_cast<int>(bin >> 5);
          left = word < hi - lo && ((t.cat_threshold_inner[lo + word] >> (bin & 31u)) & 1u);
        } else {
          const int mt = (dt >> 2) & 3;
          if ((mt == 1 && bin == static_cast<uint32_t>(F.default_bin)) ||
              (mt == 2 && bin == static_cast<uint32_t>(F.num_bin - 1))) {
            left = (dt & 2) != 0;
          } else {
            left = bin <= t.threshold_in_bin[node];
          }
        }
        node = left ? t.left_child[node] : t.right_child[node];
      }
      node = ~node;
    }
    score[row] += t.leaf_value[node];
  }
}

void AddTreeScore(const KArgs& a, const DevTree& t, const int32_t* rows, int64_t num_rows, double* score,
                  hipStream_t s) {
  if (num_rows <= 0) return;
  const int blocks = static_cast<int>(std::min<int64_t>((num_rows + 255) / 256, 8 * g_num_cus));
  hipLaunchKernelGGL(k_add_tree_score, dim3(blocks), dim3(256), 0, s, a, t, rows, num_rows, score);
}

__global__ void k_add_const(double* s, int64_t n, double v) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    s[i] += v;
}
__global__ void k_mul_const(double* s, int64_t n, double v) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    s[i] *= v;
}

__global__ void k_iota(int32_t* p, int64_t n) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    p[i] = static_cast<int32_t>(i);
}

void Iota(int32_t* p, int64_t n, hipStream_t s) {
  const int blocks = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8 * g_num_cus)));
  hipLaunchKernelGGL(k_iota, dim3(blocks), dim3(256), 0, s, p, n);
}

void AddConst(double* score, int64_t n, double v, hipStream_t s) {
  const int blocks = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8 * g_num_cus)));
  hipLaunchKernelGGL(k_add_const, dim3(blocks), dim3(256), 0, s, score, n, v);
}
void MulConst(double* score, int64_t n, double v, hipStream_t s) {
  const int blocks = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8 * g_num_cus)));
  hipLaunchKernelGGL(k_mul_const, dim3(blocks), dim3(256), 0, s, score, n, v);
}

// ==================================================================== objectives
__global__ void k_gradients(GradArgs ga) {
  const int64_t n = ga.num_data;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const double w = ga.weights ? ga.weights[i] : 1.0;
    const double y = ga.label[i];
    const double s = ga.score[i];
    double g = 0, h = 0;
    switch (ga.kind) {
      case 1:  // L2
        g = (s - y) * w;
        h = w;
        break;
      case 2: {  // L1
        const double d = s - y;
        g = ((d > 0) - (d < 0)) * w;
        h = w;
        break;
      }
      case 3: {  // Huber
        const double d = s - y;
        g = (fabs(d) <= ga.p0 ? d : ((d > 0) - (d < 0)) * ga.p0) * w;
        h = w;
        break;
      }
      case 4: {  // Fair
        const double x = s - y, c = ga.p0;
        g = c * x / (fabs(x) + c) * w;
        h = c * c / ((fabs(x) + c) * (fabs(x) + c)) * w;
        break;
      }
      case 5:  // Poisson
        g = (exp(s) - y) * w;
        h = exp(s + ga.p0) * w;
        break;
      case 6: {  // Quantile
        const float d = static_cast<float>(s - y);
        const float alpha = static_cast<float>(ga.p0);
        if (ga.weights) {
          g = (d >= 0 ? (1.0f - alpha) : -alpha) * w;
          h = w;
        } else {
          g = d >= 0 ? (1.0f - alpha) : -alpha;
          h = 1.0f;
        }
        break;
      }
      case 7: {  // MAPE
        const double d = s - y;
        g = ((d > 0) - (d < 0)) * static_cast<double>(ga.label_weight[i]);
        h = ga.weights ? ga.weights[i] : 1.0f;
        break;
      }
      case 8:  // Gamma
        if (ga.weights) {
          g = 1.0 - y / exp(s) * w;
          h = y / exp(s) * w;
        } else {
          g = 1.0 - y / exp(s);
          h = y / exp(s);
        }
        break;
      case 9: {  // Tweedie
        const double rho = ga.p0;
        const double e1 = exp((1 - rho) * s), e2 = exp((2 - rho) * s);
        g = (-y * e1 + e2) * w;
        h = (-y * (1 - rho) * e1 + (2 - rho) * e2) * w;
        break;
      }
      case 10: {  // binary logloss
        const int pos = y > 0;
        const int lab = pos ? 1 : -1;
        const double lw = pos ? ga.lw1 : ga.lw0;
        const double sig = ga.p0;
        const double resp = -lab * sig / (1.0f + exp(lab * sig * s));
        const double ar = fabs(resp);
        g = resp * lw * w;
        h = ar * (sig - ar) * lw * w;
        break;
      }
      case 11: {  // cross entropy
        const double z = 1.0f / (1.0f + exp(-s));
        g = (z - y) * w;
        h = z * (1.0f - z) * w;
        break;
      }
      case 12: {  // cross entropy lambda
        if (!ga.weights) {
          const double z = 1.0f / (1.0f + exp(-s));
          g = z - y;
          h = z * (1.0f - z);
        } else {
          const double epf = exp(s);
          const double hhat = log(1.0f + epf);
          const double z = 1.0f - exp(-w * hhat);
          const double enf = 1.0f / epf;
          g = (1.0f - y / z) * w / (1.0f + enf);
          const double c = 1.0f / (1.0f - z);
          double d = 1.0f + epf;
          const double aa = w * epf / (d * d);
          d = c - 1.0f;
          const double b = (c / (d * d)) * (1.0f + w * epf - c);
          h = aa * (1.0f + y * b);
        }
        break;
      }
      case 13: {  // multiclass softmax (all classes of row i)
        const int K = ga.num_class;
        double mx = -INFINITY;
        for (int k = 0; k < K; ++k) mx = fmax(mx, ga.score[k * n + i]);
        double den = 0.0;
        for (int k = 0; k < K; ++k) den += exp(ga.score[k * n + i] - mx);
        const int lab = static_cast<int>(y);
        for (int k = 0; k < K; ++k) {
          const double pk = exp(ga.score[k * n + i] - mx) / den;
          ga.grad[k * n + i] = static_cast<float>((lab == k ? pk - 1.0f : pk) * w);
          ga.hess[k * n + i] = static_cast<float>(ga.p0 * pk * (1.0f - pk) * w);
        }
        continue;
      }
      default:
        break;
    }
    ga.grad[i] = static_cast<float>(g);
    ga.hess[i] = static_cast<float>(h);
  }
}

void Gradients(const GradArgs& g, hipStream_t s) {
  const int blocks = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>((g.num_data + 255) / 256, 8 * g_num_cus)));
  hipLaunchKernelGGL(k_gradients, dim3(blocks), dim3(256), 0, s, g);
}

void SetNumCUs(int n) { g_num_cus = n > 0 ? n : 256; }

}  // namespace dev
}  // namespace lgbm_amd
