// Best-split search on device histograms (reference src/treelearner/feature_histogram.hpp:
// FindBestThresholdSequentially, FuncForNumricalL3, FixHistogram; serial_tree_learner.cpp
// FindBestSplitsFromHistograms).
//
// Grid (num_features, 2 leaves), one 64-wide wave per workgroup.  A wave materialises its
// feature's histogram in the leaf's pool slot (the built child copies the step buffer, its
// sibling subtracts it from the parent slot -- exact in int64), then evaluates every
// threshold of the forward / reverse scans in parallel (wave prefix sums) with the
// reference's missing-value handling, min_data / min_hessian filters, hessian-estimated
// counts, L1 / max_delta_step / path smoothing / monotone constraints.  Ties keep the
// threshold the sequential scan would keep.  Per-feature results go to feat_best; the
// last wave of a leaf to arrive (atomic ticket) picks the leaf's best split.
#include "device_common.h"

namespace lgbm_amd {
namespace dev {

namespace {

struct Cand {
  double gain;
  int thr;
  double lg, lh;
  int lc;
};

// ties: reverse scan keeps the highest threshold (first met scanning down), forward the lowest
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

// a feature's dequantised histogram with its most-frequent bin restored (FixHistogram)
struct HistView {
  const long long* h;
  double inv_g, inv_h;
  int fix_t;  // bin whose value is reconstructed from the leaf totals (-1: none)
  double fix_g, fix_h;
  __device__ __forceinline__ double G(int t) const {
    return t == fix_t ? fix_g : static_cast<double>(h[2 * t]) * inv_g;
  }
  __device__ __forceinline__ double H(int t) const {
    return t == fix_t ? fix_h : static_cast<double>(h[2 * t + 1]) * inv_h;
  }
};

// one numerical scan of one feature by one wave
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
      const double gain = SplitGain(lg, lh, rg, rh, p.lambda_l2, p, L.c, static_cast<int8_t>(mono), lc, rc,
                                    L.parent_out);
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
      const double gain = SplitGain(xg, xh, rg, rh, p.lambda_l2, p, L.c, static_cast<int8_t>(mono), xc, rc,
                                    L.parent_out);
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

__device__ void FindNumericalWave(const Feature& F, const long long* h, double inv_g, double inv_h,
                                  const LeafCtx& L, const SplitParams& p, int depth, double mono_penalty,
                                  FeatureBest* out) {
  const int nb = F.num_bin - F.offset;
  HistView hv;
  hv.h = h;
  hv.inv_g = inv_g;
  hv.inv_h = inv_h;
  hv.fix_t = -1;
  hv.fix_g = hv.fix_h = 0.0;
  if (F.mfb > 0) {
    // FixHistogram: the most frequent bin is not accumulated; rebuild it from the leaf totals
    double sg = 0.0, sh = 0.0;
    const int lane = threadIdx.x & 63;
    for (int t = lane; t < nb; t += 64) {
      if (t == F.mfb) continue;
      sg += static_cast<double>(h[2 * t]) * inv_g;
      sh += static_cast<double>(h[2 * t + 1]) * inv_h;
    }
    sg = WaveSum(sg);
    sh = WaveSum(sh);
    hv.fix_t = F.mfb;
    hv.fix_g = L.sg - sg;
    hv.fix_h = (L.sh - 2 * kEpsilon) - sh;
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
__global__ __launch_bounds__(kWave) void k_find(KArgs a) {
  const int f = blockIdx.x;
  const int side = blockIdx.y;
  const int lane = threadIdx.x;
  const Feature F = a.feat[f];
  const int nb2 = 2 * (F.num_bin - F.offset);
  int parity = 0, leaf = 0;
  bool packed = false;
  if (!ROOT) {
    const Step* st = a.st;
    if (st->done) return;
    parity = st->step & 1;
    packed = st->hist_packed != 0;
    // zero this feature's bins (pair and packed layouts) of the buffer the next step uses
    if (side == 0) {
      long long* nxt = StepScratch(a, parity + 1);
      for (int i = lane; i < nb2; i += kWave) nxt[2 * F.hist_offset + i] = 0;
      for (int i = lane; i < nb2 / 2; i += kWave) nxt[F.hist_offset + i] = 0;
    }
    if (st->skip_find) return;
    leaf = side == 0 ? st->smaller : st->larger;
  }
  const SplitParams& p = a.p.sp;
  LeafCtx L;
  int depth, slot;
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
    if (f == 0 && lane == 0) {
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

  FeatureBest o;
  o.gain = -INFINITY;
  o.feature = f;
  o.real_feature = F.real_index;
  o.thr = 0;
  o.default_left = 1;
  o.lc = o.rc = 0;
  o.mono = 0;
  o.pad = 0;
  o.lg = o.lh = o.rg = o.rh = o.lo = o.ro = 0.0;
  if (a.tree_mask[f] && !F.is_cat) {
    const int nh = 2 * a.p.total_bins;
    long long* dst = a.hist + static_cast<size_t>(slot) * nh + 2 * F.hist_offset;
    if (packed) {
      // (g | h) packed words: g = arithmetic high half, h = low half
      const unsigned long long* srcp =
          reinterpret_cast<const unsigned long long*>(StepScratch(a, parity)) + F.hist_offset;
      const int nb = nb2 / 2;
      for (int i = lane; i < nb; i += kWave) {
        const unsigned long long v = srcp[i];
        const long long g = static_cast<long long>(v) >> 32;
        const long long h = static_cast<long long>(v & 0xffffffffull);
        if (side == 0) {
          dst[2 * i] = g;
          dst[2 * i + 1] = h;
        } else {
          dst[2 * i] -= g;
          dst[2 * i + 1] -= h;
        }
      }
    } else {
      const long long* src = StepScratch(a, parity) + 2 * F.hist_offset;
      if (side == 0) {
        for (int i = lane; i < nb2; i += kWave) dst[i] = src[i];
      } else {
        for (int i = lane; i < nb2; i += kWave) dst[i] -= src[i];
      }
    }
    __syncthreads();  // the wave's own stores become visible to all its lanes
    FindNumericalWave(F, dst, a.scales[2], a.scales[3], L, p, depth, a.p.monotone_penalty, &o);
  } else {
    o.feature = -1;
  }
  FeatureBest* fb = a.feat_best + side * a.p.num_features;
  if (lane == 0) fb[f] = o;
  // arrival ticket: the last wave of this leaf reduces the per-feature results
  __shared__ int last;
  if (lane == 0) {
    __threadfence();
    const int t = atomicAdd(&a.tickets[side], 1);
    last = (t == a.p.num_features - 1) ? 1 : 0;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  int bi = -1;
  double bg = -INFINITY;
  int brf = -1;
  for (int i = lane; i < a.p.num_features; i += kWave) {
    const FeatureBest& c = fb[i];
    if (c.feature >= 0 && SplitBetter(c.gain, c.real_feature, bg, brf)) {
      bg = c.gain;
      brf = c.real_feature;
      bi = i;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const double og = __shfl_xor(bg, off, kWave);
    const int orf = __shfl_xor(brf, off, kWave);
    const int oi = __shfl_xor(bi, off, kWave);
    if (oi >= 0 && (bi < 0 || SplitBetter(og, orf, bg, brf))) {
      bg = og;
      brf = orf;
      bi = oi;
    }
  }
  if (lane == 0) {
    a.tickets[side] = 0;
    DeviceSplit& d = a.best[leaf];
    if (bi < 0 || fb[bi].gain == -INFINITY) {
      d.gain = -INFINITY;
      d.feature = -1;
      d.real_feature = -1;
    } else {
      const FeatureBest b = fb[bi];
      d.gain = b.gain;
      d.feature = b.feature;
      d.real_feature = b.real_feature;
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

void FindRoot(const KArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_find<true>, dim3(a.p.num_features, 1), dim3(kWave), 0, s, a);
}
void FindStep(const KArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_find<false>, dim3(a.p.num_features, 2), dim3(kWave), 0, s, a);
}

}  // namespace dev
}  // namespace lgbm_amd
