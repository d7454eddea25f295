// Best-split search on device histograms (reference src/treelearner/feature_histogram.hpp:
// FindBestThresholdSequentially, FuncForNumricalL3, FixHistogram; serial_tree_learner.cpp
// FindBestSplitsFromHistograms).
//
// k_find: grid (num_features, 2 leaves), one 256-thread workgroup per (feature, leaf).  It
// materialises the feature's histogram in the leaf's pool slot (the smaller child takes
// the step's reduced histogram -- or sums the few partials of a small leaf itself -- the
// larger one subtracts it from the parent slot, exact in int64), stages it dequantised in
// LDS, then evaluates every threshold of the forward / reverse scans in parallel
// (workgroup prefix sums) with the reference's missing-value handling,
// min_data / min_hessian filters, hessian-estimated counts, L1 / max_delta_step / path
// smoothing / monotone constraints.  Ties keep the threshold the sequential scan would
// keep.  Per-feature results go to feat_best; the next partition kernel picks from them.
#include <type_traits>

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

constexpr int kNoRandThr = -(1 << 30);  // ScanNumericalBlock: every threshold (no extra_trees draw)

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

// block-wide scans / reductions of the split scan (kFindThreads threads); every thread
// calls them, results are returned to every thread
struct BlockScratch {
  double d[2][kFindThreads / kWave];
  int i[kFindThreads / kWave];
  Cand c[kFindThreads / kWave];
};
constexpr int kFindWaves = kFindThreads / kWave;

__device__ __forceinline__ void BlockScan3(double& a, double& b, int& c, bool suffix, BlockScratch* sc) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  a = suffix ? WaveSuffixIncl(a) : WavePrefixIncl(a);
  b = suffix ? WaveSuffixIncl(b) : WavePrefixIncl(b);
  c = suffix ? WaveSuffixIncl(c) : WavePrefixIncl(c);
  if (lane == (suffix ? 0 : 63)) {
    sc->d[0][w] = a;
    sc->d[1][w] = b;
    sc->i[w] = c;
  }
  __syncthreads();
  double oa = 0.0, ob = 0.0;
  int oc = 0;
#pragma unroll
  for (int j = 0; j < kFindWaves; ++j) {
    if (suffix ? j > w : j < w) {
      oa += sc->d[0][j];
      ob += sc->d[1][j];
      oc += sc->i[j];
    }
  }
  __syncthreads();
  a += oa;
  b += ob;
  c += oc;
}

__device__ __forceinline__ void BlockSum3(double& a, double& b, int& c, BlockScratch* sc) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  a = WaveSum(a);
  b = WaveSum(b);
  c = WaveSum(c);
  if (lane == 0) {
    sc->d[0][w] = a;
    sc->d[1][w] = b;
    sc->i[w] = c;
  }
  __syncthreads();
  a = b = 0.0;
  c = 0;
#pragma unroll
  for (int j = 0; j < kFindWaves; ++j) {  // fixed order: identical on every thread and run
    a += sc->d[0][j];
    b += sc->d[1][j];
    c += sc->i[j];
  }
  __syncthreads();
}

__device__ __forceinline__ bool BlockAny(bool v, BlockScratch* sc) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bool wv = __any(v);
  if (lane == 0) sc->i[w] = wv ? 1 : 0;
  __syncthreads();
  int r = 0;
#pragma unroll
  for (int j = 0; j < kFindWaves; ++j) r |= sc->i[j];
  __syncthreads();
  return r != 0;
}

__device__ __forceinline__ Cand BlockBestCand(Cand c, bool reverse, BlockScratch* sc) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  c = WaveBestCand(c, reverse);
  if (lane == 0) sc->c[w] = c;
  __syncthreads();
  Cand b = sc->c[0];
#pragma unroll
  for (int j = 1; j < kFindWaves; ++j) {
    if (CandBetter(sc->c[j], b, reverse)) b = sc->c[j];
  }
  __syncthreads();
  return b;
}

// a feature's dequantised histogram with its most-frequent bin restored (FixHistogram);
// bins come from LDS (staged by the wave) or, for very wide features, from the int64 slot
struct HistView {
  const double* lg;
  const double* lh;
  const long long* h;
  double inv_g, inv_h;
  int fix_t;  // bin whose value is reconstructed from the leaf totals (-1: none)
  double fix_g, fix_h;
  __device__ __forceinline__ double RawG(int t) const {
    return lg ? lg[t] : static_cast<double>(h[2 * t]) * inv_g;
  }
  __device__ __forceinline__ double RawH(int t) const {
    return lh ? lh[t] : static_cast<double>(h[2 * t + 1]) * inv_h;
  }
  __device__ __forceinline__ double G(int t) const { return t == fix_t ? fix_g : RawG(t); }
  __device__ __forceinline__ double H(int t) const { return t == fix_t ? fix_h : RawH(t); }
};

// one numerical scan of one feature by one workgroup (each thread owns K consecutive bins)
__device__ Cand ScanNumericalBlock(const HistView& hv, int nb, int offset, int default_bin, bool reverse,
                                   bool skip_def, bool na, const LeafCtx& L, const SplitParams& p, int mono,
                                   bool* splittable, BlockScratch* sc, int rthr) {
  const int tid = threadIdx.x;
  const int K = (nb + kFindThreads - 1) / kFindThreads;
  const int b0 = tid * K;
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
    double ig = tg, ih = th;
    int ic = tc;
    BlockScan3(ig, ih, ic, true, sc);
    double rg = ig - tg, rh = ih - th;  // exclusive suffix (bins above this thread's)
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
      if (rthr != kNoRandThr && t - 1 + offset != rthr) continue;  // extra_trees
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
      BlockSum3(ag, ah, ac, sc);
      lg0 = L.sg - ag;
      lh0 = L.sh - kEpsilon - ah;
      lc0 = L.n - ac;
    }
    double ig = tg, ih = th;
    int ic = tc;
    BlockScan3(ig, ih, ic, false, sc);
    double lg = lg0 + (ig - tg), lh = lh0 + (ih - th);
    int lc = lc0 + (ic - tc);
    auto eval = [&](int t, double xg, double xh, int xc) {
      if (xc < min_n || xh < min_h) return;
      const int rc = L.n - xc;
      if (rc < min_n) return;
      const double rh = L.sh - xh;
      if (rh < min_h) return;
      const double rg = L.sg - xg;
      if (rthr != kNoRandThr && t + offset != rthr) return;  // extra_trees
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
    if (minus_one && tid == 0 && !(skip_def && offset - 1 == default_bin)) eval(-1, lg0, lh0, lc0);
    for (int t = b0; t < b1; ++t) {
      if (!acc(t)) continue;
      const double g = hv.G(t), hh = hv.H(t);
      lg += g;
      lh += hh;
      lc += RoundIntD(hh * L.cnt_factor);
      eval(t, lg, lh, lc);
    }
  }
  if (BlockAny(any, sc)) *splittable = true;
  return BlockBestCand(best, reverse, sc);
}

// returns whether any threshold was valid (the host's is_splittable)
__device__ bool FindNumericalBlock(const Feature& F, HistView hv, const LeafCtx& L, const SplitParams& p, int depth,
                                   double mono_penalty, FeatureBest* out, BlockScratch* sc, int rthr) {
  const int nb = F.num_bin - F.offset;
  hv.fix_t = -1;
  hv.fix_g = hv.fix_h = 0.0;
  if (F.mfb > 0) {
    // FixHistogram: the most frequent bin is not accumulated; rebuild it from the leaf totals
    double sg = 0.0, sh = 0.0;
    int unused = 0;
    for (int t = threadIdx.x; t < nb; t += kFindThreads) {
      if (t == F.mfb) continue;
      sg += hv.RawG(t);
      sh += hv.RawH(t);
    }
    BlockSum3(sg, sh, unused, sc);
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
      apply(ScanNumericalBlock(hv, nb, F.offset, F.default_bin, true, true, false, L, p, F.monotone, &splittable, sc, rthr), true);
      apply(ScanNumericalBlock(hv, nb, F.offset, F.default_bin, false, true, false, L, p, F.monotone, &splittable, sc, rthr), false);
    } else {
      apply(ScanNumericalBlock(hv, nb, F.offset, F.default_bin, true, false, true, L, p, F.monotone, &splittable, sc, rthr), true);
      apply(ScanNumericalBlock(hv, nb, F.offset, F.default_bin, false, false, true, L, p, F.monotone, &splittable, sc, rthr), false);
    }
  } else {
    apply(ScanNumericalBlock(hv, nb, F.offset, F.default_bin, true, false, false, L, p, F.monotone, &splittable, sc, rthr), true);
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
  return splittable;
}

// LDS of the categorical scan: per-bin ctr and the stable ctr order
constexpr int kCatPar = 128;  // prefix positions per direction scanned with the parallel path

struct CatScratch {
  double ctr[kFindMaxCatBins];
  int sorted[kFindMaxCatBins];
  int used_bin;
  // parallel prefix scan: per direction and position, the bin's then the cumulative
  // (g, h, count) and the split gain there
  double pg[2][kCatPar], ph[2][kCatPar], gain[2][kCatPar];
  int pc[2][kCatPar], cnt[2][kCatPar];
};

// categorical split of one feature (reference FindBestThresholdCategoricalInner,
// feature_histogram.hpp:277-513): one-vs-rest for few categories (parallel over the bins),
// otherwise the bins with enough data sorted by g / (h + cat_smooth) -- a stable rank
// computed in parallel -- and the sequential prefix scan from both ends (<= 2 x
// max_cat_threshold steps, thread 0) with the min_data_per_group rules.
// returns splittable (meaningful in thread 0)
__device__ __forceinline__ bool FindCategoricalBlock(const Feature& F, HistView hv, const LeafCtx& L, const SplitParams& p,
                                     FeatureBest* out, uint32_t* cat_out, BlockScratch* sc, CatScratch* cs) {
  const int tid = threadIdx.x;
  const int nb = F.num_bin - F.offset;
  hv.fix_t = -1;
  hv.fix_g = hv.fix_h = 0.0;
  if (F.mfb > 0) {  // FixHistogram
    double sg = 0.0, sh = 0.0;
    int unused = 0;
    for (int t = tid; t < nb; t += kFindThreads) {
      if (t == F.mfb) continue;
      sg += hv.RawG(t);
      sh += hv.RawH(t);
    }
    BlockSum3(sg, sh, unused, sc);
    hv.fix_t = F.mfb;
    hv.fix_g = L.sg - sg;
    hv.fix_h = (L.sh - 2 * kEpsilon) - sh;
  }
  double gain_shift;
  if (p.use_smoothing) {
    gain_shift = LeafGainGivenOutput(L.sg, L.sh, p.lambda_l1, p.lambda_l2, L.parent_out, p.use_l1);
  } else {
    gain_shift = LeafGain(L.sg, L.sh, p.lambda_l1, p.lambda_l2, p.max_delta_step, 0, L.n, 0, p.use_l1,
                          p.use_max_output, 0);
  }
  const double min_gain_shift = gain_shift + p.min_gain_to_split;
  const int offset = F.offset;
  const int bin_start = 1 - offset, bin_end = F.num_bin - offset;
  const bool onehot = F.num_bin <= p.max_cat_to_onehot;
  const double min_h = p.min_sum_hessian_in_leaf;
  const int min_n = p.min_data_in_leaf;
  out->gain = -INFINITY;
  out->default_left = 0;
  out->mono = 0;
  out->thr = 0;
  out->ncat = 0;
  double l2 = p.lambda_l2;
  bool splittable = false;
  Cand best;
  best.gain = -INFINITY;
  best.thr = 0x7fffffff;
  best.lg = best.lh = 0.0;
  best.lc = 0;
  int best_dir = 1;
  if (onehot) {
    bool any = false;
    for (int t = bin_start + tid; t < bin_end; t += kFindThreads) {
      const double g = hv.G(t), hh = hv.H(t);
      const int cnt = RoundIntD(hh * L.cnt_factor);
      if (cnt < min_n || hh < min_h) continue;
      const int other = L.n - cnt;
      if (other < min_n) continue;
      const double oh = L.sh - hh - kEpsilon;
      if (oh < min_h) continue;
      const double og = L.sg - g;
      const double gain = SplitGain(og, oh, g, hh + kEpsilon, l2, p, L.c, 0, other, cnt, L.parent_out);
      if (gain <= min_gain_shift) continue;
      any = true;
      if (gain > best.gain || (gain == best.gain && t < best.thr)) {
        best.gain = gain;
        best.thr = t;
        best.lg = g;
        best.lh = hh + kEpsilon;
        best.lc = cnt;
      }
    }
    splittable = BlockAny(any, sc);
    best = BlockBestCand(best, false, sc);
  } else {
    l2 += p.cat_l2;
    // candidates and their ctr; non-candidates get NaN (never ranked)
    for (int t = bin_start + tid; t < bin_end; t += kFindThreads) {
      const double hh = hv.H(t);
      const bool cand = static_cast<double>(RoundIntD(hh * L.cnt_factor)) >= p.cat_smooth;
      cs->ctr[t] = cand ? hv.G(t) / (hh + p.cat_smooth) : NAN;
    }
    __syncthreads();
    // stable rank among the candidates (std::stable_sort by ctr ascending)
    int ncand = 0;
    for (int t = bin_start + tid; t < bin_end; t += kFindThreads) {
      const double c = cs->ctr[t];
      if (c != c) continue;
      ++ncand;
      int r = 0;
      for (int u = bin_start; u < bin_end; ++u) {
        const double cu = cs->ctr[u];
        r += (cu < c) | ((cu == c) & (u < t));
      }
      cs->sorted[r] = t;
    }
    double d0 = 0.0, d1 = 0.0;
    BlockSum3(d0, d1, ncand, sc);
    const int used_bin = ncand;
    const int max_num_cat = min(p.max_cat_threshold, (used_bin + 1) / 2);
    const int npos = min(used_bin, max_num_cat);
    if (npos <= kCatPar) {
      // (1) every thread stages one position's bin statistics, (2) one thread per direction
      // accumulates the prefix sums in the sequential order (bit-identical sums), (3) every
      // thread evaluates the split gain of one position, (4) thread 0 applies the
      // order-dependent min_data_per_group rules over the precomputed gains
      for (int idx = tid; idx < 2 * npos; idx += kFindThreads) {
        const int o = idx / npos, i = idx % npos;
        const int t = cs->sorted[o == 0 ? i : used_bin - 1 - i];
        const double hh = hv.H(t);
        cs->pg[o][i] = hv.G(t);
        cs->ph[o][i] = hh;
        cs->cnt[o][i] = RoundIntD(hh * L.cnt_factor);
      }
      __syncthreads();
      if (tid < 2) {
        double lg = 0.0, lh = kEpsilon;
        int lc = 0;
        for (int i = 0; i < npos; ++i) {
          lg += cs->pg[tid][i];
          lh += cs->ph[tid][i];
          lc += cs->cnt[tid][i];
          cs->pg[tid][i] = lg;
          cs->ph[tid][i] = lh;
          cs->pc[tid][i] = lc;
        }
      }
      __syncthreads();
      for (int idx = tid; idx < 2 * npos; idx += kFindThreads) {
        const int o = idx / npos, i = idx % npos;
        const double lg = cs->pg[o][i], lh = cs->ph[o][i];
        const int lc = cs->pc[o][i];
        cs->gain[o][i] = SplitGain(lg, lh, L.sg - lg, L.sh - lh, l2, p, L.c, 0, lc, L.n - lc, L.parent_out);
      }
      __syncthreads();
      if (tid == 0) {
        for (int o = 0; o < 2; ++o) {
          int cnt_group = 0;
          for (int i = 0; i < npos; ++i) {
            const int lc = cs->pc[o][i];
            const double lh = cs->ph[o][i];
            cnt_group += cs->cnt[o][i];
            if (lc < min_n || lh < min_h) continue;
            const int rc = L.n - lc;
            if (rc < min_n || rc < p.min_data_per_group) break;
            if (L.sh - lh < min_h) break;
            if (cnt_group < p.min_data_per_group) continue;
            cnt_group = 0;
            const double gain = cs->gain[o][i];
            if (gain <= min_gain_shift) continue;
            splittable = true;
            if (gain > best.gain) {
              best.gain = gain;
              best.thr = i;
              best.lg = cs->pg[o][i];
              best.lh = lh;
              best.lc = lc;
              best_dir = o == 0 ? 1 : -1;
            }
          }
        }
        cs->used_bin = used_bin;
      }
    } else if (tid == 0) {
      for (int o = 0; o < 2; ++o) {
        const int dir = o == 0 ? 1 : -1;
        int pos = o == 0 ? 0 : used_bin - 1;
        int cnt_group = 0, lc = 0;
        double lg = 0.0, lh = kEpsilon;
        for (int i = 0; i < used_bin && i < max_num_cat; ++i) {
          const int t = cs->sorted[pos];
          pos += dir;
          const double g = hv.G(t), hh = hv.H(t);
          const int cnt = RoundIntD(hh * L.cnt_factor);
          lg += g;
          lh += hh;
          lc += cnt;
          cnt_group += cnt;
          if (lc < min_n || lh < min_h) continue;
          const int rc = L.n - lc;
          if (rc < min_n || rc < p.min_data_per_group) break;
          const double rh = L.sh - lh;
          if (rh < min_h) break;
          if (cnt_group < p.min_data_per_group) continue;
          cnt_group = 0;
          const double rg = L.sg - lg;
          const double gain = SplitGain(lg, lh, rg, rh, l2, p, L.c, 0, lc, rc, L.parent_out);
          if (gain <= min_gain_shift) continue;
          splittable = true;
          if (gain > best.gain) {
            best.gain = gain;
            best.thr = i;
            best.lg = lg;
            best.lh = lh;
            best.lc = lc;
            best_dir = dir;
          }
        }
      }
      cs->used_bin = used_bin;
    }
  }
  if (tid != 0 || !splittable) return splittable;
  out->lo = LeafOutputConstrained(best.lg, best.lh, l2, p, L.c, best.lc, L.parent_out);
  out->lc = best.lc;
  out->lg = best.lg;
  out->lh = best.lh - kEpsilon;
  out->ro = LeafOutputConstrained(L.sg - best.lg, L.sh - best.lh, l2, p, L.c, L.n - best.lc, L.parent_out);
  out->rc = L.n - best.lc;
  out->rg = L.sg - best.lg;
  out->rh = L.sh - best.lh - kEpsilon;
  out->gain = (best.gain - min_gain_shift) * F.penalty;
  for (int w = 0; w < kMaxCatWords; ++w) cat_out[w] = 0u;
  if (onehot) {
    const int b = best.thr + offset;
    cat_out[b >> 5] |= 1u << (b & 31);
    out->ncat = 1;
  } else {
    const int k = best.thr + 1;
    for (int i = 0; i < k; ++i) {
      const int b = (best_dir == 1 ? cs->sorted[i] : cs->sorted[cs->used_bin - 1 - i]) + offset;
      cat_out[b >> 5] |= 1u << (b & 31);
    }
    out->ncat = k;
  }
  return true;
}

}  // namespace

// KIND 0: every feature of a dataset without categorical features; 1: the numerical
// features of a dataset with some (the categorical ones only get their bookkeeping here);
// 2: the categorical features (grid over KArgs::cat_list).  The categorical scan has its
// own register / LDS footprint, so it runs in a kernel of its own (inlined: a called
// function costs ~700 B/lane of stack and ran ~10x slower).
// extra_trees: Random::Step31 applied k times (x -> 214013 x + 2531011), by squaring the map
__device__ __forceinline__ uint32_t LcgSkip(uint32_t x, int k) {
  uint32_t am = 214013u, cm = 2531011u, ar = 1u, cr = 0u;
  while (k > 0) {
    if (k & 1) {
      ar = am * ar;
      cr = am * cr + cm;
    }
    cm = am * cm + cm;
    am = am * am;
    k >>= 1;
  }
  return ar * x + cr;
}

// extra_trees: whether the host learner scans f at node mi (the feature is used by the tree,
// its parent could split on it, the node samples it and its constraints allow it) and so
// draws FeatureMeta::rand.NextInt(0, num_bin - 2) (split_finder.cpp FindNumerical)
__device__ __forceinline__ int XtDraws(const KArgs& a, const Feature& F, int f, int mi, uint32_t icmask, bool gate) {
  if (!gate || F.num_bin - 2 <= 0) return 0;
  if (a.node_mask != nullptr && !a.node_mask[static_cast<size_t>(mi) * a.p.num_features + f]) return 0;
  if (a.feat_icmask != nullptr && (icmask & a.feat_icmask[f]) == 0u) return 0;
  return 1;
}

template <bool ROOT, int KIND>
__global__ __launch_bounds__(kFindThreads) void k_find(KArgs a) {
  constexpr bool CAT = KIND == 2;
  extern __shared__ double s_bins[];  // [2][max_feature_bins] dequantised (g, h), if they fit
  __shared__ BlockScratch sc;
  __shared__ typename std::conditional<CAT, CatScratch, int>::type cat_sc;
  __shared__ unsigned long long s_red[2 * kFindThreads];  // direct partial sums of narrow features
  const long long t_entry = wall_clock64();
  const int f = CAT ? a.cat_list[blockIdx.x] : static_cast<int>(blockIdx.x);
  const int side = blockIdx.y;
  const int tid = threadIdx.x;
  // ---- independent loads first (one round trip): the feature, its mask, the scales and the
  // Step record (read before it is tested)
  const Feature F = a.feat[f];
  const int8_t tree_used = a.tree_mask[f];
  int8_t used = tree_used;  // evaluated at this node (feature_fraction_bynode)
  if (a.node_mask != nullptr) {
    const int mi = ROOT ? 0 : a.st->bynode_base + side;
    used = used && a.node_mask[static_cast<size_t>(mi) * a.p.num_features + f];
  }
  const int8_t parent_ok = ROOT ? 1 : a.parent_flags[f];
  const double ig = a.scales[2], ih = a.scales[3];
  const Step* st = a.st;
  int done = 0, skip = 0, s = 0, s_count = 0;
  ChildStats cl;
  if (!ROOT) {
    done = st->done;
    skip = st->skip_find;
    s = st->cs.s;
    s_count = st->s_count;
    cl = st->child[side];  // written with the histogram (StepBookkeeping)
  }
  // extra_trees: per feature and node, the smaller child draws before the larger one
  // (SerialTreeLearner::FindBestSplitsFromHistograms); draw k of the tree is the base state
  // stepped k times.  The smaller child's workgroup appends the step's count row.
  int xt_thr = kNoRandThr;
  if (a.xt_base != nullptr && (ROOT || !done)) {
    const int nf = a.p.num_features;
    const int prev = ROOT ? 0 : a.xt_cum[static_cast<size_t>(s) * nf + f];
    const bool gate = tree_used && parent_ok && !skip;
    const int d0 = ROOT ? XtDraws(a, F, f, 0, 0xffffffffu, gate)
                        : XtDraws(a, F, f, st->bynode_base, st->child[0].icmask, gate);
    const int d1 = ROOT ? 0 : XtDraws(a, F, f, st->bynode_base + 1, st->child[1].icmask, gate);
    if (side == 0 && tid == 0) a.xt_cum[static_cast<size_t>(ROOT ? 0 : s + 1) * nf + f] = prev + d0 + d1;
    xt_thr = 0;  // num_bin <= 2: no draw, threshold 0 only
    if (side == 0 ? d0 : d1) {
      const uint32_t x = LcgSkip(a.xt_base[f], prev + (side == 1 ? d0 : 0) + 1);
      xt_thr = static_cast<int>(x & 0x7fffffffu) % (F.num_bin - 2);
    }
  }
  const int nbf = F.num_bin - F.offset;
  const int nb2 = 2 * nbf;
  int parity = 0, nblk_direct = -1;
  if (!ROOT) {
    if (done) return;
    if (!CAT && f == 0 && side == 0 && tid == 0) {
      // the partition cursors were final for the histogram kernel: reset for the next split
      // (the reduce kernel, not launched for late splits, used to do it)
      a.st->cur_left = 0;
      a.st->cur_right = 0;
    }
    parity = (s + 1) & 1;
    // zero this feature's bins of the buffer the next step reduces into
    if (!CAT && side == 0) {
      long long* nxt = StepScratch(a, parity + 1);
      for (int i = tid; i < nb2; i += kFindThreads) nxt[2 * F.hist_offset + i] = 0;
    }
    if (skip) return;
    KTraceAt(a, s, kTrFindEntry, t_entry);
    const int nblk = HistBlocksFor(s_count, a.hist_max_blocks, a.hist_rows_cap);
    if (DirectPartials(a, nblk, s)) nblk_direct = nblk;
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
    if (f == 0 && tid == 0 && KIND != 2) {
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
    L.sg = cl.sum_g;
    L.sh = cl.sum_h + 2 * kEpsilon;
    L.n = cl.global_count;
    L.parent_out = cl.output;
    L.c.min = cl.cmin;
    L.c.max = cl.cmax;
    depth = cl.depth;
    slot = cl.slot;
  }
  if (KIND == 1 && F.is_cat) return;  // the categorical kernel scans it
  // interaction constraints: like a sampled-out feature, a disallowed one is not evaluated
  // here but keeps its histogram and its splittable flag
  if (a.feat_icmask != nullptr && ((ROOT ? 0xffffffffu : cl.icmask) & a.feat_icmask[f]) == 0u) used = 0;
  int8_t* flags = a.splittable + static_cast<size_t>(ROOT ? a.leaves[0].frow : cl.frow) * a.p.num_features;
  if (tree_used && !parent_ok) {
    // the parent could not split on f: neither child evaluates it, the smaller child's row
    // says so and the larger child keeps the parent's row (SerialTreeLearner::FindBestSplits)
    if (side == 0 && tid == 0) flags[f] = 0;
    if (tid == 0) {
      FeatureBest o;
      o.gain = -INFINITY;
      o.feature = -1;
      a.feat_best[side * a.p.num_features + f] = o;
    }
    return;
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
  o.ncat = 0;
  o.lg = o.lh = o.rg = o.rh = o.lo = o.ro = 0.0;
  // a sampled-out feature (bynode) still materialises its histogram: descendants subtract it
  if (tree_used && (!F.is_cat || F.num_bin <= kFindMaxCatBins)) {
    const int nh = 2 * a.p.total_bins;
    long long* dst = a.hist + static_cast<size_t>(slot) * nh + 2 * F.hist_offset;
    const long long* src = StepScratch(a, parity) + 2 * F.hist_offset;
    const unsigned long long* part = a.partials + F.hist_offset;
    const bool stage = a.p.max_feature_bins <= kFindLdsBins;
    double* sg = s_bins;
    double* sh = s_bins + (stage ? a.p.max_feature_bins : 0);
    // a feature with fewer bins than threads sums its direct partials with every thread:
    // kFindThreads / nbf threads per bin stride over the row blocks, then combine in LDS
    // (one thread per bin walking hundreds of partials would be a chain of round trips)
    const bool spread = nblk_direct > 1 && 2 * nbf <= kFindThreads;
    // the larger child's parent bins (first bin of each thread): loaded up front, so their
    // round trip overlaps the partial-sum loads instead of following them
    long long pg0 = 0, ph0 = 0;
    if (side == 1 && tid < nbf) {
      pg0 = dst[2 * tid];
      ph0 = dst[2 * tid + 1];
    }
    if (spread) {
      for (int j = tid; j < 2 * nbf; j += kFindThreads) s_red[j] = 0ull;
      __syncthreads();
      const int per = kFindThreads / nbf;
      const int i = tid % nbf, r = tid / nbf;
      if (r < per) {
        constexpr int kC = 8;
        long long g = 0, h = 0;
        for (int k0 = r; k0 < nblk_direct; k0 += per * kC) {
          unsigned long long v[kC];
#pragma unroll
          for (int c = 0; c < kC; ++c) {
            const int k = k0 + c * per;
            v[c] = k < nblk_direct ? part[static_cast<size_t>(k) * a.p.total_bins + i] : 0ull;
          }
#pragma unroll
          for (int c = 0; c < kC; ++c) {
            g += static_cast<long long>(v[c]) >> 32;
            h += static_cast<long long>(v[c] & 0xffffffffull);
          }
        }
        atomicAdd(&s_red[2 * i], static_cast<unsigned long long>(g));
        atomicAdd(&s_red[2 * i + 1], static_cast<unsigned long long>(h));
      }
      __syncthreads();
    }
    for (int i = tid; i < nbf; i += kFindThreads) {
      long long g = 0, h = 0;
      if (spread) {
        g = static_cast<long long>(s_red[2 * i]);
        h = static_cast<long long>(s_red[2 * i + 1]);
      } else if (nblk_direct >= 0) {
        // small leaf: sum the few per-workgroup partials here (k_hist_reduce skipped them)
        // chunks of kReduceChunk independent loads in flight
        for (int k0 = 0; k0 < nblk_direct; k0 += kReduceChunk) {
          unsigned long long v[kReduceChunk];
#pragma unroll
          for (int k = 0; k < kReduceChunk; ++k)
            v[k] = k0 + k < nblk_direct ? part[static_cast<size_t>(k0 + k) * a.p.total_bins + i] : 0ull;
#pragma unroll
          for (int k = 0; k < kReduceChunk; ++k) {
            g += static_cast<long long>(v[k]) >> 32;
            h += static_cast<long long>(v[k] & 0xffffffffull);
          }
        }
      } else {
        g = src[2 * i];
        h = src[2 * i + 1];
      }
      if (side == 1) {  // larger child = parent - smaller, in the parent's (now its) slot
        g = (i == tid ? pg0 : dst[2 * i]) - g;
        h = (i == tid ? ph0 : dst[2 * i + 1]) - h;
      }
      dst[2 * i] = g;
      dst[2 * i + 1] = h;
      if (stage) {
        sg[i] = static_cast<double>(g) * ig;
        sh[i] = static_cast<double>(h) * ih;
      }
    }
    __syncthreads();  // the workgroup's stores become visible to all its threads
    if (!ROOT) KTrace(a, s, kTrFindLoaded);
    if (!used) {
      if (tid == 0) {
        o.feature = -1;
        a.feat_best[side * a.p.num_features + f] = o;
      }
      return;
    }
    HistView hv;
    hv.lg = stage ? sg : nullptr;
    hv.lh = stage ? sh : nullptr;
    hv.h = dst;
    hv.inv_g = ig;
    hv.inv_h = ih;
    bool splittable;
    if constexpr (CAT) {
      splittable = FindCategoricalBlock(
          F, hv, L, p, &o, a.feat_cat + (static_cast<size_t>(side) * a.p.num_features + f) * kMaxCatWords, &sc,
          &cat_sc);
    } else {
      splittable = FindNumericalBlock(F, hv, L, p, depth, a.p.monotone_penalty, &o, &sc, xt_thr);
    }
    if (tid == 0) flags[f] = splittable ? 1 : 0;
    if (!ROOT) KTrace(a, s, kTrFindScanned);
  } else {
    o.feature = -1;
  }
  if (tid == 0) a.feat_best[side * a.p.num_features + f] = o;
  if (!ROOT) KTrace(a, s, kTrFindExit);
}

static size_t FindLds(const KArgs& a) {
  return a.p.max_feature_bins <= kFindLdsBins ? 2 * sizeof(double) * static_cast<size_t>(a.p.max_feature_bins) : 0;
}
void FindRoot(const KArgs& a, hipStream_t s) {
  if (a.p.has_cat) {
    hipLaunchKernelGGL((k_find<true, 1>), dim3(a.p.num_features, 1), dim3(kFindThreads), FindLds(a), s, a);
    hipLaunchKernelGGL((k_find<true, 2>), dim3(a.p.has_cat, 1), dim3(kFindThreads), FindLds(a), s, a);
  } else {
    hipLaunchKernelGGL((k_find<true, 0>), dim3(a.p.num_features, 1), dim3(kFindThreads), FindLds(a), s, a);
  }
}
void FindStep(const KArgs& a, hipStream_t s) {
  if (a.p.has_cat) {
    hipLaunchKernelGGL((k_find<false, 1>), dim3(a.p.num_features, 2), dim3(kFindThreads), FindLds(a), s, a);
    hipLaunchKernelGGL((k_find<false, 2>), dim3(a.p.has_cat, 2), dim3(kFindThreads), FindLds(a), s, a);
  } else {
    hipLaunchKernelGGL((k_find<false, 0>), dim3(a.p.num_features, 2), dim3(kFindThreads), FindLds(a), s, a);
  }
}

}  // namespace dev
}  // namespace lgbm_amd
