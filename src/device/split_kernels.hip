// Best-split search on device histograms (reference src/treelearner/feature_histogram.hpp:
// FindBestThresholdSequentially, FuncForNumricalL3, FixHistogram; serial_tree_learner.cpp
// FindBestSplitsFromHistograms).
//
// k_find: grid (num_features, 2 leaves), one 256-thread workgroup per (feature, leaf).  It
// materialises the feature's histogram in the leaf's pool slot -- the histogrammed child
// takes the step's reduced histogram (or sums the few partials of a small leaf itself), the
// other child subtracts it from the parent slot in place, exact in int64 -- stages it
// dequantised in LDS, then evaluates every threshold of the forward and reverse scans in
// parallel from ONE workgroup prefix scan (the reverse scan's right sums are the range total
// minus the prefix), with the reference's missing-value handling, min_data / min_hessian
// filters, hessian-estimated counts, L1 / max_delta_step / path smoothing / monotone
// constraints.  Ties keep the threshold the sequential scan would keep.  Per-feature results
// go to feat_best.  The last workgroup of the step to finish (a device-scope counter) then
// records the step and picks the next split (pick.h), so the next k_split starts from one
// small Step record.
#include <type_traits>

#include "pick.h"

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

// block-wide scans / reductions of the split scan (NT threads: kFindThreads, or one wave per
// workgroup for narrow features); every thread calls them, results are returned to every thread
template <int NT>
struct BlockScratch {
  double d[2][NT / kWave];
  int i[NT / kWave];
  Cand c[NT / kWave];
};

template <int NT>
__device__ __forceinline__ void BlockScan3(double& a, double& b, int& c, bool suffix, BlockScratch<NT>* sc) {
  constexpr int kFindWaves = NT / kWave;
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

template <int NT>
__device__ __forceinline__ void BlockSum3(double& a, double& b, int& c, BlockScratch<NT>* sc) {
  constexpr int kFindWaves = NT / kWave;
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

template <int NT>
__device__ __forceinline__ bool BlockAny(bool v, BlockScratch<NT>* sc) {
  constexpr int kFindWaves = NT / kWave;
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

template <int NT>
__device__ __forceinline__ Cand BlockBestCand(Cand c, bool reverse, BlockScratch<NT>* sc) {
  constexpr int kFindWaves = NT / kWave;
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

// block-wide exclusive prefix of (g, h, c) plus block totals of (g, h, c) and of three more
// sums (ag, ah: every stored bin; na*: the NaN bin) in one LDS round
struct ScanAcc {
  double g, h;
  int c;
  double ag, ah, ng, nh;
  int nc;
};
template <int NT>
struct ScanScratch {
  double d[6][NT / kWave];
  int i[2][NT / kWave];
};

template <int NT>
__device__ __forceinline__ void BlockScanNum(ScanAcc* v, ScanAcc* excl, ScanAcc* tot, ScanScratch<NT>* sc) {
  constexpr int kFindWaves = NT / kWave;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const double ig = WavePrefixIncl(v->g), ih = WavePrefixIncl(v->h);
  const int ic = WavePrefixIncl(v->c);
  const double ag = WaveSum(v->ag), ah = WaveSum(v->ah), ng = WaveSum(v->ng), nh = WaveSum(v->nh);
  const int nc = WaveSum(v->nc);
  if (lane == 63) {
    sc->d[0][w] = ig;
    sc->d[1][w] = ih;
    sc->i[0][w] = ic;
  }
  if (lane == 0) {
    sc->d[2][w] = ag;
    sc->d[3][w] = ah;
    sc->d[4][w] = ng;
    sc->d[5][w] = nh;
    sc->i[1][w] = nc;
  }
  __syncthreads();
  ScanAcc e = {0.0, 0.0, 0, 0.0, 0.0, 0.0, 0.0, 0};
  ScanAcc t = e;
#pragma unroll
  for (int j = 0; j < kFindWaves; ++j) {  // fixed order: identical on every thread and run
    if (j < w) {
      e.g += sc->d[0][j];
      e.h += sc->d[1][j];
      e.c += sc->i[0][j];
    }
    t.g += sc->d[0][j];
    t.h += sc->d[1][j];
    t.c += sc->i[0][j];
    t.ag += sc->d[2][j];
    t.ah += sc->d[3][j];
    t.ng += sc->d[4][j];
    t.nh += sc->d[5][j];
    t.nc += sc->i[1][j];
  }
  __syncthreads();
  e.g += ig - v->g;
  e.h += ih - v->h;
  e.c += ic - v->c;
  *excl = e;
  *tot = t;
}

// the best candidates of both scan directions and whether any threshold was valid, over
// the workgroup (reverse ties: higher threshold; forward ties: lower)
template <int NT>
__device__ __forceinline__ void BlockBestPair(Cand* rv, Cand* fw, bool* any, BlockScratch<NT>* sc, Cand* sc2) {
  constexpr int kFindWaves = NT / kWave;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  *rv = WaveBestCand(*rv, true);
  *fw = WaveBestCand(*fw, false);
  const bool wa = __any(*any);
  if (lane == 0) {
    sc->c[w] = *rv;
    sc2[w] = *fw;
    sc->i[w] = wa ? 1 : 0;
  }
  __syncthreads();
  Cand br = sc->c[0], bf = sc2[0];
  int an = sc->i[0];
#pragma unroll
  for (int j = 1; j < kFindWaves; ++j) {
    if (CandBetter(sc->c[j], br, true)) br = sc->c[j];
    if (CandBetter(sc2[j], bf, false)) bf = sc2[j];
    an |= sc->i[j];
  }
  __syncthreads();
  *rv = br;
  *fw = bf;
  *any = an != 0;
}

// split gain / leaf output: the plain formulas (no L1, max_delta_step, path smoothing or
// monotone constraints -- the reference's FuncForNumricalL3 with every flag off) or the
// general ones, chosen at compile time so the common case stays a few instructions
template <bool SIMPLE>
__device__ __forceinline__ double GainOf(double lg, double lh, double rg, double rh, double l2, const SplitParams& p,
                                         const ConstraintRange& c, int8_t mono, int lc, int rc, double parent_out) {
  if (SIMPLE) return (lg * lg) / (lh + l2) + (rg * rg) / (rh + l2);
  return SplitGain(lg, lh, rg, rh, l2, p, c, mono, lc, rc, parent_out);
}
template <bool SIMPLE>
__device__ __forceinline__ double OutputOf(double sg, double sh, double l2, const SplitParams& p,
                                           const ConstraintRange& c, int n, double parent_out) {
  if (SIMPLE) return -sg / (sh + l2);
  return LeafOutputConstrained(sg, sh, l2, p, c, n, parent_out);
}

// numerical split of one feature (FindBestThresholdSequentially, both directions and
// FixHistogram); returns whether any threshold was valid (the host's is_splittable).
// Every candidate -- reverse at t (right = bins t..t_start), forward at t (left = bins
// 0..t), and the forward "nothing stored on the left" start -- goes through one evaluation
// site (instruction footprint: these kernels run once per split on a cold I-cache).
template <bool SIMPLE, int NT>
__device__ bool FindNumericalBlock(const Feature& F, HistView hv, const LeafCtx& L, const SplitParams& p, int depth,
                                   double mono_penalty, FeatureBest* out, BlockScratch<NT>* sc, ScanScratch<NT>* ssc,
                                   Cand* sc2, int rthr) {
  const int tid = threadIdx.x;
  const int nb = F.num_bin - F.offset;
  const int offset = F.offset;
  const bool two = F.num_bin > 2 && F.missing_type != 0;  // reverse and forward scans
  const bool skip_def = two && F.missing_type == 1;
  const bool na = two && F.missing_type == 2;
  const int fix_t = F.mfb > 0 ? F.mfb : -1;  // most frequent bin: not accumulated, rebuilt from the totals
  const int def_t = skip_def ? F.default_bin - offset : -1;  // the default bin: in no scan
  const int K = (nb + NT - 1) / NT;
  const int b0 = tid * K;
  const int b1 = min(nb, b0 + K);
  hv.fix_t = -1;
  ScanAcc v = {0.0, 0.0, 0, 0.0, 0.0, 0.0, 0.0, 0};
#pragma unroll 1
  for (int t = b0; t < b1; ++t) {
    if (t == fix_t) continue;
    const double g = hv.RawG(t), h = hv.RawH(t);
    const int c = RoundIntD(h * L.cnt_factor);
    v.ag += g;
    v.ah += h;
    if (t != def_t) {
      v.g += g;
      v.h += h;
      v.c += c;
    }
    if (t == nb - 1) {
      v.ng = g;
      v.nh = h;
      v.nc = c;
    }
  }
  ScanAcc ex, tot;
  BlockScanNum(&v, &ex, &tot, ssc);
  // FixHistogram
  if (fix_t >= 0) {
    const double fix_g = L.sg - tot.ag;
    const double fix_h = (L.sh - 2 * kEpsilon) - tot.ah;
    const int fix_c = RoundIntD(fix_h * L.cnt_factor);
    hv.fix_t = fix_t;
    hv.fix_g = fix_g;
    hv.fix_h = fix_h;
    if (fix_t != def_t) {
      tot.g += fix_g;
      tot.h += fix_h;
      tot.c += fix_c;
      if (fix_t < b0) {
        ex.g += fix_g;
        ex.h += fix_h;
        ex.c += fix_c;
      }
    }
    if (fix_t == nb - 1) {
      tot.ng = fix_g;
      tot.nh = fix_h;
      tot.nc = fix_c;
    }
  }
  // reverse: right(t) = P(t_start) - P(t - 1) over [t_end_r, t_start]; P(t_start) = total
  // less the NaN bin when it is left out (na and skip_def exclude each other)
  const int t_start_r = nb - 1 - (na ? 1 : 0);
  const int t_end_r = 1 - offset;
  const int t_end_f = nb - 2;
  const double pr_g = na ? tot.g - tot.ng : tot.g;
  const double pr_h = na ? tot.h - tot.nh : tot.h;
  const int pr_c = na ? tot.c - tot.nc : tot.c;
  // forward: left starts empty, or (NaN as missing with bin 0 not stored) with everything
  // outside the stored bins
  const bool minus_one = na && offset == 1;
  const double lg0 = minus_one ? L.sg - tot.ag : 0.0;
  const double lh0 = minus_one ? L.sh - kEpsilon - tot.ah : kEpsilon;
  const int lc0 = minus_one ? L.n - tot.c : 0;  // (na: every stored bin is included)
  const double min_h = p.min_sum_hessian_in_leaf;
  const int min_n = p.min_data_in_leaf;
  const int8_t mono = static_cast<int8_t>(F.monotone);
  Cand rb, fb;
  rb.gain = fb.gain = -INFINITY;
  rb.thr = -1;
  fb.thr = 0x7fffffff;
  rb.lg = rb.lh = fb.lg = fb.lh = 0.0;
  rb.lc = fb.lc = 0;
  bool any = false;
  double pg = ex.g, ph = ex.h;
  int pc = ex.c;
  const int cend = 2 * (b1 - b0);
#pragma unroll 1
  for (int c = (minus_one && tid == 0) ? -1 : 0; c < cend; ++c) {
    // candidate c: -1 the forward start, 2i reverse at t = b0 + i, 2i + 1 forward at t
    const int t = b0 + (c >> 1);
    const bool rev = c >= 0 && (c & 1) == 0;
    bool ok;
    double xg, xh;
    int xc, thr;
    if (c < 0) {
      ok = true;
      xg = lg0;
      xh = lh0;
      xc = lc0;
      thr = offset - 1;
    } else if (rev) {
      ok = t != def_t && t >= t_end_r && t <= t_start_r;
      // left = total - right, right = bins t..t_start (the reference adds kEpsilon to it)
      xg = L.sg - (pr_g - pg);
      xh = L.sh - (pr_h - ph + kEpsilon);
      xc = L.n - (pr_c - pc);
      thr = t - 1 + offset;
    } else {
      if (t != def_t) {
        const double h = hv.H(t);
        pg += hv.G(t);
        ph += h;
        pc += RoundIntD(h * L.cnt_factor);
      }
      ok = two && t != def_t && t <= t_end_f;
      xg = lg0 + pg;
      xh = lh0 + ph;
      xc = lc0 + pc;
      thr = t + offset;
    }
    if (!ok || xc < min_n || xh < min_h) continue;
    const int rc = L.n - xc;
    const double rh = L.sh - xh;
    if (rc < min_n || rh < min_h) continue;
    if (rthr != kNoRandThr && thr != rthr) continue;  // extra_trees
    const double gain = GainOf<SIMPLE>(xg, xh, L.sg - xg, rh, p.lambda_l2, p, L.c, mono, xc, rc, L.parent_out);
    if (!(gain > L.min_gain_shift)) continue;
    any = true;
    const Cand& cur = rev ? rb : fb;
    if (gain > cur.gain || (gain == cur.gain && (rev ? thr > cur.thr : thr < cur.thr))) {
      Cand nc;
      nc.gain = gain;
      nc.thr = thr;
      nc.lg = xg;
      nc.lh = xh;
      nc.lc = xc;
      if (rev) rb = nc;
      else fb = nc;
    }
  }
  BlockBestPair(&rb, &fb, &any, sc, sc2);
  out->gain = -INFINITY;
  out->default_left = two ? 1 : (F.missing_type == 2 ? 0 : 1);
  out->mono = F.monotone;
#pragma unroll 1
  for (int d = 0; d < (two ? 2 : 1); ++d) {
    const Cand b = d == 0 ? rb : fb;
    if (any && b.gain > out->gain + L.min_gain_shift) {
      out->thr = b.thr;
      out->lo = OutputOf<SIMPLE>(b.lg, b.lh, p.lambda_l2, p, L.c, b.lc, L.parent_out);
      out->lc = b.lc;
      out->lg = b.lg;
      out->lh = b.lh - kEpsilon;
      out->ro = OutputOf<SIMPLE>(L.sg - b.lg, L.sh - b.lh, p.lambda_l2, p, L.c, L.n - b.lc, L.parent_out);
      out->rc = L.n - b.lc;
      out->rg = L.sg - b.lg;
      out->rh = L.sh - b.lh - kEpsilon;
      out->gain = b.gain - L.min_gain_shift;
      out->default_left = d == 1 ? 0 : (!two && F.missing_type == 2 ? 0 : 1);
    }
  }
  out->gain *= F.penalty;  // (CEGB and the monotone depth penalty follow in FindBody)
  (void)depth;
  (void)mono_penalty;
  return any;
}

// MonotoneSplitPenalty(depth, penalization)
__device__ __forceinline__ double MonotonePenalty(int depth, double mono_penalty) {
  if (mono_penalty >= depth + 1.) return kEpsilon;
  if (mono_penalty <= 1.) return 1. - mono_penalty / pow(2., depth) + kEpsilon;
  return 1. - pow(2., mono_penalty - 1. - depth) + kEpsilon;
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
template <int NT>
__device__ __forceinline__ bool FindCategoricalBlock(const Feature& F, HistView hv, const LeafCtx& L, const SplitParams& p,
                                     FeatureBest* out, uint32_t* cat_out, BlockScratch<NT>* sc, CatScratch* cs) {
  constexpr int kFindThreads = NT;
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
  CatWords bits;  // (published whole: the picking workgroup reads the winner's set)
  for (int w = 0; w < kMaxCatWords; ++w) bits.w[w] = 0u;
  if (onehot) {
    const int b = best.thr + offset;
    bits.w[b >> 5] |= 1u << (b & 31);
    out->ncat = 1;
  } else {
    const int k = best.thr + 1;
    for (int i = 0; i < k; ++i) {
      const int b = (best_dir == 1 ? cs->sorted[i] : cs->sorted[cs->used_bin - 1 - i]) + offset;
      bits.w[b >> 5] |= 1u << (b & 31);
    }
    out->ncat = k;
  }
  PublishRecord(reinterpret_cast<CatWords*>(cat_out), bits);
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
__device__ __forceinline__ int XtDraws(const KArgs& a, const Feature& F, int f, int mi, IcMask icmask, bool gate) {
  if (!gate || F.num_bin - 2 <= 0) return 0;
  if (a.node_mask != nullptr && !a.node_mask[static_cast<size_t>(mi) * a.p.num_features + f]) return 0;
  if (a.feat_icmask != nullptr && (icmask & a.feat_icmask[f]) == 0) return 0;
  return 1;
}

// GatherInfoForThreshold (reference feature_histogram.hpp; host split_finder.cpp): the split of
// a forced node at bin `thr` from the leaf's histogram, one thread.  hv holds the raw bins;
// the most frequent bin is rebuilt from the leaf totals first (FixHistogram).  Invalid (gain
// no better than the leaf's own): gain -inf, the pick then drops the forced splits.
__device__ void ForcedGather(const Feature& F, HistView hv, const LeafCtx& L, const SplitParams& p, int thr,
                             FeatureBest* out, CatWords* bits) {
  const int nb = F.num_bin - F.offset, offset = F.offset;
  const double sum_g = L.sg, sum_h = L.sh - 2 * kEpsilon;  // the leaf's raw sums
  hv.fix_t = -1;
  if (F.mfb > 0) {
    double og = 0.0, oh = 0.0;
    for (int t = 0; t < nb; ++t) {
      if (t == F.mfb) continue;
      og += hv.RawG(t);
      oh += hv.RawH(t);
    }
    hv.fix_t = F.mfb;
    hv.fix_g = sum_g - og;
    hv.fix_h = sum_h - oh;
  }
  const int smooth = p.use_smoothing;
  const double gain_shift = LeafGainGivenOutput(sum_g, sum_h, p.lambda_l1, p.lambda_l2, L.parent_out, 1);
  const double min_gain_shift = gain_shift + p.min_gain_to_split;
  const double cnt_factor = L.n / sum_h;
  FeatureBest o = {};
  o.gain = -INFINITY;
  o.feature = -1;
  o.real_feature = -1;
  for (int w = 0; w < kMaxCatWords; ++w) bits->w[w] = 0u;
  double lg, lh, rg, rh;
  int lc, rc;
  if (!F.is_cat) {
    rg = 0.0;
    rh = kEpsilon;
    rc = 0;
    const bool skip_default = F.missing_type == 1, na = F.missing_type == 2;
    for (int t = nb - 1 - (na ? 1 : 0); t >= 1 - offset; --t) {
      if (static_cast<uint32_t>(t + offset) < static_cast<uint32_t>(thr)) break;
      if (skip_default && t + offset == F.default_bin) continue;
      rg += hv.G(t);
      rh += hv.H(t);
      rc += RoundIntD(hv.H(t) * cnt_factor);
    }
    lg = sum_g - rg;
    lh = sum_h - rh;
    lc = L.n - rc;
    o.default_left = 1;
  } else {
    if (thr >= F.num_bin || thr == 0) {
      *out = o;
      return;
    }
    const double hh = hv.H(thr - offset);
    lc = RoundIntD(hh * cnt_factor);
    rc = L.n - lc;
    lh = hh + kEpsilon;
    rh = sum_h - lh;
    lg = hv.G(thr - offset);
    rg = sum_g - lg;
    o.default_left = 0;
    o.ncat = 1;
    bits->w[thr >> 5] |= 1u << (thr & 31);
  }
  const double gain = LeafGain(lg, lh, p.lambda_l1, p.lambda_l2, p.max_delta_step, p.path_smooth, lc, L.parent_out, 1, 1,
                               smooth) +
                      LeafGain(rg, rh, p.lambda_l1, p.lambda_l2, p.max_delta_step, p.path_smooth, rc, L.parent_out, 1, 1,
                               smooth);
  if (!(gain > min_gain_shift)) {  // (NaN included)
    *out = o;
    return;
  }
  o.thr = F.is_cat ? 0 : thr;
  o.lo = LeafOutputRaw(lg, lh, p.lambda_l1, p.lambda_l2, p.max_delta_step, p.path_smooth, lc, L.parent_out, 1, 1,
                       smooth);
  o.ro = LeafOutputRaw(sum_g - lg, sum_h - lh, p.lambda_l1, p.lambda_l2, p.max_delta_step, p.path_smooth, rc,
                       L.parent_out, 1, 1, smooth);
  o.lc = lc;
  o.rc = L.n - lc;
  o.lg = lg;
  o.lh = lh - kEpsilon;
  o.rg = sum_g - lg;
  o.rh = sum_h - lh - kEpsilon;
  o.gain = gain - min_gain_shift;
  o.mono = 0;
  o.feature = -2;  // (set by the caller)
  *out = o;
}

template <bool ROOT, int KIND, int NT>
struct FindShared {
  BlockScratch<NT> sc;
  ScanScratch<NT> ssc;
  Cand sc2[NT / kWave];
  typename std::conditional<KIND == 2, CatScratch, int>::type cat_sc;
  unsigned long long s_red[2 * NT];  // direct partial sums of narrow features
};

// the scan of one (feature, child) by one workgroup: every thread of the workgroup takes the
// same path (the kernel's pick tail needs all of them)
template <bool ROOT, int KIND, bool SIMPLE, int NT>
__device__ __forceinline__ void FindBody(const KArgs& a, double* s_bins, FindShared<ROOT, KIND, NT>& sh) {
  constexpr bool CAT = KIND == 2;
  constexpr int kFindThreads = NT;
  const long long t_entry = wall_clock64();
  // voting-parallel global scan: the features the vote elected for this side's leaf (an
  // empty slot still takes part in the step's workgroup count)
  const bool vote_global = a.p.vote_phase == 2;
  int f = CAT ? a.cat_list[blockIdx.x] : (a.feat_list != nullptr ? a.feat_list[blockIdx.x] : static_cast<int>(blockIdx.x));
  if (vote_global) f = a.vote_list[blockIdx.y * a.p.vote_k + blockIdx.x];
  const bool vote_empty = vote_global && f < 0;
  if (vote_empty) f = 0;
  const int side = blockIdx.y;
  const int tid = threadIdx.x;
  const int units = a.hist_units;
  // ---- independent loads first (one round trip): the feature, its mask, the scales and the
  // Step record
  const Feature F = a.feat[f];
  const int8_t tree_used = a.tree_mask[f];
  const Step* st = a.st;
  const int mi_base = ROOT ? 0 : st->bynode_next;  // this step's per-node masks (advanced by the pick)
  int8_t used = tree_used;  // evaluated at this node (feature_fraction_bynode)
  if (a.node_mask != nullptr) used = used && a.node_mask[static_cast<size_t>(mi_base + side) * a.p.num_features + f];
  // (voting: every feature is scanned -- the vote may elect one this rank could not split)
  const int8_t parent_ok = (ROOT || a.p.vote_phase != 0) ? 1 : a.parent_flags[f];
  const double ig = a.scales[2], ih = a.scales[3];
  int s = 0, pc = 0, skip = 0;
  ChildInfo c;
  SideInfo sd;
  ChildStats cl;
  if (!ROOT) {
    s = st->cs.s;
    pc = st->cs.part_count;
    c = StepChildren(a, st);
    sd = StepSide(a, st, c, side);
    cl = st->lr[sd.lr];
    skip = c.skip;
  }
  // extra_trees: per feature and node, the smaller child draws before the larger one
  // (SerialTreeLearner::FindBestSplitsFromHistograms); draw k of the tree is the base state
  // stepped k times.  The smaller child's workgroup appends the step's count row.
  int xt_thr = kNoRandThr;
  if (a.xt_base != nullptr) {
    const int nf = a.p.num_features;
    const int prev = ROOT ? 0 : a.xt_cum[static_cast<size_t>(s) * nf + f];
    const bool gate = tree_used && parent_ok && !skip;
    const IcMask icm = ROOT ? kIcAll : cl.icmask;  // both children carry the same constraints
    const int d0 = XtDraws(a, F, f, mi_base, icm, gate);
    const int d1 = ROOT ? 0 : XtDraws(a, F, f, mi_base + 1, icm, gate);
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
    parity = (s + 1) & 1;
    // zero this feature's bins of the buffer the next step reduces into (data-parallel:
    // the whole owner-major buffer is cleared before each reduction)
    if (!CAT && side == 0 && a.rs_pos == nullptr && !vote_global) {
      long long* nxt = StepScratch(a, parity + 1);
      for (int i = tid; i < nb2; i += kFindThreads) nxt[2 * F.hist_offset + i] = 0;
    }
    if (skip) return;
    KTraceAt(a, s, kTrFindEntry, t_entry);
    KTrace(a, s, kTrFindHdr);
    const int nblk = StepBlocks(a, pc);
    if (DirectPartials(a, nblk, s) && !vote_global) nblk_direct = nblk;
  }
  const SplitParams& p = a.p.sp;
  LeafCtx L;
  int depth, slot;
  if (ROOT) {
    const double* rsum = a.p.vote_phase == 1 ? a.root_local : a.root;  // voting: local, then global
    const double sg = rsum[0], shh = rsum[1];
    const int n = static_cast<int>(rsum[2]);
    ConstraintRange cr;
    cr.min = -DBL_MAX;
    cr.max = DBL_MAX;
    SplitParams rp = p;
    rp.use_l1 = 1;
    rp.use_max_output = 1;
    rp.use_smoothing = 0;
    rp.use_mc = 1;
    const double out0 = LeafOutputConstrained(sg, shh, p.lambda_l2, rp, cr, n, 0);
    const bool first = vote_global ? blockIdx.x == 0 : f == 0;
    if (first && tid == 0 && KIND != 2) {  // (write-through: the root pick rewrites leaf 0)
      Leaf& lf = a.leaves[0];
      if (a.p.vote_phase == 1) {
        PublishF64(&lf.lsum_g, sg);
        PublishF64(&lf.lsum_h, shh);
      } else {
        PublishF64(&lf.sum_g, sg);
        PublishF64(&lf.sum_h, shh);
        PublishI32(&lf.global_count, n);
        PublishF64(&lf.output, out0);
        PublishI32(&a.st->root_count, n);
      }
    }
    L.sg = sg;
    L.sh = shh + 2 * kEpsilon;
    L.n = n;
    L.parent_out = out0;
    L.c = cr;
    depth = 0;
    slot = 0;
  } else {
    L.sg = cl.sum_g;
    L.sh = cl.sum_h + 2 * kEpsilon;
    L.n = sd.global_count;
    L.parent_out = cl.output;
    L.c.min = cl.cmin;
    L.c.max = cl.cmax;
    depth = cl.depth;
    slot = sd.slot;
    if (a.p.vote_phase == 1) {
      // voting local scan: this rank's rows of the child -- the histogrammed child's sums from
      // k_split, the other one's as the parent's minus those
      const double hg = static_cast<double>(static_cast<long long>(st->loc_acc[0])) * ig;
      const double hh = static_cast<double>(static_cast<long long>(st->loc_acc[1])) * ih;
      const double lsg = sd.is_hist ? hg : st->cs.plsum_g - hg;
      const double lsh = sd.is_hist ? hh : st->cs.plsum_h - hh;
      L.sg = lsg;
      L.sh = lsh + 2 * kEpsilon;
      L.n = sd.lr == 0 ? c.total_left : pc - c.total_left;
      if (blockIdx.x == 0 && tid == 0) {
        a.leaves[sd.leaf].lsum_g = lsg;
        a.leaves[sd.leaf].lsum_h = lsh;
      }
    }
  }
  if (vote_empty) return;
  if (KIND == 1 && F.is_cat) return;  // the categorical kernel scans it
  if (CAT && !F.is_cat) return;       // (voting global scan: an elected numerical feature)
  // interaction constraints: like a sampled-out feature, a disallowed one is not evaluated
  // here but keeps its histogram and its splittable flag
  if (a.feat_icmask != nullptr && ((ROOT ? kIcAll : cl.icmask) & a.feat_icmask[f]) == 0) used = 0;
  int8_t* flags = a.splittable + static_cast<size_t>(ROOT ? a.leaves[0].frow : sd.frow) * a.p.num_features;
  FeatureBest* fb_out = &a.feat_best[FeatBestIndex(a, side, f)];
  if (tree_used && !parent_ok) {
    // the parent could not split on f: neither child evaluates it, the smaller child's row
    // says so and the larger child keeps the parent's row (SerialTreeLearner::FindBestSplits)
    if (side == 0 && tid == 0) flags[f] = 0;
    if (tid == 0) {
      FeatureBest none = {};
      none.gain = -INFINITY;
      none.feature = none.real_feature = -1;
      PublishRecord(fb_out, none);
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
    // (voting global scan: the elected feature's histogram summed over the ranks, read in place)
    long long* dst = vote_global ? a.vote_hist + static_cast<size_t>(side * a.p.vote_k + blockIdx.x) * 2 *
                                                     a.p.max_feature_bins
                                 : a.hist + static_cast<size_t>(slot) * nh + 2 * F.hist_offset;
    const long long* src = vote_global ? dst
                           : a.owned_hist != nullptr ? a.owned_hist + 2 * (F.hist_offset - a.owned_bin_lo)
                                                     : StepScratch(a, parity) + 2 * F.hist_offset;
    const size_t pstride = static_cast<size_t>(units) * a.p.total_bins;
    const unsigned long long* part = a.partials + static_cast<size_t>(units) * F.hist_offset;
    const bool stage = a.p.max_feature_bins <= kFindLdsBins;
    double* sg = s_bins;
    double* shv = s_bins + (stage ? a.p.max_feature_bins : 0);
    const bool subtract = !ROOT && !sd.is_hist && !vote_global;  // parent - the histogrammed child, in place
    // a feature with fewer bins than threads sums its direct partials with every thread:
    // kFindThreads / nbf threads per bin stride over the row blocks, then combine in LDS
    // (one thread per bin walking hundreds of partials would be a chain of round trips)
    const bool spread = nblk_direct > 1 && 2 * nbf <= kFindThreads;
    // the parent's bins (first bin of each thread): loaded up front, so their round trip
    // overlaps the partial-sum loads instead of following them
    long long pg0 = 0, ph0 = 0;
    if (subtract && tid < nbf) {
      pg0 = dst[2 * tid];
      ph0 = dst[2 * tid + 1];
    }
    if (spread) {
      for (int j = tid; j < 2 * nbf; j += kFindThreads) sh.s_red[j] = 0ull;
      __syncthreads();
      const int per = kFindThreads / nbf;
      const int i = tid % nbf, r = tid / nbf;
      if (r < per) {
        constexpr int kC = 8;
        long long g = 0, h = 0;
        for (int k0 = r; k0 < nblk_direct; k0 += per * kC) {
          unsigned long long v0[kC], v1[kC];
#pragma unroll
          for (int cc = 0; cc < kC; ++cc) {
            const int k = k0 + cc * per;
            const unsigned long long* q = part + k * pstride + static_cast<size_t>(units) * i;
            v0[cc] = k < nblk_direct ? q[0] : 0ull;
            v1[cc] = (k < nblk_direct && units == 2) ? q[1] : 0ull;
          }
#pragma unroll
          for (int cc = 0; cc < kC; ++cc) {
            long long pgv, phv;
            UnpackPartial(v0[cc], v1[cc], units, &pgv, &phv);
            g += pgv;
            h += phv;
          }
        }
        atomicAdd(&sh.s_red[2 * i], static_cast<unsigned long long>(g));
        atomicAdd(&sh.s_red[2 * i + 1], static_cast<unsigned long long>(h));
      }
      __syncthreads();
    }
    for (int i = tid; i < nbf; i += kFindThreads) {
      long long g = 0, h = 0;
      if (spread) {
        g = static_cast<long long>(sh.s_red[2 * i]);
        h = static_cast<long long>(sh.s_red[2 * i + 1]);
      } else if (nblk_direct >= 0) {
        // small leaf: sum the few per-block partials here (k_hist_reduce skipped them),
        // chunks of kDirectChunk independent loads in flight
        for (int k0 = 0; k0 < nblk_direct; k0 += kDirectChunk) {
          unsigned long long v0[kDirectChunk], v1[kDirectChunk];
#pragma unroll
          for (int k = 0; k < kDirectChunk; ++k) {
            const unsigned long long* q = part + (k0 + k) * pstride + static_cast<size_t>(units) * i;
            v0[k] = k0 + k < nblk_direct ? q[0] : 0ull;
            v1[k] = (k0 + k < nblk_direct && units == 2) ? q[1] : 0ull;
          }
#pragma unroll
          for (int k = 0; k < kDirectChunk; ++k) {
            long long pgv, phv;
            UnpackPartial(v0[k], v1[k], units, &pgv, &phv);
            g += pgv;
            h += phv;
          }
        }
      } else {
        g = src[2 * i];
        h = src[2 * i + 1];
      }
      if (subtract) {
        g = (i == tid ? pg0 : dst[2 * i]) - g;
        h = (i == tid ? ph0 : dst[2 * i + 1]) - h;
      }
      dst[2 * i] = g;
      dst[2 * i + 1] = h;
      if (stage) {
        sg[i] = static_cast<double>(g) * ig;
        shv[i] = static_cast<double>(h) * ih;
      }
    }
    __syncthreads();  // the workgroup's stores become visible to all its threads
    if (!ROOT) KTrace(a, s, kTrFindLoaded);
    if (!used) {
      if (tid == 0) {
        FeatureBest none = {};
        none.gain = -INFINITY;
        none.feature = none.real_feature = -1;
        PublishRecord(fb_out, none);
      }
      return;
    }
    HistView hv;
    hv.lg = stage ? sg : nullptr;
    hv.lh = stage ? shv : nullptr;
    hv.h = dst;
    hv.inv_g = ig;
    hv.inv_h = ih;
    bool splittable;
    if constexpr (CAT) {
      splittable = FindCategoricalBlock(F, hv, L, p, &o, a.feat_cat + FeatBestIndex(a, side, f) * kMaxCatWords, &sh.sc,
                                        &sh.cat_sc);
    } else {
      splittable = FindNumericalBlock<SIMPLE, NT>(F, hv, L, p, depth, a.p.monotone_penalty, &o, &sh.sc, &sh.ssc, sh.sc2,
                                              xt_thr);
    }
    if (tid == 0 && !vote_global) flags[f] = splittable ? 1 : 0;  // (the local scan's flags stay)
    // SerialTreeLearner::EvalFeature order: the CEGB cost (the raw candidate remembered for the
    // coupled-penalty refund), then the monotone depth penalty
    if (a.p.cegb && tid == 0) {
      const int leaf = ROOT ? 0 : sd.leaf;
      if (a.cegb_mem != nullptr) {  // (read by the pick's refunds: write-through)
        const size_t mi = static_cast<size_t>(leaf) * a.p.num_features + f;
        PublishRecord(&a.cegb_mem[mi], o);
        if (CAT) {
          const CatWords bits = *reinterpret_cast<const CatWords*>(a.feat_cat + FeatBestIndex(a, side, f) * kMaxCatWords);
          PublishRecord(reinterpret_cast<CatWords*>(a.cegb_mem_cat + mi * kMaxCatWords), bits);
        }
      }
      double delta = a.p.cegb_split * L.n;
      if (a.cegb_coupled != nullptr && !a.cegb_used[f]) delta += a.cegb_coupled[f];
      o.gain -= delta;
    }
    if (!CAT && !SIMPLE && F.monotone != 0) o.gain *= MonotonePenalty(depth, a.p.monotone_penalty);
    // a forced node on this child and feature: its split at the forced threshold (published
    // for the pick, which applies it as split k)
    if (a.forced_n > 0 && tid == 0 && !vote_global) {
      const int k = ROOT ? 0 : (s < a.forced_n ? a.forced_child[2 * s + sd.lr] : -1);
      if (k >= 0 && k < a.forced_n && a.forced_feat[k] == f) {
        FeatureBest fo;
        CatWords fbits;
        ForcedGather(F, hv, L, p, a.forced_thr[k], &fo, &fbits);
        if (fo.feature == -2) {
          fo.feature = f;
          fo.real_feature = F.real_index;
        }
        PublishRecord(reinterpret_cast<CatWords*>(a.forced_cat + static_cast<size_t>(k) * kMaxCatWords), fbits);
        PublishRecord(&a.forced_best[k], fo);
      }
    }
    if (!ROOT) KTrace(a, s, kTrFindScanned);
  } else {
    o.feature = -1;
  }
  if (tid == 0) PublishRecord(fb_out, o);
}

#ifndef LGBM_FIND_WAVE_OCC
#define LGBM_FIND_WAVE_OCC 4  // one-wave split scans: waves per SIMD the register budget allows
#endif
constexpr unsigned kFindFlatMax = 128;  // split-scan grids up to this size count arrivals on one counter

// NT: threads per workgroup -- kFindThreads, or one wave (kWave) when every feature has at
// most kWave stored bins (many narrow features: four times the workgroups in flight, and no
// cross-wave steps in the scans)
template <bool ROOT, int KIND, bool SIMPLE, int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT == kWave ? LGBM_FIND_WAVE_OCC : 1))) void k_find(KArgs a) {
  extern __shared__ double s_bins[];  // [2][max_feature_bins] dequantised (g, h), if they fit
  __shared__ FindShared<ROOT, KIND, NT> sh;
  __shared__ PickLds pl;
  __shared__ int s_last;
  Step* st = a.st;
  if (!ROOT && st->done) return;
  FindBody<ROOT, KIND, SIMPLE, NT>(a, s_bins, sh);
  // single process: the last workgroup of the step records it and picks the next split
  // (with categorical features the numerical kernel runs first and does not count)
  if (!a.pick_in_find || (KIND == 1)) return;
  // hand-off to the picking workgroup: what it reads of this launch (per-feature results,
  // category sets, CEGB candidates, the root's leaf record) was stored write-through
  // (PublishRecord); every wave drains its stores, then one lane counts the arrival.  Other
  // results (histograms, flags) are read by later kernels only.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned nwg = gridDim.x * gridDim.y;
    int last = 0;
    if (nwg <= kFindFlatMax) {
      last = atomicAdd(&st->find_count, 1u) == nwg - 1 ? 1 : 0;
    } else {
      // one counter serialises thousands of arrivals (~12 ns each at the memory-side atomic
      // unit, tools/microbench/wg_throughput.hip): kFindSub counters take a share each, the last
      // of a share reports to find_count (and resets its counter for the next step)
      const unsigned id = blockIdx.y * gridDim.x + blockIdx.x, g = id % kFindSub;
      const unsigned members = (nwg - g + kFindSub - 1) / kFindSub;
      uint32_t* sub = a.find_sub + g * kFindSubStride;
      if (atomicAdd(sub, 1u) == members - 1) {
        atomicExch(sub, 0u);
        last = atomicAdd(&st->find_count, 1u) == kFindSub - 1 ? 1 : 0;
      }
    }
    if (last) {  // one agent-scope acquire for the workgroup (then the barrier below)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  const int s = ROOT ? -1 : st->cs.s;
  if (!ROOT && a.ktrace != nullptr && threadIdx.x == 0 && s < a.p.num_leaves) {
    a.ktrace[s * kTraceSlots + kTrPickEntry] = wall_clock64();
  }
  PickAndRecord(a, st, ROOT, &pl, s);
  if (!ROOT && a.ktrace != nullptr && threadIdx.x == 0 && s < a.p.num_leaves) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    a.ktrace[s * kTraceSlots + kTrPickExit] = wall_clock64();
    a.ktrace[s * kTraceSlots + kTrClk1] = __builtin_amdgcn_s_memtime();
  }
}

// the step's bookkeeping and the next pick alone (distributed learners)
__global__ __launch_bounds__(kFindThreads) void k_pick(KArgs a, int root) {
  __shared__ PickLds pl;
  Step* st = a.st;
  if (st->done) return;
  PickAndRecord(a, st, root != 0, &pl);
}

static size_t FindLds(const KArgs& a) {
  return a.p.max_feature_bins <= kFindLdsBins ? 2 * sizeof(double) * static_cast<size_t>(a.p.max_feature_bins) : 0;
}
// plain gain formulas (no L1 / max_delta_step / path smoothing / monotone constraints)
static bool SimpleGains(const KArgs& a) {
  const SplitParams& p = a.p.sp;
  return !p.use_l1 && !p.use_max_output && !p.use_smoothing && !p.use_mc;
}
template <bool ROOT>
static void LaunchFind(const KArgs& a, hipStream_t s) {
  if (a.num_scan <= 0) return;  // a rank that owns no feature
  const dim3 g(a.num_scan, ROOT ? 1 : 2);
  const size_t lds = FindLds(a);
  const bool simple = SimpleGains(a);
  const bool narrow = a.p.max_feature_bins <= kWave;  // (categorical scans keep kFindThreads)
  const dim3 b(narrow ? kWave : kFindThreads), bc(kFindThreads);
  if (a.p.has_cat) {
    if (narrow) {
      if (simple) hipLaunchKernelGGL((k_find<ROOT, 1, true, kWave>), g, b, lds, s, a);
      else hipLaunchKernelGGL((k_find<ROOT, 1, false, kWave>), g, b, lds, s, a);
    } else {
      if (simple) hipLaunchKernelGGL((k_find<ROOT, 1, true, kFindThreads>), g, b, lds, s, a);
      else hipLaunchKernelGGL((k_find<ROOT, 1, false, kFindThreads>), g, b, lds, s, a);
    }
    const int ncat = a.p.vote_phase == 2 ? a.num_scan : a.p.has_cat;  // voting: every elected slot
    if (a.p.has_cat > 0) hipLaunchKernelGGL((k_find<ROOT, 2, false, kFindThreads>), dim3(ncat, ROOT ? 1 : 2), bc, lds, s, a);
  } else if (narrow) {
    if (simple) hipLaunchKernelGGL((k_find<ROOT, 0, true, kWave>), g, b, lds, s, a);
    else hipLaunchKernelGGL((k_find<ROOT, 0, false, kWave>), g, b, lds, s, a);
  } else {
    if (simple) hipLaunchKernelGGL((k_find<ROOT, 0, true, kFindThreads>), g, b, lds, s, a);
    else hipLaunchKernelGGL((k_find<ROOT, 0, false, kFindThreads>), g, b, lds, s, a);
  }
}
void FindRoot(const KArgs& a, hipStream_t s) { LaunchFind<true>(a, s); }
void FindStep(const KArgs& a, hipStream_t s) { LaunchFind<false>(a, s); }
void PickStep(const KArgs& a, hipStream_t s, bool root) {
  hipLaunchKernelGGL(k_pick, dim3(1), dim3(kFindThreads), 0, s, a, root ? 1 : 0);
}

}  // namespace dev
}  // namespace lgbm_amd
