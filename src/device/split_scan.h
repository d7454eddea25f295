// Split-scan primitives shared by the one-split-per-step kernels (split_kernels.hip) and the
// round-growth kernels (round_kernels.hip): block scans / argmaxes, the numerical threshold
// scan with FixHistogram (reference feature_histogram.hpp FindBestThresholdSequentially,
// FuncForNumricalL3, FixHistogram) and the categorical scan (FindBestThresholdCategoricalInner).
#pragma once

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

#ifndef LGBM_DPP_ARGMAX
#define LGBM_DPP_ARGMAX 1
#endif
// the wave's best candidate in CandBetter order: a 64-bit DPP max of the gain key (NaN below
// every number), then among the lanes holding it the threshold order (reverse: highest,
// forward: lowest) as a 32-bit DPP max, and reads of the winning lane -- instead of a
// butterfly of five-field shuffles through the LDS crossbar (~2.7 us per scan workgroup)
__device__ __forceinline__ Cand WaveBestCand(Cand c, bool reverse) {
#if LGBM_DPP_ARGMAX
  const unsigned long long k1 = c.gain != c.gain ? 1ull : GainKey(c.gain) + 1ull;  // (> 0: the DPP identity)
  const unsigned long long m1 = WaveMaxDpp(k1);
  const bool t1 = k1 == m1;
  // (thresholds are signed, -1 included: offset by 2^31 to order them as unsigned, + 1 > 0)
  const uint32_t tu = static_cast<uint32_t>(c.thr) ^ 0x80000000u;
  const unsigned long long k2 = t1 ? static_cast<unsigned long long>(reverse ? tu : ~tu) + 1ull : 0ull;
  const unsigned long long m2 = WaveMaxDpp(k2);
  const unsigned long long win = __ballot(t1 && k2 == m2);
  const int w = __builtin_amdgcn_readfirstlane(static_cast<int>(__builtin_ctzll(win)));
  Cand r;
  r.gain = ReadLane(c.gain, w);
  r.thr = ReadLane(c.thr, w);
  r.lg = ReadLane(c.lg, w);
  r.lh = ReadLane(c.lh, w);
  r.lc = ReadLane(c.lc, w);
  return r;
#else
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
#endif
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
#ifndef LGBM_FIND_PHASES
#define LGBM_FIND_PHASES 0  // (A/B instrumentation: phase timestamps of the scan, g_find_phase)
#endif
#if LGBM_FIND_PHASES
__shared__ long long g_find_phase[4];
#define LGBM_FIND_STAMP(k) \
  if (threadIdx.x == 0) g_find_phase[k] = wall_clock64()
#else
#define LGBM_FIND_STAMP(k)
#endif
template <bool SIMPLE, int NT>
__device__ bool FindNumericalBlock(const Feature& F, HistView hv, const LeafCtx& L, const SplitParams& p, int depth,
                                   double mono_penalty, FeatureBest* out, BlockScratch<NT>* sc, ScanScratch<NT>* ssc,
                                   Cand* sc2, int rthr) {
  LGBM_FIND_STAMP(0);
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
  LGBM_FIND_STAMP(1);
  // FixHistogram.  The stored bins are integers on the fixed-point grid, so every prefix of them
  // is exact in any order; the rebuilt bin is not, and it is added to a candidate's prefix last
  // (fix_in) -- the canonical sums the extra_trees replay of round growth reproduces from stored
  // prefixes (XtStorePrefix / XtEvalNum)
  double fix_g = 0.0, fix_h = 0.0;
  int fix_c = 0;
  const bool fix_in = fix_t >= 0 && fix_t != def_t;
  if (fix_t >= 0) {
    fix_g = L.sg - tot.ag;
    fix_h = (L.sh - 2 * kEpsilon) - tot.ah;
    fix_c = RoundIntD(fix_h * L.cnt_factor);
    hv.fix_t = fix_t;
    hv.fix_g = fix_g;
    hv.fix_h = fix_h;
    if (fix_in) {
      tot.g += fix_g;
      tot.h += fix_h;
      tot.c += fix_c;
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
      const bool fx = fix_in && fix_t < t;
      const double eg = fx ? pg + fix_g : pg, eh = fx ? ph + fix_h : ph;
      const int ec = fx ? pc + fix_c : pc;
      xg = L.sg - (pr_g - eg);
      xh = L.sh - (pr_h - eh + kEpsilon);
      xc = L.n - (pr_c - ec);
      thr = t - 1 + offset;
    } else {
      if (t != def_t && t != fix_t) {
        const double h = hv.RawH(t);
        pg += hv.RawG(t);
        ph += h;
        pc += RoundIntD(h * L.cnt_factor);
      }
      ok = two && t != def_t && t <= t_end_f;
      const bool fx = fix_in && fix_t <= t;
      xg = lg0 + (fx ? pg + fix_g : pg);
      xh = lh0 + (fx ? ph + fix_h : ph);
      xc = lc0 + (fx ? pc + fix_c : pc);
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
  LGBM_FIND_STAMP(2);
  BlockBestPair(&rb, &fb, &any, sc, sc2);
  LGBM_FIND_STAMP(3);
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

// extra_trees on round growth (KArgs::node_pre): the inclusive prefix over a feature's stored
// bins of (g, h, estimated rows) -- the rebuilt most frequent bin left out, the default bin in
// (the replay takes it out again).  Every stored bin is an integer on the fixed-point grid, so
// these are exactly the sums FindNumericalBlock accumulates, whatever the order, and a
// threshold drawn later is evaluated from a few entries.  Ends with a barrier (ssc is reused)
template <int NT>
__device__ void XtStorePrefix(const Feature& F, HistView hv, const LeafCtx& L, XtPre* out, ScanScratch<NT>* ssc) {
  const int tid = threadIdx.x;
  const int nb = F.num_bin - F.offset;
  const int fix_t = F.mfb > 0 ? F.mfb : -1;
  const int K = (nb + NT - 1) / NT;
  const int b0 = tid * K, b1 = min(nb, b0 + K);
  hv.fix_t = -1;
  ScanAcc v = {0.0, 0.0, 0, 0.0, 0.0, 0.0, 0.0, 0};
#pragma unroll 1
  for (int t = b0; t < b1; ++t) {
    if (t == fix_t) continue;
    const double h = hv.RawH(t);
    v.g += hv.RawG(t);
    v.h += h;
    v.c += RoundIntD(h * L.cnt_factor);
  }
  ScanAcc ex, tot;
  BlockScanNum(&v, &ex, &tot, ssc);
  double pg = ex.g, ph = ex.h;
  int pc = ex.c;
#pragma unroll 1
  for (int t = b0; t < b1; ++t) {
    if (t != fix_t) {
      const double h = hv.RawH(t);
      pg += hv.RawG(t);
      ph += h;
      pc += RoundIntD(h * L.cnt_factor);
    }
    XtPre o;
    o.g = pg;
    o.h = ph;
    o.c = pc;
    o.pad = 0;
    out[t] = o;
  }
  __syncthreads();
}

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

// MonotoneSplitPenalty(depth, penalization)
__device__ __forceinline__ double MonotonePenalty(int depth, double mono_penalty) {
  if (mono_penalty >= depth + 1.) return kEpsilon;
  if (mono_penalty <= 1.) return 1. - mono_penalty / pow(2., depth) + kEpsilon;
  return 1. - pow(2., mono_penalty - 1. - depth) + kEpsilon;
}

// LDS of the categorical scan: per-bin ctr and the stable ctr order (CAP bins: the regular
// kernel kFindCatNarrow, the wide one kFindMaxCatBins)
constexpr int kCatPar = 128;  // prefix positions per direction scanned with the parallel path

template <int CAP>
struct CatScratchT {
  static constexpr int kCap = CAP;
  double ctr[CAP];
  int sorted[CAP];
  int used_bin;
  uint32_t bits[kMaxCatWords];  // the winner's category set, built here and published word-parallel
  int ok, best_thr, best_dir;
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
// the candidates' stable order by ctr for wide features: a bitonic sort of (ctr, bin) pairs
// in LDS (the ctr array holds the keys in bin order on entry; non-candidates, NaN, sort last).
// (ctr, bin) is a total order, so the result equals std::stable_sort by ctr.
template <int NT, typename CS>
__device__ __forceinline__ void CatBitonicOrder(CS* cs, int bin_start, int n) {
  int P = 1;
  while (P < n) P <<= 1;
  for (int i = threadIdx.x; i < P; i += NT) {
    if (i >= n) cs->ctr[i] = INFINITY;
    cs->sorted[i] = i < n ? bin_start + i : 0x7fffffff;
  }
  for (int i = threadIdx.x; i < n; i += NT) {
    if (cs->ctr[i] != cs->ctr[i]) {  // non-candidate: after every candidate and the padding's order
      cs->ctr[i] = INFINITY;
      cs->sorted[i] = (1 << 30) + bin_start + i;
    }
  }
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += NT) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const double ka = cs->ctr[i], kb = cs->ctr[ixj];
          const int ia = cs->sorted[i], ib = cs->sorted[ixj];
          const bool a_gt = ka > kb || (ka == kb && ia > ib);
          if (a_gt == ((i & k) == 0)) {
            cs->ctr[i] = kb;
            cs->ctr[ixj] = ka;
            cs->sorted[i] = ib;
            cs->sorted[ixj] = ia;
          }
        }
      }
      __syncthreads();
    }
  }
}

template <int NT, typename CS>
__device__ __forceinline__ bool FindCategoricalBlock(const Feature& F, HistView hv, const LeafCtx& L, const SplitParams& p,
                                     FeatureBest* out, uint32_t* cat_out, BlockScratch<NT>* sc, CS* cs,
                                     bool xt = false, uint32_t xt_r = 0u, int* drew = nullptr) {
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
  // extra_trees (xt): the feature's next draw xt_r (31 bits) picks the one threshold evaluated,
  // NextInt(bin_start, bin_end) one-vs-rest, NextInt(0, max_threshold) sorted -- drawn only when
  // the range is not empty (*drew: whether this scan consumed a draw); without a draw the
  // threshold stays 0, as in the reference
  if (drew != nullptr) *drew = 0;
  if (onehot) {
    int rthr = -1;
    if (xt) {
      const bool d = bin_end - bin_start > 0;
      rthr = d ? bin_start + static_cast<int>(xt_r % static_cast<uint32_t>(bin_end - bin_start)) : 0;
      if (drew != nullptr) *drew = d ? 1 : 0;
    }
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
      if (rthr >= 0 && t != rthr) continue;
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
    const bool wide = CS::kCap > kFindCatNarrow && bin_end - bin_start > kFindCatNarrow;
    int ncand = 0;
    for (int t = bin_start + tid; t < bin_end; t += kFindThreads) {
      const double hh = hv.H(t);
      const bool cand = static_cast<double>(RoundIntD(hh * L.cnt_factor)) >= p.cat_smooth;
      const double c = cand ? hv.G(t) / (hh + p.cat_smooth) : NAN;
      cs->ctr[wide ? t - bin_start : t] = c;
      ncand += c == c ? 1 : 0;
    }
    __syncthreads();
    if (wide) {
      CatBitonicOrder<NT>(cs, bin_start, bin_end - bin_start);
    } else {
      // stable rank among the candidates (std::stable_sort by ctr ascending)
      for (int t = bin_start + tid; t < bin_end; t += kFindThreads) {
        const double c = cs->ctr[t];
        if (c != c) continue;
        int r = 0;
        for (int u = bin_start; u < bin_end; ++u) {
          const double cu = cs->ctr[u];
          r += (cu < c) | ((cu == c) & (u < t));
        }
        cs->sorted[r] = t;
      }
    }
    double d0 = 0.0, d1 = 0.0;
    BlockSum3(d0, d1, ncand, sc);
    const int used_bin = ncand;
    const int max_num_cat = min(p.max_cat_threshold, (used_bin + 1) / 2);
    const int npos = min(used_bin, max_num_cat);
    int rthr = -1;
    if (xt) {
      const int mt = max(npos - 1, 0);
      rthr = mt > 0 ? static_cast<int>(xt_r % static_cast<uint32_t>(mt)) : 0;
      if (drew != nullptr) *drew = mt > 0 ? 1 : 0;
    }
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
            if (rthr >= 0 && i != rthr) continue;
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
          if (rthr >= 0 && i != rthr) continue;
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
  // the winner's category set (thread 0's decision), in LDS, then published by every thread
  if (tid == 0) {
    cs->ok = splittable ? 1 : 0;
    cs->best_thr = best.thr;
    cs->best_dir = best_dir;
  }
  __syncthreads();
  if (cs->ok) {
    for (int w = tid; w < kMaxCatWords; w += kFindThreads) cs->bits[w] = 0u;
    __syncthreads();
    const int k = onehot ? 1 : cs->best_thr + 1;
    for (int i = tid; i < k; i += kFindThreads) {
      const int b = (onehot ? cs->best_thr : cs->best_dir == 1 ? cs->sorted[i] : cs->sorted[cs->used_bin - 1 - i]) + offset;
      atomicOr(&cs->bits[b >> 5], 1u << (b & 31));
    }
    __syncthreads();
    GlobalU64* dst = (GlobalU64*)(cat_out);
    for (int w = tid; w < kMaxCatWords / 2; w += kFindThreads) {
      const unsigned long long v = static_cast<unsigned long long>(cs->bits[2 * w]) |
                                   (static_cast<unsigned long long>(cs->bits[2 * w + 1]) << 32);
      __hip_atomic_store(dst + w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
  out->ncat = onehot ? 1 : best.thr + 1;
  return true;
}

}  // namespace

}  // namespace dev
}  // namespace lgbm_amd
