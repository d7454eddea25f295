// Step bookkeeping and the choice of the next split (reference serial_tree_learner.cpp
// Train loop: ArgMax over best_split_per_leaf_, SplitInner's leaf statistics;
// monotone_constraints.hpp BasicLeafConstraints), as device functions of one workgroup.
// Run by the last split-scan workgroup of a step (single process) or by k_pick after the
// per-feature results were gathered from every rank (distributed learners).
//
//  1. bookkeeping of the step just scanned (thread 0): the children's index ranges from the
//     partition cursors, histogram slots (the histogrammed child took the new leaf's slot),
//     splittable rows, exact counts into the split record.
//  2. pick (first wave): the per-leaf best split of the freshly scanned children (argmax over
//     their per-feature results, SplitInfo order: larger gain, then smaller real feature),
//     then the leaf to split (argmax over all leaves: gain, real feature, lower leaf id -- the
//     host loop's order).  Every load of the pick is independent of the others (one round
//     trip) except the winner's records.
//  3. record (thread 0): Step::cs / lr / hist_left for the next k_split, the children's
//     constraint ranges, the split record (k_split snapshots the parent's splittable row
//     before the children's scans overwrite it).
#pragma once

#include "device_common.h"

namespace lgbm_amd {
namespace dev {

// an argmax candidate in SplitInfo order: larger gain, then smaller real feature, then lower
// index; `x` travels with it (idx < 0: no candidate)
struct ArgC {
  double g;
  int rf, idx, x;
};

__device__ __forceinline__ ArgC ArgNone() {
  ArgC c;
  c.g = -INFINITY;
  c.rf = -1;
  c.idx = -1;
  c.x = -1;
  return c;
}

__device__ __forceinline__ void ArgTake(ArgC* c, const ArgC& o) {
  const bool take = o.idx >= 0 && (c->idx < 0 || SplitBetter(o.g, o.rf, c->g, c->rf) ||
                                   (!SplitBetter(c->g, c->rf, o.g, o.rf) && o.idx < c->idx));
  if (take) *c = o;
}

__device__ __forceinline__ ArgC ArgShflXor(const ArgC& c, int o) {
  ArgC r;
  r.g = __shfl_xor(c.g, o, kWave);
  r.rf = __shfl_xor(c.rf, o, kWave);
  r.idx = __shfl_xor(c.idx, o, kWave);
  r.x = __shfl_xor(c.x, o, kWave);
  return r;
}

// the wave's best candidate in ArgTake order (larger gain, NaN = -inf; smaller real feature;
// lower index): two 64-bit DPP max-reductions and a read of the winning lane instead of a
// butterfly of 4-field shuffles through the LDS crossbar
__device__ __forceinline__ ArgC ArgWaveBest(ArgC c) {
  const bool live = c.idx >= 0;
  const unsigned long long k1 = live ? GainKey(c.g) : 0ull;  // (GainKey(-inf) > 0: a live -inf still counts)
  const unsigned long long m1 = WaveMaxDpp(k1);
  if (m1 == 0ull) return ArgNone();
  const bool t1 = live && k1 == m1;
  const unsigned long long k2 = t1 ? ((static_cast<unsigned long long>(~static_cast<uint32_t>(c.rf)) << 32) |
                                      static_cast<unsigned long long>(~static_cast<uint32_t>(c.idx)))
                                   : 0ull;
  const unsigned long long m2 = WaveMaxDpp(k2);
  const int w = __builtin_amdgcn_readfirstlane(static_cast<int>(__builtin_ctzll(__ballot(t1 && k2 == m2))));
  ArgC r;
  r.g = ReadLane(c.g, w);
  r.rf = ReadLane(c.rf, w);
  r.idx = ReadLane(c.idx, w);
  r.x = ReadLane(c.x, w);
  return r;
}

// three independent wave argmaxes (the pick's two fresh children and the other leaves), each
// over DPP max-reductions of ordered keys (the butterfly of 4-field shuffles through the LDS
// crossbar this replaced cost ~5 us per pick even interleaved)
__device__ __forceinline__ void WaveArgBest3(ArgC* a, ArgC* b, ArgC* c) {
  *a = ArgWaveBest(*a);
  *b = ArgWaveBest(*b);
  *c = ArgWaveBest(*c);
}

// cat: the feature's category set (KArgs::feat_cat) when b is a categorical split
__device__ __forceinline__ void ToDeviceSplit(const FeatureBest& b, const uint32_t* cat, DeviceSplit* d) {
  d->gain = b.gain;
  d->feature = b.feature;
  d->real_feature = b.real_feature;
  d->threshold = b.thr;
  d->left_count = b.lc;
  d->right_count = b.rc;
  d->left_output = b.lo;
  d->right_output = b.ro;
  d->left_sum_gradient = b.lg;
  d->left_sum_hessian = b.lh;
  d->right_sum_gradient = b.rg;
  d->right_sum_hessian = b.rh;
  d->default_left = static_cast<int8_t>(b.default_left);
  d->monotone_type = static_cast<int8_t>(b.mono);
  d->is_categorical = b.ncat > 0 ? 1 : 0;
  d->pad0 = 0;
  d->num_cat_threshold = b.ncat;
  if (b.ncat > 0) {
    for (int w = 0; w < kMaxCatWords; ++w) d->cat_bits[w] = cat[w];
  }
}

// per-feature results of side (0 smaller, 1 larger) for inner feature f (distributed
// learners: rank-major blocks, gathered from every rank after the scans)
__device__ __forceinline__ size_t FeatBestIndex(const KArgs& a, int side, int f) {
  if (a.fb_index != nullptr) return static_cast<size_t>(a.fb_index[f]) + static_cast<size_t>(side) * a.fb_side;
  return static_cast<size_t>(side) * a.p.num_features + f;
}
__device__ __forceinline__ const uint32_t* FeatCat(const KArgs& a, int side, int f) {
  return a.feat_cat + FeatBestIndex(a, side, f) * kMaxCatWords;
}

__device__ __forceinline__ void NoSplit(DeviceSplit* d) {
  d->gain = -INFINITY;
  d->feature = -1;
  d->real_feature = -1;
}

struct PickResult {
  int done;
  int forced;  // the split is forced node s (reference ForceSplits)
  int s, leaf;
  int fresh_idx[2];  // winning feature of the fresh children (-1: none)
  Leaf P;
  Feature F;
  DeviceSplit split;
};

// workgroup-shared state of one pick.  Every global record the pick reads is copied into it
// first (lane-parallel word copies, loads only), the decisions are made on the LDS copies and
// every global write comes last: loads and stores of one wave complete in issue order, so an
// interleaved copy would wait for each store before the next load.
struct PickLds {
  PickResult pk;
  int s, fresh, sm, lg;        // the step's bookkeeping (nsplit, fresh sides, smaller / larger leaf)
  int sm_frow, lg_frow;
  int win_feature;             // the winner's inner feature (-1: none)
  int new_frow;                // splittable row of leaf s + 1 (the new leaf of the next split)
  FeatureBest fb[2];           // the fresh children's winning per-feature results
  uint32_t fcat[2][kMaxCatWords];
  DeviceSplit fsplit[2];       // ... as split records
  ChildStats lc, rc;
  IcMask icm;
  FeatureBest ffb;  // the forced split's record and category set
  uint32_t ffcat[kMaxCatWords];
  int forced_rank;  // feature-parallel: the rank whose forced record is valid (the feature's owner)
};
// the forced record of node s as rank r wrote it (KArgs::forced_world ranks, or this process)
__device__ __forceinline__ const FeatureBest& ForcedRecord(const KArgs& a, int r, int s) {
  return a.forced_world > 1 ? a.forced_all[static_cast<size_t>(r) * a.forced_n + s] : a.forced_best[s];
}
__device__ __forceinline__ const uint32_t* ForcedCat(const KArgs& a, int r, int s) {
  return a.forced_world > 1 ? a.forced_cat_all + (static_cast<size_t>(r) * a.forced_n + s) * kMaxCatWords
                            : a.forced_cat + static_cast<size_t>(s) * kMaxCatWords;
}

template <typename T>
__device__ __forceinline__ void CopyWords(const T* src, T* dst, int lane, int lanes) {
  static_assert(sizeof(T) % 4 == 0, "word copy");
  const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
  uint32_t* d = reinterpret_cast<uint32_t*>(dst);
  for (int i = lane; i < static_cast<int>(sizeof(T) / 4); i += lanes) d[i] = s[i];
}

// 1. the step's bookkeeping (one thread): every load, then every store
__device__ __forceinline__ void StepBookkeeping(const KArgs& a, Step* st, PickLds* pl) {
  const ChildInfo c = StepChildren(a, st);
  const CurSplit& cs = st->cs;
  const int leaf = cs.leaf, nl = cs.new_leaf, s = cs.s;
  const int pb = cs.part_begin, pc = cs.part_count, src_buf = cs.src_buf;
  const int parent_slot = cs.parent_slot, new_frow = cs.new_frow, parent_frow = cs.parent_frow;
  const int hist_left = st->hist_left;
  const int bynode_next = st->bynode_next;
  // ---- stores
  Leaf* P = &a.leaves[leaf];
  Leaf* R = &a.leaves[nl];
  P->begin = pb;
  P->count = c.total_left;
  R->begin = pb + c.total_left;
  R->count = pc - c.total_left;
  P->buf = 1 - src_buf;
  R->buf = 1 - src_buf;
  if (!a.p.data_parallel) {
    P->global_count = c.left_count;
    R->global_count = c.right_count;
    SplitRecord& rec = a.rec[s];
    rec.left_count = c.left_count;
    rec.right_count = c.right_count;
  }
  // the histogrammed child took the new leaf's slot, the other one the parent's (StepSide)
  P->slot = hist_left ? nl : parent_slot;
  R->slot = hist_left ? parent_slot : nl;
  // the splittable rows follow the smaller child (the host swaps its rows too)
  const bool swap = !c.skip && c.small_is_left;
  if (swap) {
    P->frow = new_frow;
    R->frow = parent_frow;
  }
  const int pf = swap ? new_frow : parent_frow, rf = swap ? parent_frow : new_frow;
  a.best[leaf].gain = -INFINITY;
  a.best[leaf].feature = -1;
  a.best[leaf].real_feature = -1;
  a.best[nl].gain = -INFINITY;
  a.best[nl].feature = -1;
  a.best[nl].real_feature = -1;
  st->smaller = c.smaller;
  st->larger = c.larger;
  if (!c.skip) {  // the host learner samples the smaller, then the larger child
    st->bynode_base = bynode_next;
    st->bynode_next = bynode_next + 2;
  }
  st->fresh = c.skip ? 0 : 2;
  st->nsplit = s + 1;
  pl->s = s + 1;
  pl->fresh = c.skip ? 0 : 2;
  pl->sm = c.smaller;
  pl->lg = c.larger;
  pl->sm_frow = c.small_is_left ? pf : rf;
  pl->lg_frow = c.small_is_left ? rf : pf;
}

// 2. the pick, by the first wave, from the bookkeeping in LDS; loads only
__device__ __forceinline__ void PickWave(const KArgs& a, PickLds* pl) {
  const int lane = threadIdx.x;
  const int L = a.p.num_leaves, NF = a.p.num_features;
  const int s = pl->s, fresh = pl->fresh, sm = pl->sm, lg = pl->lg;
  PickResult* out = &pl->pk;
  if (s >= L - 1) {
    if (lane == 0) {
      out->done = 1;
      out->s = s;
    }
    return;
  }
  // every input in one round of loads: lanes take (side, feature) items of the fresh sides
  // and leaves 0..s; then the two per-side feature argmaxes and the argmax over the other
  // leaves in one interleaved reduction; the fresh children join the leaf argmax last (the
  // order is total, so folding them in afterwards picks the same leaf as one pass)
  // the next new leaf's splittable row (leaf s + 1: untouched by the bookkeeping), with the
  // pick's other loads instead of after the pick
  const int pre_frow = (lane == 0 && s + 1 < L) ? a.leaves[s + 1].frow : 0;
  double lgv = -INFINITY;  // this lane's leaf (l = lane, the common case s < 64), loaded first
  int lrf = -1, lfv = -1;
  if (lane <= s && lane < L) {
    lgv = a.best[lane].gain;
    lrf = a.best[lane].real_feature;
    lfv = a.best[lane].feature;
  }
  ArgC c0 = ArgNone(), c1 = ArgNone();  // this lane's best feature of side 0 / 1
  const int nitems = fresh * NF;
  if (nitems <= kWave) {  // one item per lane
    const int side_of_lane = lane < NF ? 0 : 1;
    const int i = lane - side_of_lane * NF;
    if (lane < nitems) {
      const FeatureBest& fbv = a.feat_best[FeatBestIndex(a, side_of_lane, i)];
      const double cg = fbv.gain;
      const int crf = fbv.real_feature, cf = fbv.feature;
      if (cf >= 0) {  // (no reference to c0 / c1 chosen at run time: it would put both in scratch)
        ArgC c;
        c.g = cg;
        c.rf = crf;
        c.idx = i;
        c.x = -1;
        if (side_of_lane == 0) c0 = c;
        else c1 = c;
      }
    }
  } else {
    // many features: strided per lane, kPickBatch independent loads in flight per round
    // trip (a rolled one-load loop costs a memory round trip per 64 features: ~60 us for
    // 2 x 2000 features)
    constexpr int kPickBatch = 8;
#pragma unroll 1
    for (int side = 0; side < fresh; ++side) {
      ArgC c = ArgNone();
#pragma unroll 1
      for (int i0 = lane; i0 < NF; i0 += kPickBatch * kWave) {
        double cg[kPickBatch];
        int crf[kPickBatch], cf[kPickBatch];
#pragma unroll
        for (int k = 0; k < kPickBatch; ++k) {
          const int i = i0 + k * kWave;
          cf[k] = -1;
          if (i < NF) {
            const FeatureBest& fbv = a.feat_best[FeatBestIndex(a, side, i)];
            cg[k] = fbv.gain;
            crf[k] = fbv.real_feature;
            cf[k] = fbv.feature;
          }
        }
#pragma unroll
        for (int k = 0; k < kPickBatch; ++k) {  // ascending feature order, as a rolled loop
          if (cf[k] >= 0 && (c.idx < 0 || SplitBetter(cg[k], crf[k], c.g, c.rf))) {
            c.g = cg[k];
            c.rf = crf[k];
            c.idx = i0 + k * kWave;
          }
        }
      }
      if (side == 0) c0 = c;
      else c1 = c;
    }
  }
  // the leaves other than the fresh children (their records are final); the winner's inner
  // feature travels with it
  ArgC cl = ArgNone();
#pragma unroll 1
  for (int l = lane; l <= s && l < L; l += kWave) {
    if ((fresh >= 1 && l == sm) || (fresh == 2 && l == lg)) continue;
    double cg;
    int crf, cf;
    if (l == lane) {
      cg = lgv;
      crf = lrf;
      cf = lfv;
    } else {
      cg = a.best[l].gain;
      crf = a.best[l].real_feature;
      cf = a.best[l].feature;
    }
    if (cl.idx < 0 || SplitBetter(cg, crf, cl.g, cl.rf)) {
      cl.g = cg;
      cl.rf = crf;
      cl.idx = l;
      cl.x = cf;
    }
  }
  WaveArgBest3(&c0, &c1, &cl);
  if (c0.idx >= 0 && c0.g == -INFINITY) c0.idx = -1;  // no valid threshold on any feature
  if (c1.idx >= 0 && c1.g == -INFINITY) c1.idx = -1;
  const int fi0 = c0.idx, fi1 = c1.idx;
  if (a.ktrace != nullptr && lane == 0 && s - 1 >= 0) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    a.ktrace[(s - 1) * kTraceSlots + kTrPW1] = wall_clock64();
  }
  // the leaf to split: the fresh children's bests join the other leaves' winner
  ArgC win = cl;
  if (fresh >= 1) {
    ArgC f;
    f.g = fi0 >= 0 ? c0.g : -INFINITY;
    f.rf = fi0 >= 0 ? c0.rf : -1;
    f.idx = sm;
    f.x = fi0;
    ArgTake(&win, f);
  }
  if (fresh == 2) {
    ArgC f;
    f.g = fi1 >= 0 ? c1.g : -INFINITY;
    f.rf = fi1 >= 0 ? c1.rf : -1;
    f.idx = lg;
    f.x = fi1;
    ArgTake(&win, f);
  }
  if (lane != 0) return;
  pl->new_frow = pre_frow;
  const double g = win.g;
  const int leaf = win.idx, wf = win.x;
  if (a.ktrace != nullptr && s - 1 >= 0) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    a.ktrace[(s - 1) * kTraceSlots + kTrPW2] = wall_clock64();
  }
  out->s = s;
  out->leaf = leaf;
  out->fresh_idx[0] = fi0;
  out->fresh_idx[1] = fi1;
  pl->win_feature = wf;
  out->done = (g > 0.0 && wf >= 0) ? 0 : 1;
  out->forced = 0;
  // forced splits: node s, while every earlier one was valid; an invalid one ends them and
  // the normal pick above stands (reference ForceSplits' abort)
  if (s < a.forced_n && !a.st->forced_abort) {
    // (feature-parallel: only the owner of the node's feature scanned it -- the other ranks'
    // records are the tree's reset ones)
    int fr = -1;
    for (int r = 0; r < max(1, a.forced_world) && fr < 0; ++r) {
      const FeatureBest& fb = ForcedRecord(a, r, s);
      if (fb.feature >= 0 && fb.gain > -INFINITY && fb.lc + fb.rc > 0) fr = r;  // (an all-zero record: nobody's)
    }
    if (fr >= 0) {
      out->forced = 1;
      out->leaf = a.forced_leaf[s];
      pl->win_feature = ForcedRecord(a, fr, s).feature;
      pl->forced_rank = fr;
      out->done = 0;
    } else {
      a.st->forced_abort = 1;
    }
  }
}

// ---- intermediate monotone constraints (Params::mono_inter) --------------------------------
// The leaves the previous split re-bounded were re-scanned as sides 2.. of this step's split
// scans: their best splits (per-feature results, SplitInfo order) replace KArgs::best before
// the pick (SerialTreeLearner::RecomputeBestSplitForLeaf).  Every wave takes whole leaves.
__device__ void MonoInterFold(const KArgs& a) {
  const int n = a.mt_upd[0];
  const int nf = a.p.num_features, lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int k = w; k < n; k += nw) {
    const int u = a.mt_upd[1 + k];
    ArgC c = ArgNone();
    for (int f = lane; f < nf; f += kWave) {
      const FeatureBest& fb = a.feat_best[FeatBestIndex(a, 2 + k, f)];
      if (fb.feature >= 0 && (c.idx < 0 || SplitBetter(fb.gain, fb.real_feature, c.g, c.rf))) {
        c.g = fb.gain;
        c.rf = fb.real_feature;
        c.idx = f;
      }
    }
#pragma unroll 1
    for (int o = 32; o > 0; o >>= 1) ArgTake(&c, ArgShflXor(c, o));
    if (lane == 0) {
      if (c.idx >= 0 && c.g != -INFINITY) {
        ToDeviceSplit(a.feat_best[FeatBestIndex(a, 2 + k, c.idx)], FeatCat(a, 2 + k, c.idx), &a.best[u]);
      } else {
        NoSplit(&a.best[u]);
      }
    }
  }
}

// After the pick of split s (leaf -> leaf, s + 1): the reference's intermediate method
// (monotone_constraints.hpp IntermediateLeafConstraints; host LeafConstraints::BeforeSplit /
// Update / GoUp / GoDown) on the tree so far, walked by one thread in LDS: the children bound
// each other by their outputs (inside a monotone subtree), and at every monotone ancestor the
// leaves of the other subtree that can touch the new leaves are re-bounded by the new outputs;
// those whose bound changed are re-scanned by the next split scan.  Leaves that will not split
// (best gain -inf) keep their bounds.
__device__ void MonoInterUpdate(const KArgs& a, PickLds* pl, unsigned char* lds_raw) {
  PickResult* pk = &pl->pk;
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int L = a.p.num_leaves, s = pk->s, leaf = pk->leaf, nl = s + 1;
  int* lpar = reinterpret_cast<int*>(lds_raw);
  int* npar = lpar + L;
  int* nlc = npar + L;
  int* nrc = nlc + L;
  int* nfeat = nrc + L;
  int* nthv = nfeat + L;
  int* nnum = nthv + L;
  int* nmono = nnum + L;
  int* insub = nmono + L;
  int* dead = insub + L;
  int* pf = dead + L;
  int* pt = pf + L;
  int* pr = pt + L;
  int* seen = pr + L;
  int* stale = seen + L;      // [L + 1]: count, then leaves
  int* stk = stale + L + 1;   // [3 L]
  double* cmn = reinterpret_cast<double*>(lds_raw + ((static_cast<size_t>(19 * L + 1) * sizeof(int) + 7) & ~size_t(7)));
  double* cmx = cmn + L;
  // the tree so far (nodes 0..s-1, leaves 0..s), in LDS
  for (int i = tid; i <= s; i += nthr) {
    lpar[i] = a.mt_leaf_parent[i];
    insub[i] = a.mt_in_sub[i];
    dead[i] = a.best[i].gain == -INFINITY ? 1 : 0;
    cmn[i] = a.leaves[i].cmin;
    cmx[i] = a.leaves[i].cmax;
    seen[i] = 0;
    if (i < s) {
      npar[i] = a.mt_node[3 * i];
      nlc[i] = a.mt_node[3 * i + 1];
      nrc[i] = a.mt_node[3 * i + 2];
      const DeviceSplit& r = a.rec[i].split;
      nfeat[i] = r.feature;
      nthv[i] = r.threshold;
      nnum[i] = r.is_categorical ? 0 : 1;
    }
  }
  __syncthreads();
  for (int i = tid; i < s; i += nthr) nmono[i] = a.feat[nfeat[i]].monotone;
  // (the previous step's fresh children: their bests are in pl->fsplit until step 5 stores them)
  if (tid == 0) {
    if (pl->fresh >= 1 && pl->sm >= 0) dead[pl->sm] = pl->fsplit[0].gain == -INFINITY ? 1 : 0;
    if (pl->fresh == 2 && pl->lg >= 0) dead[pl->lg] = pl->fsplit[1].gain == -INFINITY ? 1 : 0;
  }
  __syncthreads();
  if (tid == 0) {
    const DeviceSplit& sp = pk->split;
    const int mono = sp.monotone_type;
    const bool numerical = !sp.is_categorical;
    // BeforeSplit, then Tree::Split
    if (mono != 0 || insub[leaf]) {
      insub[leaf] = 1;
      insub[nl] = 1;
    } else {
      insub[nl] = 0;
    }
    const int parent = lpar[leaf];
    npar[s] = parent;
    if (parent >= 0) {
      if (nlc[parent] == ~leaf) nlc[parent] = s;
      else nrc[parent] = s;
    }
    nlc[s] = ~leaf;
    nrc[s] = ~nl;
    lpar[leaf] = s;
    lpar[nl] = s;
    nfeat[s] = sp.feature;
    nthv[s] = sp.threshold;
    nnum[s] = numerical ? 1 : 0;
    nmono[s] = pk->F.monotone;
    int nst = 0;
    double lmin = cmn[leaf], lmax = cmx[leaf], rmin = -DBL_MAX, rmax = DBL_MAX;
    if (insub[leaf]) {
      rmin = lmin;
      rmax = lmax;
      if (numerical) {
        if (mono < 0) {
          lmin = fmax(lmin, sp.right_output);
          rmax = fmin(rmax, sp.left_output);
        } else if (mono > 0) {
          lmax = fmin(lmax, sp.right_output);
          rmin = fmax(rmin, sp.left_output);
        }
      }
      const double lo_out = sp.left_output, ro_out = sp.right_output;
      const uint32_t sthr = static_cast<uint32_t>(sp.threshold);
      const int sinner = sp.feature;
      // GoUp from the new node
      int node = s, plen = 0;
      for (;;) {
        const int par = npar[node];
        if (par < 0) break;
        const int inner = nfeat[par], pmono = nmono[par];
        const int from_right = nrc[par] == node ? 1 : 0;
        bool relevant = true;
        if (nnum[node]) {
          for (int i = 0; i < plen; ++i) {
            if (pf[i] == inner && pr[i] == from_right) {
              relevant = false;
              break;
            }
          }
        }
        if (relevant) {
          if (pmono != 0) {
            const bool node_is_left = nlc[par] == node;
            const bool update_max = pmono < 0 ? node_is_left : !node_is_left;
            // GoDown over the other subtree (explicit stack: node, use_left, use_right)
            int top = 0;
            stk[0] = node_is_left ? nrc[par] : nlc[par];
            stk[1] = 1;
            stk[2] = 1;
            top = 1;
            while (top > 0) {
              --top;
              const int nd = stk[3 * top], ul = stk[3 * top + 1], ur = stk[3 * top + 2];
              if (nd < 0) {
                const int lf = ~nd;
                if (dead[lf]) continue;
                double lo, hi;
                if (ul && ur) {
                  lo = fmin(ro_out, lo_out);
                  hi = fmax(ro_out, lo_out);
                } else if (ur) {
                  lo = hi = ro_out;
                } else {
                  lo = hi = lo_out;
                }
                bool changed = false;
                if (!update_max) {
                  if (hi > cmn[lf]) {
                    cmn[lf] = hi;
                    changed = true;
                  }
                } else if (lo < cmx[lf]) {
                  cmx[lf] = lo;
                  changed = true;
                }
                if (changed && !seen[lf]) {
                  seen[lf] = 1;
                  stale[1 + nst++] = lf;
                }
                continue;
              }
              const int inn = nfeat[nd];
              const uint32_t thr = static_cast<uint32_t>(nthv[nd]);
              const bool num = nnum[nd] != 0;
              bool go_left = true, go_right = true;
              if (num) {
                for (int i = 0; i < plen && (go_left || go_right); ++i) {
                  if (pf[i] != inn) continue;
                  if (thr >= static_cast<uint32_t>(pt[i]) && !pr[i]) go_right = false;
                  if (thr <= static_cast<uint32_t>(pt[i]) && pr[i]) go_left = false;
                }
              }
              bool left_for_right = true, right_for_left = true;
              if (num && inn == sinner) {
                if (thr >= sthr) left_for_right = false;
                if (thr <= sthr) right_for_left = false;
              }
              // (the reference recurses left, then right: pushed in reverse)
              if (go_right) {
                stk[3 * top] = nrc[nd];
                stk[3 * top + 1] = (left_for_right && ul) ? 1 : 0;
                stk[3 * top + 2] = ur;
                ++top;
              }
              if (go_left) {
                stk[3 * top] = nlc[nd];
                stk[3 * top + 1] = ul;
                stk[3 * top + 2] = (right_for_left && ur) ? 1 : 0;
                ++top;
              }
            }
          }
          pf[plen] = inner;
          pt[plen] = nthv[par];
          pr[plen] = from_right;
          ++plen;
        }
        node = par;
      }
    }
    pl->lc.cmin = lmin;
    pl->lc.cmax = lmax;
    pl->rc.cmin = rmin;
    pl->rc.cmax = rmax;
    stale[0] = nst;
  }
  __syncthreads();
  // stores: the re-bounded leaves and their list, the grown topology
  const int nst = stale[0];
  for (int k = tid; k < nst; k += nthr) {
    const int u = stale[1 + k];
    a.leaves[u].cmin = cmn[u];
    a.leaves[u].cmax = cmx[u];
    a.mt_upd[1 + k] = u;
  }
  if (tid == 0) {
    a.mt_upd[0] = nst;
    a.mt_leaf_parent[leaf] = s;
    a.mt_leaf_parent[nl] = s;
    a.mt_in_sub[leaf] = static_cast<int8_t>(insub[leaf]);
    a.mt_in_sub[nl] = static_cast<int8_t>(insub[nl]);
    a.mt_node[3 * s] = npar[s];
    a.mt_node[3 * s + 1] = nlc[s];
    a.mt_node[3 * s + 2] = nrc[s];
    const int parent = npar[s];
    if (parent >= 0) {
      a.mt_node[3 * parent + 1] = nlc[parent];
      a.mt_node[3 * parent + 2] = nrc[parent];
    }
  }
  __syncthreads();
}

// in-kernel stamp of the picking workgroup (LGBM_AMD_KTRACE)
__device__ __forceinline__ void PickTrace(const KArgs& a, int s, int slot) {
  if (a.ktrace != nullptr && threadIdx.x == 0 && s >= 0 && s < a.p.num_leaves) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    a.ktrace[s * kTraceSlots + slot] = wall_clock64();
  }
}

__device__ __forceinline__ void PickAndRecord(const KArgs& a, Step* st, bool root, PickLds* pl, int ts = -1,
                                              unsigned char* mono_lds = nullptr) {
  const int tid = threadIdx.x, lane = tid & 63, nthr = blockDim.x;
  PickResult* pk = &pl->pk;
  // 1. bookkeeping, by a thread outside the picking wave (its stores do not hold up the
  //    wave's loads; one-wave workgroups: by the wave's first thread, before the pick)
  if (root) {
    if (tid == 0) {
      // the tree's global root rows, on every rank (the scan of inner feature 0 publishes them
      // too, but a distributed rank that does not own that feature never runs it): the host
      // replays the tree's by-node / extra_trees draws only when the root was scanned
      st->root_count = static_cast<int>(a.root[2]);
      pl->s = 0;
      pl->fresh = 1;
      pl->sm = 0;
      pl->lg = -1;
      pl->sm_frow = -1;
      pl->lg_frow = -1;
    }
  } else if (tid == (nthr > kWave ? kWave : 0)) {
    StepBookkeeping(a, st, pl);
  }
  __syncthreads();
  // intermediate monotone: the re-scanned leaves' new bests join the per-leaf table first
  if (a.p.mono_inter && !root) {
    MonoInterFold(a);
    __syncthreads();
  }
  PickTrace(a, ts, kTrPick1);
  if (a.ktrace != nullptr && tid == 0 && ts >= 0 && ts < a.p.num_leaves) a.ktrace[ts * kTraceSlots + kTrClk0] = __builtin_amdgcn_s_memtime();
  // 2. the pick
  if (tid < kWave) PickWave(a, pl);
  __syncthreads();
  PickTrace(a, ts, kTrPick2);
  if (a.ktrace != nullptr && a.p.trace_repeat) {  // diagnostics: the same pick again, warm
    if (tid < kWave) PickWave(a, pl);
    __syncthreads();
    PickTrace(a, ts, kTrPickRep);
  }
  if (pk->done) {
    if (tid == 0) {
      st->done = 1;
      st->nsplit = pk->s;
    }
  } else {
    // 3. records into LDS: the fresh children's winners, the winning leaf and feature
    const int fresh = pl->fresh, leaf = pk->leaf, w = tid >> 6;
    const int nw = nthr >> 6;
    const bool win_fresh = !pk->forced && ((fresh >= 1 && leaf == pl->sm) || (fresh == 2 && leaf == pl->lg));
    for (int side = 0; side < fresh; ++side) {
      if (w == (side % nw) && pk->fresh_idx[side] >= 0) {
        CopyWords(&a.feat_best[FeatBestIndex(a, side, pk->fresh_idx[side])], &pl->fb[side], lane, kWave);
        CopyWords(reinterpret_cast<const uint32_t(*)[kMaxCatWords]>(FeatCat(a, side, pk->fresh_idx[side])),
                  &pl->fcat[side], lane, kWave);
      }
    }
    if (pk->forced) {
      if (w == (2 % nw)) {
        CopyWords(&ForcedRecord(a, pl->forced_rank, pk->s), &pl->ffb, lane, kWave);
        CopyWords(reinterpret_cast<const uint32_t(*)[kMaxCatWords]>(ForcedCat(a, pl->forced_rank, pk->s)), &pl->ffcat,
                  lane, kWave);
      }
    } else if (!win_fresh && w == (2 % nw)) {
      CopyWords(&a.best[leaf], &pk->split, lane, kWave);
    }
    if (w == (3 % nw)) {
      CopyWords(&a.leaves[leaf], &pk->P, lane, kWave);
      CopyWords(&a.feat[pl->win_feature], &pk->F, lane, kWave);
    }
    __syncthreads();
    PickTrace(a, ts, kTrPick3);
    // 4. conversions (lane k: fresh side k, lane 2: the forced split -- side by side in one
    //    wave) and the children's statistics (thread 0), LDS only
    if (tid < fresh) {
      if (pk->fresh_idx[tid] >= 0) ToDeviceSplit(pl->fb[tid], pl->fcat[tid], &pl->fsplit[tid]);
      else NoSplit(&pl->fsplit[tid]);
    } else if (tid == 2 && pk->forced) {
      ToDeviceSplit(pl->ffb, pl->ffcat, &pk->split);
    }
    __syncthreads();
    if (tid == 0) {
      if (win_fresh) pk->split = pl->fsplit[leaf == pl->sm ? 0 : 1];
      const DeviceSplit& sp = pk->split;
      const Leaf& P = pk->P;
      const int s = pk->s, nl = s + 1;
      const int depth = P.depth + 1;
      double pmin = P.cmin, pmax = P.cmax, rmin = P.cmin, rmax = P.cmax;
      if (!sp.is_categorical) {
        const double mid = (sp.left_output + sp.right_output) / 2.0f;
        if (sp.monotone_type < 0) {
          pmin = fmax(pmin, mid);
          rmax = fmin(rmax, mid);
        } else if (sp.monotone_type > 0) {
          pmax = fmin(pmax, mid);
          rmin = fmax(rmin, mid);
        }
      }
      ChildStats& lc = pl->lc;
      ChildStats& rc = pl->rc;
      lc.sum_g = sp.left_sum_gradient;
      lc.sum_h = sp.left_sum_hessian;
      lc.output = sp.left_output;
      lc.cmin = pmin;
      lc.cmax = pmax;
      lc.global_count = sp.left_count;
      lc.depth = depth;
      lc.slot = P.slot;
      lc.leaf = leaf;
      lc.frow = P.frow;
      rc.sum_g = sp.right_sum_gradient;
      rc.sum_h = sp.right_sum_hessian;
      rc.output = sp.right_output;
      rc.cmin = rmin;
      rc.cmax = rmax;
      rc.global_count = sp.right_count;
      rc.depth = depth;
      rc.slot = nl;
      rc.leaf = nl;
      rc.frow = -1;  // the new leaf's row (below)
    }
    __syncthreads();
    if (a.p.mono_inter && mono_lds != nullptr && !pk->forced) MonoInterUpdate(a, pl, mono_lds);
    PickTrace(a, ts, kTrPick4);
    // 5. loads that depend on the winner: the new leaf's splittable row id, the constraint
    //    mask of the split feature (the parent's splittable row is snapshot by k_split)
    const DeviceSplit& sp = pk->split;
    const int s = pk->s, nl = s + 1;
    const int new_frow = pl->new_frow;
    IcMask fmask = kIcAll;
    if (tid == 0 && a.feat_icmask != nullptr) fmask = a.feat_icmask[sp.feature];
    // ---- stores only from here
    // the fresh children's bests become part of the per-leaf table
    for (int side = 0; side < fresh; ++side) {
      const int l = side == 0 ? pl->sm : pl->lg;
      CopyWords(&pl->fsplit[side], &a.best[l], tid, nthr);
    }
    if (a.p.cegb && a.cegb_coupled != nullptr) {
      // CEGB (CostEffectiveGB::OnSplit): the winner's feature is used by the model from now on;
      // the other leaves' remembered candidates on it get its coupled penalty back and replace
      // their best split if they now beat it
      __syncthreads();
      const int f = sp.feature;
      const bool first_use = f >= 0 && !a.cegb_used[f];
      __syncthreads();
      if (first_use) {
        if (tid == 0) a.cegb_used[f] = 1;
        const double refund = a.cegb_coupled[f];
        const int nf = a.p.num_features;
        for (int i = tid; i < s + 1; i += nthr) {
          if (i == leaf) continue;
          const size_t mi = static_cast<size_t>(i) * nf + f;
          FeatureBest cand = a.cegb_mem[mi];
          cand.gain += refund;
          DeviceSplit& cur = a.best[i];
          const int cf = cur.real_feature < 0 ? 0x7fffffff : cur.real_feature;
          const int nf_real = cand.feature < 0 ? 0x7fffffff : cand.real_feature;
          if (cur.gain > -INFINITY && (cand.gain > cur.gain || (cand.gain == cur.gain && nf_real < cf))) {
            ToDeviceSplit(cand, a.cegb_mem_cat + mi * kMaxCatWords, &cur);
          }
        }
      }
    }
    CopyWords(&pk->split, &a.rec[s].split, tid, nthr);
    CopyWords(&pk->split, &st->cs.split, tid, nthr);
    CopyWords(&pk->F, &st->cs.feat, tid, nthr);
    if (tid == 0) {
      const Leaf& P = pk->P;
      const IcMask icm = P.icmask & fmask;  // both children keep the constraints that hold the feature
      ChildStats lc = pl->lc, rc = pl->rc;
      lc.icmask = rc.icmask = icm;
      rc.frow = new_frow;
      SplitRecord& rec = a.rec[s];
      rec.leaf = leaf;
      rec.left_count = sp.left_count;
      rec.right_count = sp.right_count;
      Leaf* PL = &a.leaves[leaf];
      Leaf* RL = &a.leaves[nl];
      PL->depth = lc.depth;
      PL->sum_g = lc.sum_g;
      PL->sum_h = lc.sum_h;
      PL->output = lc.output;
      PL->global_count = lc.global_count;
      PL->cmin = lc.cmin;
      PL->cmax = lc.cmax;
      RL->depth = rc.depth;
      RL->sum_g = rc.sum_g;
      RL->sum_h = rc.sum_h;
      RL->output = rc.output;
      RL->global_count = rc.global_count;
      RL->cmin = rc.cmin;
      RL->cmax = rc.cmax;
      PL->icmask = RL->icmask = icm;
      st->lr[0] = lc;
      st->lr[1] = rc;
      CurSplit& cs = st->cs;
      cs.s = s;
      cs.leaf = leaf;
      cs.new_leaf = nl;
      cs.part_begin = P.begin;
      cs.part_count = P.count;
      cs.src_buf = P.buf;
      cs.child_depth = lc.depth;
      cs.parent_slot = P.slot;
      cs.parent_frow = P.frow;
      cs.new_frow = new_frow;
      cs.plsum_g = P.lsum_g;
      cs.plsum_h = P.lsum_h;
      // k_split histograms the child with fewer rows by the estimated counts
      st->hist_left = sp.left_count <= sp.right_count ? 1 : 0;
    }
  }
  if (tid == 0) {
    st->cur_left = 0;  // the next k_split's partition cursors
    st->cur_right = 0;
    st->find_count = 0u;
    st->loc_acc[0] = 0ull;  // voting: the next k_split's local sums
    st->loc_acc[1] = 0ull;
  }
}

}  // namespace dev
}  // namespace lgbm_amd
