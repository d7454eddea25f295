// Split selection + data partition (reference serial_tree_learner.cpp Train / Split,
// FindBestSplitsFromHistograms' per-leaf argmax, src/treelearner/data_partition.hpp Split,
// monotone_constraints.hpp BasicLeafConstraints).
//
// k_partition, device mode, split s:
//  1. pick (first wave of every workgroup, redundantly -- no extra launch, no cross-
//     workgroup hand-off): the per-leaf best split of the children that were just scanned
//     (argmax over their per-feature results, SplitInfo order), then the leaf to split
//     (argmax over all leaves: higher gain, smaller real feature, lower leaf id -- the host
//     loop's order).  All loads of the pick are independent of each other (one round trip)
//     except the winner's records (a second one).  Workgroup 0 records the split (Step::cs,
//     SplitRecord, children statistics, per-leaf bests).
//  2. partition: the leaf's index range [begin, +count) of its buffer is moved into the same
//     range of the other buffer, lefts growing up from the front and rights down from the
//     back.  Each 8192-row tile reserves its output slots with one device-scope atomic per
//     side (no grid-wide prefix pass); rows keep their order inside a tile, tiles land in
//     arrival order -- histograms are exact integer sums, so the row order never changes a
//     result.  The cursors' final values are the children's sizes (StepChildren).  Rows are
//     read from the column-major copy of the split column (1 byte per row).
// Host mode: the host wrote Step::cs; only step 2 runs.
#include "device_common.h"

namespace lgbm_amd {
namespace dev {

namespace {

__device__ __forceinline__ void MakeRule(const DeviceSplit& sp, const Feature& f, SplitRule* r,
                                         uint32_t* cat_bits_lds) {
  r->threshold = sp.threshold;
  r->default_left = sp.default_left;
  r->is_cat = sp.is_categorical;
  r->missing_type = f.missing_type;
  r->default_bin = f.default_bin;
  r->max_bin = f.num_bin - 1;
  if (sp.is_categorical) {
    for (int i = threadIdx.x; i < kMaxCatWords; i += blockDim.x) cat_bits_lds[i] = sp.cat_bits[i];
  }
}

// argmax over (gain, real feature, index) in SplitInfo order; ties on both -> lower index
__device__ __forceinline__ void WaveArgBest(double* g, int* rf, int* idx) {
  for (int o = 32; o > 0; o >>= 1) {
    const double og = __shfl_xor(*g, o, kWave);
    const int orf = __shfl_xor(*rf, o, kWave);
    const int oi = __shfl_xor(*idx, o, kWave);
    const bool take = oi >= 0 && (*idx < 0 || SplitBetter(og, orf, *g, *rf) ||
                                  (!SplitBetter(*g, *rf, og, orf) && oi < *idx));
    if (take) {
      *g = og;
      *rf = orf;
      *idx = oi;
    }
  }
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

__device__ __forceinline__ const uint32_t* FeatCat(const KArgs& a, int side, int f) {
  return a.feat_cat + (static_cast<size_t>(side) * a.p.num_features + f) * kMaxCatWords;
}

__device__ __forceinline__ void NoSplit(DeviceSplit* d) {
  d->gain = -INFINITY;
  d->feature = -1;
  d->real_feature = -1;
}

struct PickResult {
  int done;
  int s, leaf;
  int fresh_idx[2];  // winning feature of the fresh children (-1: none)
  Leaf P;
  Feature F;
  DeviceSplit split;
};

// the pick, by the first wave; the result goes to LDS.  Every load that does not depend on
// another one is issued first (Step, both sides' per-feature results, every leaf's best
// gain): one round trip, then one more for the winner's records.
__device__ void PickWave(const KArgs& a, const Step* st, PickResult* out) {
  const int lane = threadIdx.x;
  const int L = a.p.num_leaves, NF = a.p.num_features;
  const int s = st->nsplit;
  const int fresh = st->fresh;
  const int sm = st->smaller, lg = st->larger;
  // per-feature candidates of both sides (lane-strided) and per-leaf candidates
  double g0 = -INFINITY, g1 = -INFINITY;
  int rf0 = -1, rf1 = -1, i0 = -1, i1 = -1;
  for (int i = lane; i < NF; i += kWave) {
    const FeatureBest& b0 = a.feat_best[i];
    const FeatureBest& b1 = a.feat_best[NF + i];
    const double cg0 = b0.gain, cg1 = b1.gain;
    const int crf0 = b0.real_feature, crf1 = b1.real_feature;
    const int cf0 = b0.feature, cf1 = b1.feature;
    if (cf0 >= 0 && (i0 < 0 || SplitBetter(cg0, crf0, g0, rf0))) {
      g0 = cg0;
      rf0 = crf0;
      i0 = i;
    }
    if (cf1 >= 0 && (i1 < 0 || SplitBetter(cg1, crf1, g1, rf1))) {
      g1 = cg1;
      rf1 = crf1;
      i1 = i;
    }
  }
  double lgain[kMaxLeaves / kWave];
  int lrf[kMaxLeaves / kWave];
#pragma unroll
  for (int k = 0; k < kMaxLeaves / kWave; ++k) {
    const int l = lane + k * kWave;
    if (l < L) {
      lgain[k] = a.best[l].gain;
      lrf[k] = a.best[l].real_feature;
    }
  }
  if (s >= L - 1) {
    if (lane == 0) {
      out->done = 1;
      out->s = s;
    }
    return;
  }
  // per-leaf bests of the freshly scanned children
  int fi[2] = {-1, -1};
  double fg[2] = {-INFINITY, -INFINITY};
  int frf[2] = {-1, -1};
  if (fresh >= 1) {
    WaveArgBest(&g0, &rf0, &i0);
    if (i0 >= 0 && g0 == -INFINITY) i0 = -1;  // no valid threshold on any feature
    fi[0] = i0;
    fg[0] = i0 >= 0 ? g0 : -INFINITY;
    frf[0] = i0 >= 0 ? rf0 : -1;
  }
  if (fresh == 2) {
    WaveArgBest(&g1, &rf1, &i1);
    if (i1 >= 0 && g1 == -INFINITY) i1 = -1;
    fi[1] = i1;
    fg[1] = i1 >= 0 ? g1 : -INFINITY;
    frf[1] = i1 >= 0 ? rf1 : -1;
  }
  // the leaf to split: argmax over leaves 0..s (fresh children use the new results)
  double g = -INFINITY;
  int rf = -1, leaf = -1;
#pragma unroll
  for (int k = 0; k < kMaxLeaves / kWave; ++k) {
    const int l = lane + k * kWave;
    if (l > s) continue;
    double cg = lgain[k];
    int crf = lrf[k];
    if (fresh >= 1 && l == sm) {
      cg = fg[0];
      crf = frf[0];
    } else if (fresh == 2 && l == lg) {
      cg = fg[1];
      crf = frf[1];
    }
    if (leaf < 0 || SplitBetter(cg, crf, g, rf)) {
      g = cg;
      rf = crf;
      leaf = l;
    }
  }
  WaveArgBest(&g, &rf, &leaf);
  if (lane != 0) return;
  out->s = s;
  out->leaf = leaf;
  out->fresh_idx[0] = fi[0];
  out->fresh_idx[1] = fi[1];
  DeviceSplit* sp = &out->split;  // straight into LDS (no private copy)
  if (fresh >= 1 && leaf == sm) {
    if (fi[0] >= 0) ToDeviceSplit(a.feat_best[fi[0]], FeatCat(a, 0, fi[0]), sp);
    else NoSplit(sp);
  } else if (fresh == 2 && leaf == lg) {
    if (fi[1] >= 0) ToDeviceSplit(a.feat_best[NF + fi[1]], FeatCat(a, 1, fi[1]), sp);
    else NoSplit(sp);
  } else {
    *sp = a.best[leaf];
  }
  if (!(sp->gain > 0.0) || sp->feature < 0) {
    out->done = 1;
    return;
  }
  out->done = 0;
  out->P = a.leaves[leaf];
  out->F = a.feat[sp->feature];
}

// workgroup 0, one thread: record the split for the later kernels and future picks
__device__ void RecordSplit(const KArgs& a, Step* st, const PickResult& pk) {
  const int fresh = st->fresh;
  const int NF = a.p.num_features;
  // the fresh children's bests become part of the per-leaf table
  for (int side = 0; side < fresh; ++side) {
    const int l = side == 0 ? st->smaller : st->larger;
    DeviceSplit& d = a.best[l];
    if (pk.fresh_idx[side] >= 0) {
      ToDeviceSplit(a.feat_best[side * NF + pk.fresh_idx[side]], FeatCat(a, side, pk.fresh_idx[side]), &d);
    }
    else NoSplit(&d);
  }
  const int s = pk.s, leaf = pk.leaf, nl = s + 1;
  const DeviceSplit& sp = pk.split;
  SplitRecord& rec = a.rec[s];
  rec.leaf = leaf;
  rec.split = sp;
  rec.left_count = sp.left_count;
  rec.right_count = sp.right_count;
  // children statistics (left keeps the leaf id); ranges are set after the partition
  const Leaf& P = pk.P;
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
  // both children keep the constraints that also hold the split feature
  const uint32_t icm = a.feat_icmask != nullptr ? P.icmask & a.feat_icmask[sp.feature] : 0xffffffffu;
  ChildStats lc, rc;
  lc.icmask = rc.icmask = icm;
  lc.sum_g = sp.left_sum_gradient;
  lc.sum_h = sp.left_sum_hessian;
  lc.output = sp.left_output;
  lc.cmin = pmin;
  lc.cmax = pmax;
  lc.global_count = sp.left_count;
  lc.depth = depth;
  lc.slot = P.slot;
  lc.leaf = leaf;
  rc.sum_g = sp.right_sum_gradient;
  rc.sum_h = sp.right_sum_hessian;
  rc.output = sp.right_output;
  rc.cmin = rmin;
  rc.cmax = rmax;
  rc.global_count = sp.right_count;
  rc.depth = depth;
  rc.slot = nl;  // a new leaf's slot is its own id (k_tree_begin)
  rc.leaf = nl;
  Leaf* PL = &a.leaves[leaf];
  Leaf* RL = &a.leaves[nl];
  PL->depth = depth;
  PL->sum_g = lc.sum_g;
  PL->sum_h = lc.sum_h;
  PL->output = lc.output;
  PL->global_count = lc.global_count;
  PL->cmin = pmin;
  PL->cmax = pmax;
  RL->depth = depth;
  RL->sum_g = rc.sum_g;
  RL->sum_h = rc.sum_h;
  RL->output = rc.output;
  RL->global_count = rc.global_count;
  RL->cmin = rmin;
  RL->cmax = rmax;
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
  cs.child_depth = depth;
  cs.parent_slot = P.slot;
  cs.parent_frow = P.frow;
  cs.new_frow = a.leaves[nl].frow;
  cs.feat = pk.F;
  cs.split = sp;
}

}  // namespace

__global__ __launch_bounds__(kPartThreads) void k_partition(KArgs a) {
  __shared__ uint32_t cat_bits[kMaxCatWords];
  __shared__ int wl[kPartRowsPerThread][kPartThreads / kWave];
  __shared__ int base[2];
  __shared__ PickResult pk;
  const long long t_entry = wall_clock64();
  Step* st = a.st;
  if (st->done) return;
  int pb, pc, src_buf;
  const DeviceSplit* spp;
  const Feature* fp;
  if (a.host_mode) {
    pb = st->cs.part_begin;
    pc = st->cs.part_count;
    src_buf = st->cs.src_buf;
    spp = &st->cs.split;
    fp = &st->cs.feat;
  } else {
    if (threadIdx.x < kWave) PickWave(a, st, &pk);
    __syncthreads();
    if (pk.done) {
      if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
        st->done = 1;
        st->nsplit = pk.s;
      }
      return;
    }
    // recorded by the last workgroup: it has no rows to move unless the leaf is large
    if (blockIdx.x == gridDim.x - 1) {
      if (threadIdx.x == 0) RecordSplit(a, st, pk);
      // the parent's splittable row, before the children's scans overwrite it
      const int8_t* row = a.splittable + static_cast<size_t>(pk.P.frow) * a.p.num_features;
      for (int f = threadIdx.x; f < a.p.num_features; f += kPartThreads) a.parent_flags[f] = row[f];
    }
    KTraceAt(a, pk.s, kTrPartEntry, t_entry);
    KTrace(a, pk.s, kTrPartPicked);
    pb = pk.P.begin;
    pc = pk.P.count;
    src_buf = pk.P.buf;
    spp = &pk.split;
    fp = &pk.F;
  }
  const int32_t* src = src_buf ? a.tmp : a.idx;
  int32_t* dst = src_buf ? a.idx : a.tmp;
  const int ntiles = (pc + kPartTile - 1) / kPartTile;
  if (static_cast<int>(blockIdx.x) >= ntiles) return;
  const Feature F = *fp;
  SplitRule r;
  MakeRule(*spp, F, &r, cat_bits);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int nw = kPartThreads / kWave;
  const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int t0 = t * kPartTile;
    int row[kPartRowsPerThread];
#pragma unroll
    for (int k = 0; k < kPartRowsPerThread; ++k) {
      const int i = t0 + k * kPartThreads + threadIdx.x;
      row[k] = i < pc ? src[pb + i] : -1;
    }
    const int ts = a.host_mode ? -1 : (t == 0 ? pk.s : -1);
    KTrace(a, ts, kTrPartRows);
    uint32_t gb[kPartRowsPerThread];
#pragma unroll
    for (int k = 0; k < kPartRowsPerThread; ++k) gb[k] = row[k] >= 0 ? ColBin(a, row[k], F.group) : 0u;
    KTrace(a, ts, kTrPartBins);
    bool left[kPartRowsPerThread];
    unsigned long long mask[kPartRowsPerThread];
#pragma unroll
    for (int k = 0; k < kPartRowsPerThread; ++k) {
      left[k] = row[k] >= 0 && GoesLeft(r, cat_bits, FeatureBinOf(F, gb[k]));
      mask[k] = __ballot(left[k]);
    }
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < kPartRowsPerThread; ++k) wl[k][w] = __popcll(mask[k]);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int nl = 0;
      for (int k = 0; k < kPartRowsPerThread; ++k)
        for (int j = 0; j < nw; ++j) nl += wl[k][j];
      const int valid = min(kPartTile, pc - t0);
      if (ntiles == 1) {  // sole workgroup: no reservation round trip
        base[0] = base[1] = 0;
        st->cur_left = nl;
        st->cur_right = valid - nl;
      } else {
        base[0] = atomicAdd(&st->cur_left, nl);
        base[1] = atomicAdd(&st->cur_right, valid - nl);
      }
    }
    __syncthreads();
    const int lbase = pb + base[0];
    const int rbase = pb + pc - 1 - base[1];
    // rows are ordered (k, thread) inside the tile
    int sub_l = 0;
#pragma unroll
    for (int k = 0; k < kPartRowsPerThread; ++k) {
      int wbefore = 0, sub_tot = 0;
#pragma unroll
      for (int j = 0; j < nw; ++j) {
        const int c = wl[k][j];
        wbefore += j < w ? c : 0;
        sub_tot += c;
      }
      if (row[k] >= 0) {
        const int lpos = sub_l + wbefore + __popcll(mask[k] & lt);  // lefts before me in the tile
        const int pos = k * kPartThreads + threadIdx.x;             // my position in the tile
        if (left[k]) dst[lbase + lpos] = row[k];
        else dst[rbase - (pos - lpos)] = row[k];
      }
      sub_l += sub_tot;
    }
    __syncthreads();  // wl / base are rewritten by the next tile
  }
  if (!a.host_mode) KTrace(a, pk.s, kTrPartExit);
}

void Partition(const KArgs& a, hipStream_t s) {
  // one workgroup per CU: at most ~num_data / (kPartTile * CUs) tile reservations each
  const int grid = std::max(1, std::min((a.num_data + kPartTile - 1) / kPartTile, NumCUs()));
  hipLaunchKernelGGL(k_partition, dim3(grid), dim3(kPartThreads), 0, s, a);
}

}  // namespace dev
}  // namespace lgbm_amd
