// Split selection + data partition (reference serial_tree_learner.cpp Train/Split,
// src/treelearner/data_partition.hpp Split, monotone_constraints.hpp BasicLeafConstraints).
//
// k_select_count: every workgroup picks the best leaf (argmax over best[], ties -> lower
// leaf index, same order as the host loop) and counts the rows of its chunk that go left;
// workgroup 0 also records the split and the children's statistics.
// k_part_scatter: stable scatter of the leaf's index range into `tmp` (lefts first), plus
// the children's ranges, the smaller/larger choice and the histogram-slot hand-over.
// Rows are read from the column-major copy of the split column (1 byte per row).
#include "device_common.h"

namespace lgbm_amd {
namespace dev {

namespace {

// argmax of best[0..s] (host loop order: higher gain, then smaller real feature, then lower
// leaf id); wave 0 reduces with shuffles, the result is broadcast through LDS
__device__ int PickLeaf(const KArgs& a, int s) {
  __shared__ int pick;
  if (threadIdx.x < kWave) {
    double bg = -INFINITY;
    int bf = -1, bl = 0x7fffffff;
    for (int l = threadIdx.x; l <= s; l += kWave) {
      const double g = a.best[l].gain;
      const int f = a.best[l].real_feature;
      if (bl == 0x7fffffff || SplitBetter(g, f, bg, bf)) {
        bg = g;
        bf = f;
        bl = l;
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const double og = __shfl_xor(bg, o, kWave);
      const int of = __shfl_xor(bf, o, kWave);
      const int ol = __shfl_xor(bl, o, kWave);
      const bool take = ol != 0x7fffffff &&
                        (bl == 0x7fffffff || SplitBetter(og, of, bg, bf) ||
                         (!SplitBetter(bg, bf, og, of) && ol < bl));
      if (take) {
        bg = og;
        bf = of;
        bl = ol;
      }
    }
    if (threadIdx.x == 0) pick = bl;
  }
  __syncthreads();
  return pick;
}

__device__ __forceinline__ void PartGeometry(int count, int* nb_out, int* rpb_out) {
  int nb = (count + kPartTile - 1) / kPartTile;
  nb = max(1, min(kMaxPartBlocks, nb));
  int rpb = (count + nb - 1) / nb;
  rpb = ((rpb + kPartTile - 1) / kPartTile) * kPartTile;
  if (rpb == 0) rpb = kPartTile;
  *nb_out = max(1, (count + rpb - 1) / rpb);
  *rpb_out = rpb;
}

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

// left count of rows [s0, s1) of the leaf range starting at pb
__device__ int CountLeft(const KArgs& a, const SplitRule& r, const Feature& F, const uint32_t* cat_bits, int pb,
                         int s0, int s1) {
  int cnt = 0;
  for (int t0 = s0; t0 < s1; t0 += kPartTile) {
    int row[kPartRowsPerThread];
#pragma unroll
    for (int k = 0; k < kPartRowsPerThread; ++k) {
      const int i = t0 + k * kPartThreads + threadIdx.x;
      row[k] = i < s1 ? a.idx[pb + i] : -1;
    }
    uint32_t gb[kPartRowsPerThread];
#pragma unroll
    for (int k = 0; k < kPartRowsPerThread; ++k) gb[k] = row[k] >= 0 ? ColBin(a, row[k], F.group) : 0u;
#pragma unroll
    for (int k = 0; k < kPartRowsPerThread; ++k) {
      if (row[k] >= 0 && GoesLeft(r, cat_bits, FeatureBinOf(F, gb[k]))) ++cnt;
    }
  }
  return cnt;
}

}  // namespace

// ---------------------------------------------------------------- device mode
__global__ __launch_bounds__(kPartThreads) void k_select_count(KArgs a) {
  __shared__ uint32_t cat_bits[kMaxCatWords];
  __shared__ int red[kPartThreads / kWave];
  Step* st = a.st;
  if (st->done) return;
  const int s = st->step;
  const int L = a.p.num_leaves;
  if (s >= L - 1) {
    if (blockIdx.x == 0 && threadIdx.x == 0) st->done = 1;
    return;
  }
  const int leaf = PickLeaf(a, s);
  const DeviceSplit sp = a.best[leaf];
  if (!(sp.gain > 0.0) || sp.feature < 0) {
    if (blockIdx.x == 0 && threadIdx.x == 0) st->done = 1;
    return;
  }
  const int pb = a.leaves[leaf].begin, pc = a.leaves[leaf].count;
  int nb, rpb;
  PartGeometry(pc, &nb, &rpb);
  const int b = blockIdx.x;
  if (b == 0 && threadIdx.x == 0) {
    const int nl = s + 1;
    st->leaf = leaf;
    st->new_leaf = nl;
    st->split = sp;
    st->part_begin = pb;
    st->part_count = pc;
    st->num_blocks = nb;
    st->rows_per_block = rpb;
    SplitRecord& rec = a.rec[s];
    rec.leaf = leaf;
    rec.split = sp;
    rec.left_count = sp.left_count;
    rec.right_count = sp.right_count;
    // children statistics (left keeps the leaf id); begin/count are set by the scatter
    Leaf* P = &a.leaves[leaf];
    Leaf* R = &a.leaves[nl];
    const int depth = P->depth + 1;
    double pmin = P->cmin, pmax = P->cmax, rmin = P->cmin, rmax = P->cmax;
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
    R->depth = depth;
    R->sum_g = sp.right_sum_gradient;
    R->sum_h = sp.right_sum_hessian;
    R->output = sp.right_output;
    R->global_count = sp.right_count;
    R->cmin = rmin;
    R->cmax = rmax;
    P->depth = depth;
    P->sum_g = sp.left_sum_gradient;
    P->sum_h = sp.left_sum_hessian;
    P->output = sp.left_output;
    P->global_count = sp.left_count;
    P->cmin = pmin;
    P->cmax = pmax;
  }
  if (b >= nb) return;
  SplitRule r;
  const Feature F = a.feat[sp.feature];
  MakeRule(sp, F, &r, cat_bits);
  __syncthreads();
  int cnt = CountLeft(a, r, F, cat_bits, pb, b * rpb, min(pc, b * rpb + rpb));
  cnt = BlockSum(cnt, red);
  if (threadIdx.x == 0) a.blk[b] = cnt;
}

void SelectAndCount(const KArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_select_count, dim3(kMaxPartBlocks), dim3(kPartThreads), 0, s, a);
}

// ---------------------------------------------------------------- host-assisted mode
__global__ __launch_bounds__(kPartThreads) void k_part_count(KArgs a) {
  __shared__ uint32_t cat_bits[kMaxCatWords];
  __shared__ int red[kPartThreads / kWave];
  const Step* st = a.st;
  if (st->done) return;
  const int b = blockIdx.x;
  if (b >= st->num_blocks) return;
  SplitRule r;
  const DeviceSplit& sp = st->split;
  const Feature F = a.feat[sp.feature];
  MakeRule(sp, F, &r, cat_bits);
  __syncthreads();
  const int pc = st->part_count, rpb = st->rows_per_block;
  int cnt = CountLeft(a, r, F, cat_bits, st->part_begin, b * rpb, min(pc, b * rpb + rpb));
  cnt = BlockSum(cnt, red);
  if (threadIdx.x == 0) a.blk[b] = cnt;
}

void PartitionCount(const KArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_part_count, dim3(kMaxPartBlocks), dim3(kPartThreads), 0, s, a);
}

// ---------------------------------------------------------------- scatter (both modes)
__global__ __launch_bounds__(kPartThreads) void k_part_scatter(KArgs a) {
  __shared__ uint32_t cat_bits[kMaxCatWords];
  __shared__ int red[kPartThreads / kWave];
  __shared__ int wl[kPartRowsPerThread][kPartThreads / kWave];
  Step* st = a.st;
  if (st->done) return;
  const int b = blockIdx.x;
  const int nb = st->num_blocks;
  if (b >= nb) return;
  SplitRule r;
  const DeviceSplit& sp = st->split;
  const Feature F = a.feat[sp.feature];
  MakeRule(sp, F, &r, cat_bits);
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
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int run_l = 0;
  const int left_base = pb + before;
  const int right_base = pb + total + (s0 - before);
  for (int t0 = s0; t0 < s1; t0 += kPartTile) {
    int row[kPartRowsPerThread];
#pragma unroll
    for (int k = 0; k < kPartRowsPerThread; ++k) {
      const int i = t0 + k * kPartThreads + threadIdx.x;
      row[k] = i < s1 ? a.idx[pb + i] : -1;
    }
    uint32_t gb[kPartRowsPerThread];
#pragma unroll
    for (int k = 0; k < kPartRowsPerThread; ++k) gb[k] = row[k] >= 0 ? ColBin(a, row[k], F.group) : 0u;
    bool left[kPartRowsPerThread];
    unsigned long long mask[kPartRowsPerThread];
#pragma unroll
    for (int k = 0; k < kPartRowsPerThread; ++k) {
      left[k] = row[k] >= 0 && GoesLeft(r, cat_bits, FeatureBinOf(F, gb[k]));
      mask[k] = __ballot(left[k]);
    }
    __syncthreads();
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < kPartRowsPerThread; ++k) wl[k][w] = __popcll(mask[k]);
    }
    __syncthreads();
    // rows are ordered (k, thread) inside the tile
    int sub_l = 0;
#pragma unroll
    for (int k = 0; k < kPartRowsPerThread; ++k) {
      int wbefore = 0, sub_tot = 0;
      for (int j = 0; j < nw; ++j) {
        if (j < w) wbefore += wl[k][j];
        sub_tot += wl[k][j];
      }
      if (row[k] >= 0) {
        const int lpos = run_l + sub_l + wbefore + __popcll(mask[k] & lt);  // lefts before me in the chunk
        const int pos = (t0 - s0) + k * kPartThreads + threadIdx.x;        // my position in the chunk
        if (left[k]) a.tmp[left_base + lpos] = row[k];
        else a.tmp[right_base + (pos - lpos)] = row[k];
      }
      sub_l += sub_tot;
    }
    run_l += sub_l;
  }
  if (b == 0 && threadIdx.x == 0) {
    const int leaf = st->leaf, nl = st->new_leaf;
    Leaf* P = &a.leaves[leaf];
    Leaf* R = &a.leaves[nl];
    P->begin = pb;
    P->count = total;
    R->begin = pb + total;
    R->count = pc - total;
    SplitRecord& rec = a.rec[st->step];
    if (!a.p.data_parallel) {
      P->global_count = P->count;
      R->global_count = R->count;
      rec.left_count = P->count;
      rec.right_count = R->count;
    }
    const int nlft = P->global_count, nrgt = R->global_count;
    const bool skip = (a.p.max_depth > 0 && P->depth >= a.p.max_depth) ||
                      (nrgt < 2 * a.p.sp.min_data_in_leaf && nlft < 2 * a.p.sp.min_data_in_leaf) ||
                      (st->step + 1 >= a.p.num_leaves - 1);
    int small_rows = 0;
    if (!skip) {
      if (nlft < nrgt) {
        // parent histogram moves to the (larger) right child
        const int t = P->slot;
        P->slot = R->slot;
        R->slot = t;
        st->smaller = leaf;
        st->larger = nl;
        small_rows = P->count;
      } else {
        st->smaller = nl;
        st->larger = leaf;
        small_rows = R->count;
      }
    }
    // small children are histogrammed straight into packed global words (see HistBody)
    st->hist_packed = (!a.p.data_parallel && small_rows <= a.hist_rows_cap) ? 1 : 0;
    a.best[leaf].gain = -INFINITY;
    a.best[leaf].feature = -1;
    a.best[leaf].real_feature = -1;
    a.best[nl].gain = -INFINITY;
    a.best[nl].feature = -1;
    a.best[nl].real_feature = -1;
    st->skip_find = skip ? 1 : 0;
    st->total_left = total;
    st->step = st->step + 1;
  }
}

void PartitionScatter(const KArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_part_scatter, dim3(kMaxPartBlocks), dim3(kPartThreads), 0, s, a);
}

}  // namespace dev
}  // namespace lgbm_amd
