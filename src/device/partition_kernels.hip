// Split selection + data partition (reference serial_tree_learner.cpp Train/Split,
// src/treelearner/data_partition.hpp Split, monotone_constraints.hpp BasicLeafConstraints).
//
// k_partition: the split leaf's index range [part_begin, +part_count) of buffer src_buf is
// moved into the same range of the other buffer, lefts growing up from the front and
// rights down from the back.  Each 8192-row tile reserves its output slots with one
// device-scope atomic per side (no grid-wide prefix pass); rows keep their order inside a
// tile, tiles land in arrival order -- histograms are exact integer sums, so the row order
// never changes a result.  The cursors' final values are the children's sizes, read by
// the histogram kernel (StepChildren).  Rows are read from the column-major copy of the
// split column (1 byte per row).
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

}  // namespace

__global__ __launch_bounds__(kPartThreads) void k_partition(KArgs a) {
  __shared__ uint32_t cat_bits[kMaxCatWords];
  __shared__ int wl[kPartRowsPerThread][kPartThreads / kWave];
  __shared__ int base[2];
  Step* st = a.st;
  if (st->done) return;
  const int pb = st->part_begin, pc = st->part_count;
  const int src_buf = st->src_buf;
  const int32_t* src = src_buf ? a.tmp : a.idx;
  int32_t* dst = src_buf ? a.idx : a.tmp;
  const int ntiles = (pc + kPartTile - 1) / kPartTile;
  if (static_cast<int>(blockIdx.x) >= ntiles) return;
  const DeviceSplit& sp = st->split;
  const Feature F = st->sfeat;
  SplitRule r;
  MakeRule(sp, F, &r, cat_bits);
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
}

void Partition(const KArgs& a, hipStream_t s) {
  // one workgroup per CU: at most ~num_data / (kPartTile * CUs) tile reservations each
  const int grid = std::max(1, std::min((a.num_data + kPartTile - 1) / kPartTile, NumCUs()));
  hipLaunchKernelGGL(k_partition, dim3(grid), dim3(kPartThreads), 0, s, a);
}

}  // namespace dev
}  // namespace lgbm_amd
