// Device-side helpers shared by the HIP translation units of src/device/ (hipcc only).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>

#include "kernels.h"

namespace lgbm_amd {
namespace dev {

int NumCUs();  // compute units of the current device (SetNumCUs)

constexpr int kWave = 64;
constexpr int kFindLdsBins = 2048;  // split scan stages features up to this many bins in LDS
constexpr int kFindThreads = 256;   // split-scan workgroup

// in-kernel trace point: the first thread of workgroup (0, 0) stamps slot `slot` of split
// `s` after its outstanding memory operations completed (LGBM_AMD_KTRACE diagnostics)
__device__ __forceinline__ void KTrace(const KArgs& a, int s, int slot) {
  if (a.ktrace != nullptr && threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0 && s >= 0 &&
      s < a.p.num_leaves) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    a.ktrace[s * kTraceSlots + slot] = wall_clock64();
  }
}

__device__ __forceinline__ void KTraceAt(const KArgs& a, int s, int slot, long long t) {
  if (a.ktrace != nullptr && threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0 && s >= 0 &&
      s < a.p.num_leaves) {
    a.ktrace[s * kTraceSlots + slot] = t;
  }
}

inline int GridFor(int64_t n) {
  return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8 * NumCUs())));
}

__device__ __forceinline__ int RoundIntD(double x) { return static_cast<int>(x + 0.5f); }

// rows of the tree's root: a device-drawn bag keeps its size on the device (so the tree's
// captured graph does not depend on it)
__device__ __forceinline__ int RootRows(const KArgs& a) { return a.num_rows_dev ? *a.num_rows_dev : a.num_rows; }

// bin of storage column `group` for `row`, column-major copy (partition kernels)
__device__ __forceinline__ uint32_t ColBin(const KArgs& a, int64_t row, int group) {
  if (a.bin_bytes == 1) return a.bins_col[static_cast<int64_t>(group) * a.num_data + row];
  return reinterpret_cast<const uint16_t*>(a.bins_col)[static_cast<int64_t>(group) * a.num_data + row];
}

// bin of storage column `group` for `row`, row-major matrix
__device__ __forceinline__ uint32_t RowBin(const KArgs& a, int64_t row, int group) {
  if (a.bin_bytes == 1) return static_cast<const uint8_t*>(a.bins)[row * (4 * a.words_per_row) + group];
  return static_cast<const uint16_t*>(a.bins)[row * (2 * a.words_per_row) + group];
}

// group bin -> feature bin (Dataset::FeatureBin)
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

template <typename T>
__device__ __forceinline__ T WaveSum(T v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// block-wide sum (every thread gets the result); sh needs blockDim/64 entries
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

// SplitInfo ordering: larger gain first, then smaller real feature index (NaN = -inf)
__device__ __forceinline__ bool SplitBetter(double ga, int fa, double gb, int fb) {
  if (ga != ga) ga = -INFINITY;
  if (gb != gb) gb = -INFINITY;
  if (fa < 0) fa = 0x7fffffff;
  if (fb < 0) fb = 0x7fffffff;
  if (ga != gb) return ga > gb;
  return fa < fb;
}

// histogram buffers: the root uses buffer 0, split s buffer (s + 1) & 1; the split scan of
// split s zeroes the other one for split s + 1
__device__ __forceinline__ long long* StepScratch(const KArgs& a, int parity) {
  return a.scratch + static_cast<size_t>(parity & 1) * 2 * a.p.total_bins;
}

// a step histogram with this many row blocks -- or any step from split direct_from_split
// on, whose tree graph has no reduce kernel -- is summed by the split scan itself (the
// reduce kernel skips it); data-parallel training always reduces (the all-reduce needs it)
__device__ __forceinline__ bool DirectPartials(const KArgs& a, int nblk, int split) {
  return !a.p.data_parallel && (nblk <= kReduceChunk || split >= a.p.direct_from_split);
}

// outcome of the step's partition, derived from Step::cs and the final cursors (every
// histogram workgroup computes it; one also stores it in Step for the later kernels)
struct ChildInfo {
  int total_left;
  int left_count, right_count;  // global counts (== local ones without data-parallel)
  int smaller, larger;          // leaf ids
  int small_is_left;
  int skip;
  int s_begin, s_count, buf;    // the smaller child's local rows
};

__device__ __forceinline__ ChildInfo StepChildren(const KArgs& a, const Step* st) {
  ChildInfo c;
  const CurSplit& cs = st->cs;
  const int pb = cs.part_begin, pc = cs.part_count;
  c.total_left = st->cur_left;
  c.left_count = a.p.data_parallel ? cs.split.left_count : c.total_left;
  c.right_count = a.p.data_parallel ? cs.split.right_count : pc - c.total_left;
  const int md = a.p.sp.min_data_in_leaf;
  c.skip = (a.p.max_depth > 0 && cs.child_depth >= a.p.max_depth) ||
           (c.right_count < 2 * md && c.left_count < 2 * md) || (cs.s + 1 >= a.p.num_leaves - 1);
  c.small_is_left = c.left_count < c.right_count;
  c.smaller = c.small_is_left ? cs.leaf : cs.new_leaf;
  c.larger = c.small_is_left ? cs.new_leaf : cs.leaf;
  c.s_begin = c.small_is_left ? pb : pb + c.total_left;
  c.s_count = c.small_is_left ? c.total_left : pc - c.total_left;
  c.buf = 1 - cs.src_buf;
  return c;
}

}  // namespace dev
}  // namespace lgbm_amd
