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

// a group's bin from the row bytes at its offset, by its width (Feature::gwide: 0 8-bit,
// 1 16-bit, 2 / 3 the low / high 4 bits)
__device__ __forceinline__ uint32_t GroupBinAt(const uint8_t* p, int gwide) {
  if (gwide == 1) return static_cast<uint32_t>(*reinterpret_cast<const uint16_t*>(p));
  const uint32_t b = *p;
  return gwide >= 2 ? (b >> ((gwide & 1) * 4)) & 15u : b;
}
// bin of a storage column for `row` in the row-major matrix, from the group's byte offset
// in a row and its width (Feature::gbyte / gwide)
__device__ __forceinline__ uint32_t RowBin(const KArgs& a, int64_t row, int gbyte, int gwide) {
  const uint8_t* p = static_cast<const uint8_t*>(a.bins) + row * (4 * static_cast<int64_t>(a.row_words)) + gbyte;
  return GroupBinAt(p, gwide);
}

// (g, h) of a row (KArgs::gh_stride)
__device__ __forceinline__ float2 GhAt(const KArgs& a, int64_t row) {
  return reinterpret_cast<const float2*>(a.gh)[row * a.gh_stride];
}

// index buffer b (Leaf::buf): 0 idx, 1 tmp, b > 1 (round growth) tmp + (b - 1) * stride
__host__ __device__ __forceinline__ int32_t* RowBuf(int32_t* idx, int32_t* tmp, int64_t stride, int b) {
  return b == 0 ? idx : tmp + static_cast<int64_t>(b - 1) * stride;
}
__host__ __device__ __forceinline__ const int32_t* RowBuf(const int32_t* idx, const int32_t* tmp, int64_t stride, int b) {
  return b == 0 ? idx : tmp + static_cast<int64_t>(b - 1) * stride;
}
__device__ __forceinline__ int32_t* RowBuf(const KArgs& a, int b) { return RowBuf(a.idx, a.tmp, a.buf_stride, b); }

// the split column's bin for the partition: from the column-major copy when there is one,
// else from the row-major matrix (whose line the histogram pass then reads again)
__device__ __forceinline__ uint32_t ColBin(const KArgs& a, int64_t row, int gbyte, int gwide, int64_t col_off) {
  if (a.bins_col == nullptr) return RowBin(a, row, gbyte, gwide);
  if (gwide == 1) return reinterpret_cast<const uint16_t*>(a.bins_col + col_off)[row];  // (4-bit groups: bytes)
  return a.bins_col[col_off + row];
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

// Wave-wide prefix sums and sums over DPP lane moves (row_shr within rows of 16 lanes, then
// row_bcast:15 / row_bcast:31 across rows): six VALU-issued moves per 32-bit half instead of
// six ds_bpermute round trips through the LDS crossbar.  Every lane of the wave must be active.
#ifndef LGBM_DPP_SCAN
#define LGBM_DPP_SCAN 1
#endif
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ int DppI32(int v) {
  // (disabled rows and lanes without a source read 0: the identity of the sums)
  return __builtin_amdgcn_update_dpp(0, v, CTRL, ROW_MASK, 0xf, true);
}
template <int CTRL, int ROW_MASK = 0xf, typename T>
__device__ __forceinline__ T DppMove(T v) {
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, DppI32<CTRL, ROW_MASK>(__builtin_bit_cast(int, v)));
  } else {
    static_assert(sizeof(T) == 8, "DppMove: 4- or 8-byte values");
    const long long x = __builtin_bit_cast(long long, v);
    const int lo = DppI32<CTRL, ROW_MASK>(static_cast<int>(x));
    const int hi = DppI32<CTRL, ROW_MASK>(static_cast<int>(x >> 32));
    return __builtin_bit_cast(T, static_cast<long long>((static_cast<unsigned long long>(static_cast<unsigned>(hi)) << 32) |
                                                        static_cast<unsigned>(lo)));
  }
}
template <typename T>
__device__ __forceinline__ T WavePrefixInclDpp(T v) {
  v += DppMove<0x111>(v);       // row_shr:1
  v += DppMove<0x112>(v);       // row_shr:2
  v += DppMove<0x114>(v);       // row_shr:4
  v += DppMove<0x118>(v);       // row_shr:8
  v += DppMove<0x142, 0xa>(v);  // row_bcast:15 -> rows 1, 3
  v += DppMove<0x143, 0xc>(v);  // row_bcast:31 -> rows 2, 3
  return v;
}
template <typename T>
__device__ __forceinline__ T WaveLane63(T v) {
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
  } else {
    const long long x = __builtin_bit_cast(long long, v);
    const unsigned lo = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(x), 63));
    const unsigned hi = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(x >> 32), 63));
    return __builtin_bit_cast(T, static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
  }
}

// lane l's value (l wave-uniform)
template <typename T>
__device__ __forceinline__ T ReadLane(T v, int l) {
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
  } else {
    const long long x = __builtin_bit_cast(long long, v);
    const unsigned lo = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(x), l));
    const unsigned hi = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(x >> 32), l));
    return __builtin_bit_cast(T, static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
  }
}

template <typename T>
__device__ __forceinline__ T WaveSum(T v) {
#if LGBM_DPP_SCAN
  return WaveLane63(WavePrefixInclDpp(v));
#else
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
#endif
}

// wave-wide max over DPP lane moves (every lane of the wave active; 0 is the identity)
template <typename T>
__device__ __forceinline__ T WaveMaxDpp(T v) {
  v = max(v, DppMove<0x111>(v));
  v = max(v, DppMove<0x112>(v));
  v = max(v, DppMove<0x114>(v));
  v = max(v, DppMove<0x118>(v));
  v = max(v, DppMove<0x142, 0xa>(v));
  v = max(v, DppMove<0x143, 0xc>(v));
  return WaveLane63(v);
}

// order-preserving key of a gain: a larger gain has a larger key, NaN orders as -inf, and
// every key of a number (-inf included) is above 0 (the identity of WaveMaxDpp)
__device__ __forceinline__ unsigned long long GainKey(double g) {
  if (g != g) g = -INFINITY;
  if (g == 0.0) g = 0.0;  // (-0.0 and 0.0 compare equal: one key)
  const unsigned long long b = static_cast<unsigned long long>(__double_as_longlong(g));
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

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
#if LGBM_DPP_SCAN
  return WavePrefixInclDpp(v);
#else
  const int lane = threadIdx.x & 63;
  for (int o = 1; o < 64; o <<= 1) {
    T t = __shfl_up(v, o, kWave);
    if (lane >= o) v += t;
  }
  return v;
#endif
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

// Write-through publication of a record that another workgroup of the same launch reads
// (the split scans' per-feature results, read by the picking workgroup): 8-byte agent-scope
// relaxed atomic stores are `global_store ... sc1` on gfx950 -- the bytes leave the XCD's L2
// at once, so no release fence (an L2 write-back, serialised per XCD: ~15 ns per workgroup
// of a 4000-workgroup launch, tools/microbench/wg_throughput.hip) is needed.  The writing
// waves drain them (s_waitcnt vmcnt(0)) before the arrival counter is bumped; the picker
// takes one agent-scope acquire (cdna_hip_programming.md Guideline 16, R1).
typedef __attribute__((address_space(1))) unsigned long long GlobalU64;
// (Other targets: agent-scope relaxed stores may stay in a non-coherent cache; there the
// stores are followed by a release fence before the arrival count -- ArrivalRelease.)
#if !defined(__gfx942__) && !defined(__gfx950__) && defined(__HIP_DEVICE_COMPILE__)
#define LGBM_PUBLISH_NEEDS_FENCE 1
#else
#define LGBM_PUBLISH_NEEDS_FENCE 0
#endif
__device__ __forceinline__ void ArrivalRelease() {
#if LGBM_PUBLISH_NEEDS_FENCE
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
#endif
}
template <typename T>
__device__ __forceinline__ void PublishRecord(T* dst, const T& v) {
  static_assert(sizeof(T) % 8 == 0, "8-byte words");
  GlobalU64* d = (GlobalU64*)(dst);
#pragma unroll
  for (int i = 0; i < static_cast<int>(sizeof(T) / 8); ++i) {
    unsigned long long w;  // (memcpy: the record's fields are not u64 -- no type-punned loads)
    __builtin_memcpy(&w, reinterpret_cast<const char*>(&v) + 8 * i, 8);
    __hip_atomic_store(d + i, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
__device__ __forceinline__ void PublishF64(double* dst, double v) {
  __hip_atomic_store((GlobalU64*)(dst), static_cast<unsigned long long>(__double_as_longlong(v)), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void PublishI32(int32_t* dst, int32_t v) {
  typedef __attribute__((address_space(1))) int32_t GlobalI32;
  __hip_atomic_store((GlobalI32*)(dst), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
struct CatWords {
  uint32_t w[kMaxCatWords];
};
// Category sets are copied / published write-through in 64-bit words, a few registers at a
// time: a whole CatWords value is 128 VGPRs, and one indexed by category lives in scratch.
// (u64 word i holds the uint32 words 2i and 2i + 1: bin b is bit b & 63 of word b >> 6)
__device__ __forceinline__ void PublishCatCopy(uint32_t* dst, const uint32_t* src) {
  const unsigned long long* s = reinterpret_cast<const unsigned long long*>(src);
  GlobalU64* d = (GlobalU64*)(dst);
#pragma unroll 1
  for (int i0 = 0; i0 < kMaxCatWords / 2; i0 += 8) {
    unsigned long long v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = s[i0 + k];
#pragma unroll
    for (int k = 0; k < 8; ++k) __hip_atomic_store(d + i0 + k, v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// the set {bin} (bin < 0: the empty set)
__device__ __forceinline__ void PublishCatSingle(uint32_t* dst, int bin) {
  GlobalU64* d = (GlobalU64*)(dst);
#pragma unroll 1
  for (int i = 0; i < kMaxCatWords / 2; ++i) {
    const unsigned long long v = (bin >= 0 && (bin >> 6) == i) ? (1ull << (bin & 63)) : 0ull;
    __hip_atomic_store(d + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
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
  return a.scratch + static_cast<size_t>(parity & 1) * a.scratch_stride;
}


// outcome of the step's partition, derived from Step::cs and the final cursors (every
// split-scan workgroup computes it; the pick stores what later steps need)
struct ChildInfo {
  int total_left;               // local rows that went left
  int left_count, right_count;  // global counts (== local ones without data-parallel)
  int smaller, larger;          // leaf ids (exact counts; ties: the right child is smaller)
  int small_is_left;
  int skip;                     // neither child can be split (depth / min_data / last split)
};

// min_data_in_leaf of the rule that skips a step's scans when both children are too small
// (Params::skip_min_data: voting's local scans hold local parameters)
__device__ __forceinline__ int SkipMinData(const KArgs& a) {
  return a.p.skip_min_data > 0 ? a.p.skip_min_data - 1 : a.p.sp.min_data_in_leaf;
}
__device__ __forceinline__ ChildInfo StepChildren(const KArgs& a, const Step* st) {
  ChildInfo c;
  const CurSplit& cs = st->cs;
  const int pc = cs.part_count;
  c.total_left = st->cur_left;
  c.left_count = a.p.data_parallel ? cs.split.left_count : c.total_left;
  c.right_count = a.p.data_parallel ? cs.split.right_count : pc - c.total_left;
  const int md = SkipMinData(a);
  c.skip = (a.p.max_depth > 0 && cs.child_depth >= a.p.max_depth) ||
           (c.right_count < 2 * md && c.left_count < 2 * md) || (cs.s + 1 >= a.p.num_leaves - 1);
  c.small_is_left = c.left_count < c.right_count;
  c.smaller = c.small_is_left ? cs.leaf : cs.new_leaf;
  c.larger = c.small_is_left ? cs.new_leaf : cs.leaf;
  return c;
}

// one child of the step as seen by the split scan: k = 0 the smaller, 1 the larger child.
// The child whose rows k_split histogrammed (Step::hist_left) takes the new leaf's slot; the
// other one is parent - that histogram, computed in place in the parent's slot.
struct SideInfo {
  int lr;            // 0 left child (keeps the leaf id), 1 right child (the new leaf)
  int leaf, slot, frow;
  int is_hist;
  int global_count;
};

__device__ __forceinline__ SideInfo StepSide(const KArgs& a, const Step* st, const ChildInfo& c, int k) {
  const CurSplit& cs = st->cs;
  SideInfo d;
  d.lr = ((k == 0) == (c.small_is_left != 0)) ? 0 : 1;
  d.leaf = d.lr == 0 ? cs.leaf : cs.new_leaf;
  d.is_hist = (d.lr == 0) == (st->hist_left != 0);
  d.slot = d.is_hist ? cs.new_leaf : cs.parent_slot;
  d.frow = k == 0 ? cs.new_frow : cs.parent_frow;  // the larger child inherits the parent's row
  d.global_count = a.p.data_parallel ? st->lr[d.lr].global_count : (d.lr == 0 ? c.left_count : c.right_count);
  return d;
}

// row blocks of the step's histogram (k_split deals the parent's rows out in blocks)
__device__ __forceinline__ int StepBlocks(const KArgs& a, int parent_count) {
  return HistBlocksFor(parent_count, a.split_grid, a.hist_rows_cap, a.blk_min_rows);
}

// a step histogram with this many row blocks -- or any step from split direct_from_split
// on, whose tree graph has no reduce kernel -- is summed by the split scan itself (the
// reduce kernel skips it); data-parallel training always reduces (the collectives need it)
__device__ __forceinline__ bool DirectPartials(const KArgs& a, int nblk, int split) {
  return !a.p.data_parallel && (nblk <= kDirectChunk || split >= a.p.direct_from_split);
}

// max |h| with the sign bit set when any h is negative (k_scales then keeps the packed h half
// signed): the hessian maxima of the gradient / packing kernels and their reductions
__device__ __forceinline__ float HessMax(float a, float b) {
  const unsigned s = (__float_as_uint(a) | __float_as_uint(b)) & 0x80000000u;
  return __uint_as_float(__float_as_uint(fmaxf(fabsf(a), fabsf(b))) | s);
}

// (g, h) of partial word(s) v: packed (g in the signed high half, h in the low half) or wide.
// A packed word is g * 2^32 + h.  h lies in [0, 2^31] when no hessian is negative and in
// [-2^30, 2^30] otherwise (k_scales): the two ranges decode apart, a low half from 3 * 2^30 on
// being a negative h (whose borrow is returned to g).
__device__ __forceinline__ void UnpackPartial(unsigned long long v0, unsigned long long v1, int units, long long* g,
                                              long long* h) {
  if (units == 1) {
    const unsigned lo = static_cast<unsigned>(v0);
    const long long hv = lo >= 0xC0000000u ? static_cast<long long>(lo) - (1ll << 32) : static_cast<long long>(lo);
    *g = static_cast<long long>(v0 - static_cast<unsigned long long>(hv)) >> 32;
    *h = hv;
  } else {
    *g = static_cast<long long>(v0);
    *h = static_cast<long long>(v1);
  }
}

// the fixed-point scales of a tree from absmax = (max |g| bits, max |h| bits, rows cap or 0,
// negative-hessian flag): scales[0..1] = 2^k per component, scales[2..3] their inverses (see
// k_scales in misc_kernels.hip for the headroom rules).  One thread.
__device__ inline void ScalesFromAbsmax(const uint32_t absmax[4], int rows_cap, int units, double* scales) {
  if (absmax[2] != 0u) rows_cap = static_cast<int>(absmax[2]);
  const double lim[2] = {units == 1 ? 1073741824.0 : 2147483648.0,
                        units == 1 && absmax[3] != 0u ? 1073741824.0 : 2147483648.0};
  const double rows = units == 1 ? static_cast<double>(rows_cap) : 1.0;
  for (int k = 0; k < 2; ++k) {
    const double m = static_cast<double>(__uint_as_float(absmax[k]));
    double sc = 1.0;
    if (m > 0.0 && isfinite(m)) {
      int e = static_cast<int>(floor(log2(lim[k] / (rows * m))));
      e = max(-120, min(120, e));
      sc = ldexp(1.0, e);
    }
    scales[k] = sc;
    scales[2 + k] = 1.0 / sc;
  }
}

}  // namespace dev
}  // namespace lgbm_amd
