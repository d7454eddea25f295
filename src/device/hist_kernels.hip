// Histogram construction (reference: the GPU learner's histogram256 OpenCL kernel and
// DenseBin::ConstructHistogram, src/treelearner/ocl/histogram256.cl, src/io/dense_bin.hpp).
//
// Layout: row-major bin matrix (one 32-bit word = 4 uint8 or 2 uint16 storage columns).
// Grid: (row chunks, column tiles).  A workgroup accumulates a LDS-private histogram of
// its tile's columns over its chunk of the leaf's rows, then adds the non-empty bins to
// the global histogram with 64-bit integer atomics.
//
// Accumulation is fixed point: (g * scale_g, h * scale_h) rounded to integers and packed
// into one uint64 (g in the signed high half, h in the low half) -> one ds_add_u64 per
// row and feature.  ds_add_f32 runs at ~0.33 lane-ops/CU/clk on gfx950, ds_add_u64 at ~5
// (tools/microbench/lds_atomics.hip); the scale (k_scales) leaves headroom for the largest
// per-workgroup row count so the 32-bit halves never overflow, and global sums are int64
// (exact, deterministic regardless of atomic order, and summable across ranks with RCCL).
#include "device_common.h"

namespace lgbm_amd {
namespace dev {

namespace {

__device__ __forceinline__ unsigned long long PackFixed(float2 v, float sg, float sh) {
  const long long gq = __float2ll_rn(v.x * sg);
  const long long hq = __float2ll_rn(v.y * sh);
  return (static_cast<unsigned long long>(gq) << 32) + static_cast<unsigned long long>(hq);
}

// Group bin 0 holds every row whose features all sit in their most frequent bin: it is
// outside every feature's histogram range (bin_offsets start at 1) and is restored by
// FixHistogram, so it is never accumulated (this also skips most rows of sparse columns).
template <int GPW>
__device__ __forceinline__ void AddRow(unsigned long long* lds, const int* goff, uint32_t w, unsigned long long pk) {
#pragma unroll
  for (int j = 0; j < GPW; ++j) {
    const uint32_t b = GPW == 4 ? ((w >> (8 * j)) & 0xffu) : ((w >> (16 * j)) & 0xffffu);
    if (goff[j] >= 0 && b != 0u) atomicAdd(&lds[goff[j] + b], pk);
  }
}

// MODE 0 root (buffer 0), 1 split step (buffer = step parity), 2 explicit range (buffer 0)
template <int MODE, int GPW>
__device__ void HistBody(const KArgs& a, unsigned long long* lds) {
  int begin, count;
  const int32_t* src;
  long long* out_buf = a.scratch;
  if (MODE == 0) {
    begin = 0;
    count = a.num_rows;
    src = a.root_identity ? nullptr : a.idx;
  } else if (MODE == 2) {
    begin = a.range_begin;
    count = a.num_rows;
    src = a.idx;
  } else {
    const Step* st = a.st;
    if (st->done) return;
    // copy the partitioned range of the split leaf back into the index array
    const int pb = st->part_begin, pc = st->part_count;
    const int nthreads = gridDim.x * gridDim.y * blockDim.x;
    const int gtid = (blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x;
    for (int i = gtid; i < pc; i += nthreads) a.idx[pb + i] = a.tmp[pb + i];
    if (st->skip_find) return;
    const Leaf& sm = a.leaves[st->smaller];
    begin = sm.begin;
    count = sm.count;
    src = a.tmp;
    out_buf = StepScratch(a, st->step);
    if (st->hist_packed) {
      // small leaf: every (row, word) adds its packed (g|h) word straight to the global
      // histogram -- no LDS zero/flush; count <= hist_rows_cap keeps the halves exact
      unsigned long long* outp = reinterpret_cast<unsigned long long*>(out_buf);
      const float sgs = static_cast<float>(a.scales[0]);
      const float shs = static_cast<float>(a.scales[1]);
      const int wpr = a.words_per_row;
      const int64_t pairs = static_cast<int64_t>(count) * wpr;
      const int64_t nthreads = static_cast<int64_t>(gridDim.x) * gridDim.y * blockDim.x;
      const uint32_t* bins32 = static_cast<const uint32_t*>(a.bins);
      const float2* gh = reinterpret_cast<const float2*>(a.gh);
      for (int64_t p = (static_cast<int64_t>(blockIdx.y) * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x;
           p < pairs; p += nthreads) {
        const int i = static_cast<int>(p / wpr);
        const int w = static_cast<int>(p - static_cast<int64_t>(i) * wpr);
        const int row = src[begin + i];
        const uint32_t word = bins32[static_cast<int64_t>(row) * wpr + w];
        if (word == 0u) continue;
        const unsigned long long pk = PackFixed(gh[row], sgs, shs);
#pragma unroll
        for (int j = 0; j < GPW; ++j) {
          const int g = w * GPW + j;
          const uint32_t b = GPW == 4 ? ((word >> (8 * j)) & 0xffu) : ((word >> (16 * j)) & 0xffffu);
          if (b != 0u && g < a.p.num_groups) atomicAdd(&outp[a.group_off[g] + b], pk);
        }
      }
      return;
    }
  }
  if (count <= 0) return;
  const int active = min(static_cast<int>(gridDim.x), max(1, count / kMinRowsPerHistBlock));
  if (static_cast<int>(blockIdx.x) >= active) return;
  const int chunk = (count + active - 1) / active;
  const int r0 = begin + blockIdx.x * chunk;
  const int r1 = min(begin + count, r0 + chunk);

  const int w0 = blockIdx.y * a.tile_words;
  const int w1 = min(a.words_per_row, w0 + a.tile_words);
  const int g0 = w0 * GPW;
  const int g_end = min(a.p.num_groups, w1 * GPW);
  const int lo_bin = a.group_off[g0];
  const int hi_bin = g_end < a.p.num_groups ? a.group_off[g_end] : a.p.total_bins;
  const int nbins = hi_bin - lo_bin;
  for (int i = threadIdx.x; i < nbins; i += blockDim.x) lds[i] = 0ull;
  __syncthreads();

  const float sg = static_cast<float>(a.scales[0]);
  const float sh = static_cast<float>(a.scales[1]);
  const int tpr = w1 - w0;  // threads per row
  const int rpp = blockDim.x / tpr;
  const int q = threadIdx.x % tpr;
  const int rs = threadIdx.x / tpr;
  if (rs < rpp) {
    const int w = w0 + q;
    int goff[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int g = w * GPW + j;
      goff[j] = (j < GPW && g < a.p.num_groups) ? (a.group_off[g] - lo_bin) : -1;
    }
    const uint32_t* bins32 = static_cast<const uint32_t*>(a.bins);
    const float2* gh = reinterpret_cast<const float2*>(a.gh);
    const int64_t wpr = a.words_per_row;
    const bool write_iota = MODE == 0 && src == nullptr && q == 0 && blockIdx.y == 0;
    int i = r0 + rs;
    // 4 rows in flight per thread
    for (; i + 3 * rpp < r1; i += 4 * rpp) {
      int r[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] = src ? src[i + k * rpp] : i + k * rpp;
      if (write_iota) {
#pragma unroll
        for (int k = 0; k < 4; ++k) a.idx[i + k * rpp] = i + k * rpp;
      }
      float2 v[4];
      uint32_t wd[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[k] = gh[r[k]];
        wd[k] = bins32[r[k] * wpr + w];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) AddRow<GPW>(lds, goff, wd[k], PackFixed(v[k], sg, sh));
    }
    for (; i < r1; i += rpp) {
      const int ra = src ? src[i] : i;
      if (write_iota) a.idx[i] = i;
      AddRow<GPW>(lds, goff, bins32[ra * wpr + w], PackFixed(gh[ra], sg, sh));
    }
  }
  __syncthreads();
  unsigned long long* out = reinterpret_cast<unsigned long long*>(out_buf) + 2 * lo_bin;
  for (int i = threadIdx.x; i < nbins; i += blockDim.x) {
    const unsigned long long v = lds[i];
    if (v != 0ull) {
      const long long gsum = static_cast<long long>(v) >> 32;  // h (low half) is non-negative
      const unsigned long long hsum = v & 0xffffffffull;
      atomicAdd(&out[2 * i], static_cast<unsigned long long>(gsum));
      atomicAdd(&out[2 * i + 1], hsum);
    }
  }
}

}  // namespace

template <int MODE, int GPW>
__global__ __launch_bounds__(kHistBlockThreads) void k_hist(KArgs a) {
  extern __shared__ unsigned long long lds[];
  HistBody<MODE, GPW>(a, lds);
}

template <int MODE>
static void LaunchHistMode(const KArgs& a, hipStream_t s) {
  const size_t lds_bytes = sizeof(unsigned long long) * static_cast<size_t>(a.tile_bins);
  dim3 grid(HistGridBlocks(), a.hist_tiles);
  if (a.bin_bytes == 1) {
    hipLaunchKernelGGL((k_hist<MODE, 4>), grid, dim3(kHistBlockThreads), lds_bytes, s, a);
  } else {
    hipLaunchKernelGGL((k_hist<MODE, 2>), grid, dim3(kHistBlockThreads), lds_bytes, s, a);
  }
}

void HistRoot(const KArgs& a, hipStream_t s) { LaunchHistMode<0>(a, s); }
void HistStep(const KArgs& a, hipStream_t s) { LaunchHistMode<1>(a, s); }
void HistRange(const KArgs& a, hipStream_t s) { LaunchHistMode<2>(a, s); }

}  // namespace dev
}  // namespace lgbm_amd
