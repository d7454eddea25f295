// Histogram construction of whole row sets -- the tree's root and explicit index ranges of
// host-assisted growth -- and the exact reduction of per-row-block partial histograms
// (reference: the GPU learner's histogram256 OpenCL kernel and DenseBin::ConstructHistogram,
// src/treelearner/ocl/histogram256.cl, src/io/dense_bin.hpp).  The per-split histograms
// are built by k_split (partition_kernels.hip) together with the row partition.
//
// Layout: row-major bin matrix (one 32-bit word = 4 uint8 or 2 uint16 storage columns; a
// mixed layout keeps 8-bit groups 4 to a word next to words of 16-bit groups), or row-sparse
// lists of each row's stored bins (hist_common.h AddSparseRows).
// Grid: (row workgroups, column tiles) of 1024-thread workgroups.  A workgroup accumulates
// an LDS-private histogram of its tile's columns over one row block at a time and stores it
// whole as that block's partial histogram -- no global atomics (on gfx950 those execute at
// the memory side; a per-workgroup atomic flush of a 7K-bin tile took ~22 us).
// k_hist_reduce then sums the partials of every bin into int64 (g, h).
//
// Accumulation is fixed point (see hist_common.h): each row's (g, h) is rounded to integers
// at the tree's scales and added with LDS integer atomics (ds_add_f32 runs at ~0.33
// lane-ops/CU/clk on gfx950, ds_add_u64 at ~5: tools/microbench/lds_atomics.hip).  Packed
// mode (hist_units 1): one u64 per bin, g in the signed high half and h in the low half, one
// ds_add_u64 per row and feature; a row block holds at most kHistRowsCap rows so the halves
// never overflow, whatever the number of rows.  Wide mode (hist_units 2, gpu_use_dp): int64 g
// and h, each row quantised to 31 bits of the tree's max |g| / max h.  Global sums are int64:
// exact, independent of the row order and summable across ranks.
#include "hist_common.h"

namespace lgbm_amd {
namespace dev {

namespace {

template <int MODE>
__device__ __forceinline__ void HistRowSet(const KArgs& a, int* begin, int* count, const int32_t** src) {
  if (MODE == 0) {
    *begin = 0;
    *count = RootRows(a);
    *src = a.root_identity ? nullptr : a.idx;
  } else {
    *begin = a.range_begin;
    *count = a.num_rows;
    *src = a.idx;
  }
}

template <int MODE, int GPW, int UNITS>
__global__ __launch_bounds__(kHistThreads) void k_hist(KArgs a) {
  extern __shared__ unsigned long long lds[];
  TileCtx t;
  InitTile<GPW>(a, &t);
  int begin, count;
  const int32_t* src;
  HistRowSet<MODE>(a, &begin, &count, &src);
  if (count <= 0) return;
  const int nblk = HistBlocksFor(count, gridDim.x, a.hist_rows_cap, kHistMinRows);
  const int chunk = (count + nblk - 1) / nblk;
  const size_t pstride = static_cast<size_t>(UNITS) * a.p.total_bins;
  for (int kb = blockIdx.x; kb < nblk; kb += gridDim.x) {
    HistBlock<MODE == 0, GPW, UNITS>(a, lds, src, begin + kb * chunk, min(begin + count, begin + kb * chunk + chunk), t,
                                a.partials + kb * pstride + static_cast<size_t>(UNITS) * t.lo_bin);
  }
}

// partials [block][bin] -> int64 (g, h) pairs.  Each thread sums up to kReduceChunk
// partials of one bin; with more blocks than that the chunks are combined by int64 atomics
// into the (pre-zeroed) buffer, otherwise the single chunk stores directly.
// MODE 0 root, 1 the step's child histogram (k_split's blocks of the parent), 2 range.
template <int MODE, int UNITS>
__global__ __launch_bounds__(256) void k_hist_reduce(KArgs a) {
  const long long t_entry = wall_clock64();
  int nblk;
  long long* out;
  int ts = -1;
  if (MODE == 1) {
    const Step* st = a.st;
    if (st->done) return;
    const int s = st->cs.s;
    ts = s;
    KTraceAt(a, ts, kTrRedEntry, t_entry);
    nblk = StepBlocks(a, st->cs.part_count);
    if (DirectPartials(a, nblk, s)) {  // summed by the split scan
      KTrace(a, ts, kTrRedExit);
      return;
    }
    out = StepScratch(a, s + 1);
  } else {
    int begin, count;
    const int32_t* src;
    HistRowSet<MODE>(a, &begin, &count, &src);
    nblk = HistBlocksFor(count, a.root_grid, a.hist_rows_cap, kHistMinRows);
    out = a.scratch;
  }
  if (static_cast<int>(blockIdx.y) * kReduceChunk >= nblk) return;
  const int bin = blockIdx.x * blockDim.x + threadIdx.x;
  const int nb = a.p.total_bins;
  if (bin >= nb) return;
  const size_t pstride = static_cast<size_t>(UNITS) * nb;
  long long g = 0, h = 0;
  // chunks blockIdx.y, + gridDim.y, ...: a few workgroup rows walk all the chunks (every
  // launched workgroup costs launch time even when it exits at once)
  for (int k0 = blockIdx.y * kReduceChunk; k0 < nblk; k0 += gridDim.y * kReduceChunk) {
    const unsigned long long* p = a.partials + k0 * pstride + static_cast<size_t>(UNITS) * bin;
    const int kn = min(kReduceChunk, nblk - k0);
    if (UNITS == 1) {
      unsigned long long v[kReduceChunk];
#pragma unroll
      for (int k = 0; k < kReduceChunk; ++k) v[k] = k < kn ? p[k * pstride] : 0ull;
#pragma unroll
      for (int k = 0; k < kReduceChunk; ++k) {
        long long pg, ph;
        UnpackPartial(v[k], 0ull, 1, &pg, &ph);
        g += pg;
        h += ph;
      }
    } else {
      ulonglong2 v[kReduceChunk];
#pragma unroll
      for (int k = 0; k < kReduceChunk; ++k) {
        v[k] = k < kn ? *reinterpret_cast<const ulonglong2*>(p + k * pstride) : make_ulonglong2(0ull, 0ull);
      }
#pragma unroll
      for (int k = 0; k < kReduceChunk; ++k) {
        g += static_cast<long long>(v[k].x);
        h += static_cast<long long>(v[k].y);
      }
    }
  }
  const int pos = a.rs_pos != nullptr ? a.rs_pos[bin] : bin;  // owner-major layout (data-parallel)
  if (pos < 0) return;  // (a group no rank scans this tree)
  if (nblk <= kReduceChunk) {
    out[2 * pos] = g;
    out[2 * pos + 1] = h;
  } else {
    atomicAdd(reinterpret_cast<unsigned long long*>(&out[2 * pos]), static_cast<unsigned long long>(g));
    atomicAdd(reinterpret_cast<unsigned long long*>(&out[2 * pos + 1]), static_cast<unsigned long long>(h));
  }
  KTrace(a, ts, kTrRedExit);
}

// the largest dynamic LDS a workgroup may declare (the device's per-block limit)
static int MaxDynLds() {
  int dev = 0, v = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess) {
    (void)hipGetLastError();
    return 65536;
  }
  return v;
}

template <typename K>
static void AllowLds(K kernel) {
  const int mx = MaxDynLds();
  if (mx > 65536 && hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, mx) != hipSuccess) {
    (void)hipGetLastError();  // not fatal: launches above 64 KiB then fail loudly
  }
}

template <int MODE>
static void LaunchHist(const KArgs& a, hipStream_t s) {
  const size_t lds_bytes = sizeof(unsigned long long) * a.hist_units * static_cast<size_t>(a.tile_bins);

  const dim3 grid(a.root_grid, a.hist_tiles);
  if (a.sp_ptr != nullptr) {
    if (a.hist_units == 1) hipLaunchKernelGGL((k_hist<MODE, kSparseGPW, 1>), grid, dim3(kHistThreads), lds_bytes, s, a);
    else hipLaunchKernelGGL((k_hist<MODE, kSparseGPW, 2>), grid, dim3(kHistThreads), lds_bytes, s, a);
  } else if (a.hist_units == 1) {
    if (a.nibbles) hipLaunchKernelGGL((k_hist<MODE, 8, 1>), grid, dim3(kHistThreads), lds_bytes, s, a);
    else if (a.bin_bytes == 1) hipLaunchKernelGGL((k_hist<MODE, 4, 1>), grid, dim3(kHistThreads), lds_bytes, s, a);
    else if (a.bin_bytes == 2) hipLaunchKernelGGL((k_hist<MODE, 2, 1>), grid, dim3(kHistThreads), lds_bytes, s, a);
    else hipLaunchKernelGGL((k_hist<MODE, 0, 1>), grid, dim3(kHistThreads), lds_bytes, s, a);
  } else {
    if (a.nibbles) hipLaunchKernelGGL((k_hist<MODE, 8, 2>), grid, dim3(kHistThreads), lds_bytes, s, a);
    else if (a.bin_bytes == 1) hipLaunchKernelGGL((k_hist<MODE, 4, 2>), grid, dim3(kHistThreads), lds_bytes, s, a);
    else if (a.bin_bytes == 2) hipLaunchKernelGGL((k_hist<MODE, 2, 2>), grid, dim3(kHistThreads), lds_bytes, s, a);
    else hipLaunchKernelGGL((k_hist<MODE, 0, 2>), grid, dim3(kHistThreads), lds_bytes, s, a);
  }
  LaunchReduce<MODE>(a, s);
}

}  // namespace

#ifndef LGBM_REDUCE_ROWS
#define LGBM_REDUCE_ROWS 4
#endif
constexpr int kReduceRows = LGBM_REDUCE_ROWS;  // workgroup rows of a reduction (each walks chunks)

template <int MODE>
void LaunchReduce(const KArgs& a, hipStream_t s) {
  const dim3 rgrid((a.p.total_bins + 255) / 256,
                   std::min(kReduceRows, (a.hist_max_blocks + kReduceChunk - 1) / kReduceChunk));
  if (a.hist_units == 1) hipLaunchKernelGGL((k_hist_reduce<MODE, 1>), rgrid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((k_hist_reduce<MODE, 2>), rgrid, dim3(256), 0, s, a);
}
template void LaunchReduce<1>(const KArgs&, hipStream_t);

void PrepareSplitKernels(int max_lds);
void PrepareRoundKernels(int max_lds);
void PrepareRankKernels(int max_lds);

// dynamic LDS above 64 KiB must be enabled per kernel (outside any graph capture)
void PrepareKernels() {
  AllowLds(k_hist<0, 8, 1>);
  AllowLds(k_hist<0, 8, 2>);
  AllowLds(k_hist<2, 8, 1>);
  AllowLds(k_hist<2, 8, 2>);
  AllowLds(k_hist<0, 4, 1>);
  AllowLds(k_hist<0, 2, 1>);
  AllowLds(k_hist<0, 4, 2>);
  AllowLds(k_hist<0, 2, 2>);
  AllowLds(k_hist<2, 4, 1>);
  AllowLds(k_hist<2, 2, 1>);
  AllowLds(k_hist<2, 4, 2>);
  AllowLds(k_hist<2, 2, 2>);
  AllowLds(k_hist<0, 0, 1>);
  AllowLds(k_hist<0, 0, 2>);
  AllowLds(k_hist<2, 0, 1>);
  AllowLds(k_hist<2, 0, 2>);
  AllowLds(k_hist<0, kSparseGPW, 1>);
  AllowLds(k_hist<0, kSparseGPW, 2>);
  AllowLds(k_hist<2, kSparseGPW, 1>);
  AllowLds(k_hist<2, kSparseGPW, 2>);
  PrepareSplitKernels(MaxDynLds());
  PrepareRoundKernels(MaxDynLds());
  PrepareRankKernels(MaxDynLds());
}

void HistRoot(const KArgs& a, hipStream_t s) { LaunchHist<0>(a, s); }
void HistRange(const KArgs& a, hipStream_t s) { LaunchHist<2>(a, s); }

}  // namespace dev
}  // namespace lgbm_amd
