// One split step of device-resident growth, fused: the split picked into Step::cs is applied
// to the leaf's rows AND one child's rows are histogrammed, in the same pass over them
// (reference: data_partition.hpp Split + serial_tree_learner.cpp ConstructHistograms of the
// smaller leaf; the GPU learner's histogram256.cl).
//
// k_split, grid (split_grid, hist_tiles) of 1024-thread workgroups.  The parent's rows
// [begin, +count) of its index buffer are dealt out in row blocks (HistBlocksFor); each
// block is processed in sub-tiles of kSplitSub rows:
//  A. row per thread: index + split column byte (column-major copy) -> side; per-wave
//     ballots give the sub-tile's left count; one device-scope atomic per side reserves the
//     output slots (lefts grow up from the range's front, rights down from its back -- rows
//     keep their order inside a sub-tile, sub-tiles land in arrival order: histograms are
//     exact integer sums, so the order never changes a result); the rows of the histogrammed
//     child are compacted into an LDS row list.  Only column tile 0 writes the partition.
//  B. word per thread: the listed rows' bin words and (g, h) are gathered and added to the
//     LDS histogram of the tile (hist_common.h); row-sparse storage: kSparseTeam threads per
//     listed row walk its stored bins.  The block's histogram is stored as a partial when
//     its sub-tiles are done.
// The histogrammed child is the one with fewer rows by the split's estimated counts (the
// pick sets Step::hist_left): if the estimate is off, the larger child is histogrammed and
// the smaller one derived -- exact integer sums make both ways bit-identical.  The final
// cursors are the children's local sizes (StepChildren).
// Host-assisted growth runs the partition alone (HIST = false) on the split the host wrote.
#include "hist_common.h"

namespace lgbm_amd {
namespace dev {

namespace {

constexpr int kPartWaves = kPartThreads / kWave;
static_assert(kSplitRows * kPartWaves == kWave, "k_split: one wave lane per (row slot, wave) piece");
// phase B: independent row gathers per thread and pass (k_split's GR).  Narrow rows (<= 8
// words per tile) gather 2 (fewer VGPRs, ~150 rows per pass already), wide rows 8 (few rows
// per pass): A/B on the headline 10M x 28 (7 words) 8/4/2/1 rows = 4.39/4.28/4.21/4.26
// ms/iter; Yahoo 175 words 2 vs 8 rows = 23.3 vs 21.2, MS-LTR 35 words 19.1 vs 18.3
constexpr int kGatherNarrow = 2, kGatherWide = 8, kGatherNarrowMaxWords = 8;

__device__ __forceinline__ int ValidInWave(int valid, int k, int w) {
  return min(kWave, max(0, valid - k * kPartThreads - w * kWave));
}

}  // namespace

template <int GPW, int UNITS, bool HIST, int GR>
__global__ __launch_bounds__(kPartThreads) void k_split(KArgs a) {
  extern __shared__ unsigned long long lds[];  // [UNITS * tile_bins] histogram, then the row list
  __shared__ uint32_t cat_bits[kMaxCatWords];
  __shared__ int wl[kSplitRows][kPartWaves];
  __shared__ int lpre[kSplitRows][kPartWaves];
  __shared__ int hpre[kSplitRows][kPartWaves];
  __shared__ int base[2];
  __shared__ int nh_s;
  const long long t_entry = wall_clock64();
  Step* st = a.st;
  // ---- every load that does not depend on another one first (a single round trip)
  const int done = st->done;
  const CurSplit& cs = st->cs;
  const int s = cs.s;
  const int pb = cs.part_begin, pc = cs.part_count, src_buf = cs.src_buf;
  const int hist_left = st->hist_left;
  const int fbyte = cs.feat.gbyte, fwide = cs.feat.gwide;
  const int64_t fcol = cs.feat.col_off;
  Feature F;
  F.sub_lo = cs.feat.sub_lo;
  F.sub_hi = cs.feat.sub_hi;
  F.offset = cs.feat.offset;
  F.mfb = cs.feat.mfb;
  SplitRule r;
  r.threshold = cs.split.threshold;
  r.default_left = cs.split.default_left;
  r.is_cat = cs.split.is_categorical;
  r.missing_type = cs.feat.missing_type;
  r.default_bin = cs.feat.default_bin;
  r.max_bin = cs.feat.num_bin - 1;
  TileCtx t;
  if (HIST) InitTile<GPW>(a, &t);
  if (done) return;
  if (HIST && blockIdx.x == 0 && blockIdx.y == 0) {
    // the parent's splittable row, before the children's scans overwrite it (their scans skip
    // what the parent could not split on)
    const int8_t* prow = a.splittable + static_cast<size_t>(cs.parent_frow) * a.p.num_features;
    for (int f = threadIdx.x; f < a.p.num_features; f += kPartThreads) a.parent_flags[f] = prow[f];
  }
  const int ts = a.host_mode ? -1 : s;
  KTraceAt(a, ts, kTrSplitEntry, t_entry);
  const int nblk = HIST ? StepBlocks(a, pc) : (pc + kSplitSub - 1) / kSplitSub;
  if (static_cast<int>(blockIdx.x) >= nblk) return;
  if (r.is_cat && threadIdx.x < kMaxCatWords) cat_bits[threadIdx.x] = cs.split.cat_bits[threadIdx.x];
  const int chunk = (pc + nblk - 1) / nblk;
  const bool single = nblk == 1 && pc <= kSplitSub;  // sole sub-tile: no reservation round trip
  const bool writer = blockIdx.y == 0;
  const int32_t* src = src_buf ? a.tmp : a.idx;
  int32_t* dst = src_buf ? a.idx : a.tmp;
  int* rowlist = reinterpret_cast<int*>(lds + (HIST ? static_cast<size_t>(UNITS) * a.tile_bins : 0));
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  const bool hl = hist_left != 0;
  // voting-parallel: the histogrammed rows' fixed-point (g, h), summed by the threads of
  // word 0 of column tile 0 (each row once) -- that child's local sums
  const bool loc_sums = HIST && a.p.vote_phase != 0 && blockIdx.y == 0;
  long long loc_g = 0, loc_h = 0;
  // software pipeline over the workgroup's sub-tiles: the next sub-tile's row indices are
  // loaded while this one is processed, and its split-column bins before the sub-tile ends
  // (two dependent round trips off every sub-tile but the first; large parents run ~10
  // sub-tiles per workgroup)
  int row[kSplitRows];
  uint32_t gb[kSplitRows];
  auto load_rows = [&](int t0n, int r1n, int* rr) {
    const int vn = min(kSplitSub, r1n - t0n);
#pragma unroll
    for (int k = 0; k < kSplitRows; ++k) {
      const int i = k * kPartThreads + threadIdx.x;
      rr[k] = i < vn ? src[pb + t0n + i] : -1;
    }
  };
  if (static_cast<int>(blockIdx.x) < nblk) {
    const int r0 = blockIdx.x * chunk;
    load_rows(r0, min(pc, r0 + chunk), row);
#pragma unroll
    for (int k = 0; k < kSplitRows; ++k) gb[k] = row[k] >= 0 ? ColBin(a, row[k], fbyte, fwide, fcol) : 0u;
  }
  for (int kb = blockIdx.x; kb < nblk; kb += gridDim.x) {
    const int r0 = kb * chunk, r1 = min(pc, r0 + chunk);
    const bool first_trace = kb == static_cast<int>(blockIdx.x);
    for (int t0 = r0; t0 < r1; t0 += kSplitSub) {
      const int valid = min(kSplitSub, r1 - t0);
      const bool tr = first_trace && t0 == r0;
      // the next sub-tile of this workgroup (this block's next one, or the next block's first)
      int nt0 = t0 + kSplitSub, nr1 = r1;
      if (nt0 >= r1) {
        const int nkb = kb + gridDim.x;
        nt0 = nkb < nblk ? nkb * chunk : pc;
        nr1 = nkb < nblk ? min(pc, nt0 + chunk) : pc;
      }
      int nrow[kSplitRows];
      load_rows(nt0, nr1, nrow);
      // ---- A: sides
      if (HIST && t0 == r0) {
        __syncthreads();  // the previous block's partial was stored from this LDS
        for (int j = threadIdx.x; j < UNITS * t.nbins; j += kPartThreads) lds[j] = 0ull;
      }
      if (tr) KTrace(a, ts, kTrSplitRows);
      if (tr) KTrace(a, ts, kTrSplitSide);
      bool left[kSplitRows];
      unsigned long long mask[kSplitRows];
#pragma unroll
      for (int k = 0; k < kSplitRows; ++k) {
        left[k] = row[k] >= 0 && GoesLeft(r, cat_bits, FeatureBinOf(F, gb[k]));
        mask[k] = __ballot(left[k]);
      }
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < kSplitRows; ++k) wl[k][w] = __popcll(mask[k]);
      }
      __syncthreads();
      // wave 0: exclusive prefixes over the (k, wave) pieces in row order -- lefts and rows of
      // the histogrammed child -- and the left total; thread 0 reserves the output slots
      if (w == 0) {
        const int k = lane / kPartWaves, j = lane % kPartWaves;  // 64 lanes = kSplitRows x kPartWaves pieces
        const int c = wl[k][j];
        const int hc = hl ? c : ValidInWave(valid, k, j) - c;
        const int ci = WavePrefixIncl(c), hi = WavePrefixIncl(hc);
        lpre[k][j] = ci - c;
        hpre[k][j] = hi - hc;
        const int nl = __shfl(ci, kWave - 1, kWave);
        if (lane == kWave - 1) nh_s = hi;
        if (lane == 0 && writer) {
          if (single) {
            base[0] = base[1] = 0;
            st->cur_left = nl;
            st->cur_right = valid - nl;
          } else {
            base[0] = atomicAdd(&st->cur_left, nl);
            base[1] = atomicAdd(&st->cur_right, valid - nl);
          }
        }
      }
      __syncthreads();
      if (tr) KTrace(a, ts, kTrSplitResv);
      int nh = 0;
      if (HIST) {
        nh = nh_s;
#pragma unroll
        for (int k = 0; k < kSplitRows; ++k) {
          const unsigned long long vm = __ballot(row[k] >= 0);
          const unsigned long long hm = hl ? mask[k] : (~mask[k] & vm);
          if (row[k] >= 0 && left[k] == hl) rowlist[hpre[k][w] + __popcll(hm & lt)] = row[k];
        }
      }
      if (writer) {
        const int lbase = pb + base[0];
        const int rbase = pb + pc - 1 - base[1];
#pragma unroll
        for (int k = 0; k < kSplitRows; ++k) {
          if (row[k] >= 0) {
            const int lpos = lpre[k][w] + __popcll(mask[k] & lt);  // lefts before me in the sub-tile
            const int pos = k * kPartThreads + threadIdx.x;        // my position in the sub-tile
            if (left[k]) dst[lbase + lpos] = row[k];
            else dst[rbase - (pos - lpos)] = row[k];
          }
        }
      }
      if (HIST) __syncthreads();  // the row list is complete
      // ---- B: histogram of the listed rows
      if (HIST && t.rs < t.rpp) {
        const int wi = t.w0 + t.q;
        const uint32_t* bins32 = static_cast<const uint32_t*>(a.bins);
        const int64_t wpr = a.row_words;
        for (int j0 = t.rs; j0 < nh; j0 += GR * t.rpp) {
          int rr[GR];
#pragma unroll
          for (int k = 0; k < GR; ++k) {
            const int j = j0 + k * t.rpp;
            rr[k] = j < nh ? rowlist[j] : -1;
          }
          float2 v[GR];
          if constexpr (GPW == kSparseGPW) {
#pragma unroll
            for (int k = 0; k < GR; ++k) v[k] = GhAt(a, rr[k] >= 0 ? rr[k] : 0);
            if (tr && j0 == t.rs) KTrace(a, ts, kTrSplitGather);
            AddSparseRows<GR, UNITS>(a, lds, t, rr, v);
          } else {
            uint32_t wd[GR];
#pragma unroll
            for (int k = 0; k < GR; ++k) {
              const int x = rr[k] >= 0 ? rr[k] : 0;
              v[k] = GhAt(a, x);
              wd[k] = rr[k] >= 0 ? bins32[x * wpr + wi] : 0u;  // word 0: every bin skipped
            }
            if (tr && j0 == t.rs) KTrace(a, ts, kTrSplitGather);
#pragma unroll
            for (int k = 0; k < GR; ++k) AddRow<GPW, UNITS>(lds, t.goff, t.bits, wd[k], v[k], t.sg, t.sh);
          }
          if (loc_sums && t.q == 0) {
#pragma unroll
            for (int k = 0; k < GR; ++k) {
              if (rr[k] >= 0) {
                loc_g += __float2ll_rn(v[k].x * t.sg);
                loc_h += __float2ll_rn(v[k].y * t.sh);
              }
            }
          }
        }
      }
      // the next sub-tile's split-column bins (its rows arrived during this one)
#pragma unroll
      for (int k = 0; k < kSplitRows; ++k) {
        row[k] = nrow[k];
        gb[k] = row[k] >= 0 ? ColBin(a, row[k], fbyte, fwide, fcol) : 0u;
      }
      __syncthreads();  // row list, wave counts and bases are rewritten by the next sub-tile
      if (tr) KTrace(a, ts, kTrSplitAccum);
    }
    if (HIST) {
      unsigned long long* out = a.partials + static_cast<size_t>(kb) * UNITS * a.p.total_bins +
                                static_cast<size_t>(UNITS) * t.lo_bin;
      for (int j = threadIdx.x; j < UNITS * t.nbins; j += kPartThreads) out[j] = lds[j];
    }
  }
  if (loc_sums) {
    loc_g = WaveSum(loc_g);
    loc_h = WaveSum(loc_h);
    if (lane == 0 && (loc_g != 0 || loc_h != 0)) {
      atomicAdd(&st->loc_acc[0], static_cast<unsigned long long>(loc_g));
      atomicAdd(&st->loc_acc[1], static_cast<unsigned long long>(loc_h));
    }
  }
  KTrace(a, ts, kTrSplitExit);
}

static size_t SplitLds(const KArgs& a) {
  return sizeof(unsigned long long) * a.hist_units * static_cast<size_t>(a.tile_bins) + sizeof(int) * kSplitSub;
}

// dynamic LDS above 64 KiB must be enabled per kernel (up to the CU's 160 KiB)
template <typename K>
static void AllowLds(K kernel, int bytes) {
  if (bytes > 65536 && hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess) {
    (void)hipGetLastError();  // not fatal: launches above 64 KiB then fail loudly
  }
}

template <int GR>
static void LaunchSplit(const KArgs& a, hipStream_t s) {
  const dim3 grid(a.split_grid, a.hist_tiles);
  const size_t lds = SplitLds(a);

  if (a.sp_ptr != nullptr) {
    if (a.hist_units == 1) hipLaunchKernelGGL((k_split<kSparseGPW, 1, true, GR>), grid, dim3(kPartThreads), lds, s, a);
    else hipLaunchKernelGGL((k_split<kSparseGPW, 2, true, GR>), grid, dim3(kPartThreads), lds, s, a);
  } else if (a.hist_units == 1) {
    if (a.nibbles) hipLaunchKernelGGL((k_split<8, 1, true, GR>), grid, dim3(kPartThreads), lds, s, a);
    else if (a.bin_bytes == 1) hipLaunchKernelGGL((k_split<4, 1, true, GR>), grid, dim3(kPartThreads), lds, s, a);
    else if (a.bin_bytes == 2) hipLaunchKernelGGL((k_split<2, 1, true, GR>), grid, dim3(kPartThreads), lds, s, a);
    else hipLaunchKernelGGL((k_split<0, 1, true, GR>), grid, dim3(kPartThreads), lds, s, a);
  } else {
    if (a.nibbles) hipLaunchKernelGGL((k_split<8, 2, true, GR>), grid, dim3(kPartThreads), lds, s, a);
    else if (a.bin_bytes == 1) hipLaunchKernelGGL((k_split<4, 2, true, GR>), grid, dim3(kPartThreads), lds, s, a);
    else if (a.bin_bytes == 2) hipLaunchKernelGGL((k_split<2, 2, true, GR>), grid, dim3(kPartThreads), lds, s, a);
    else hipLaunchKernelGGL((k_split<0, 2, true, GR>), grid, dim3(kPartThreads), lds, s, a);
  }
}

void SplitStep(const KArgs& a, hipStream_t s, bool reduce) {
  if (a.sp_ptr != nullptr || a.tile_words <= kGatherNarrowMaxWords) LaunchSplit<kGatherNarrow>(a, s);
  else LaunchSplit<kGatherWide>(a, s);
  if (reduce) LaunchReduce<1>(a, s);
}

template <int GR>
static void AllowSplitLds(int mx) {
  AllowLds(k_split<8, 1, true, GR>, mx);
  AllowLds(k_split<8, 2, true, GR>, mx);
  AllowLds(k_split<4, 1, true, GR>, mx);
  AllowLds(k_split<2, 1, true, GR>, mx);
  AllowLds(k_split<4, 2, true, GR>, mx);
  AllowLds(k_split<2, 2, true, GR>, mx);
  AllowLds(k_split<0, 1, true, GR>, mx);
  AllowLds(k_split<0, 2, true, GR>, mx);
  AllowLds(k_split<kSparseGPW, 1, true, GR>, mx);
  AllowLds(k_split<kSparseGPW, 2, true, GR>, mx);
}

void PrepareSplitKernels(int mx) {
  AllowSplitLds<kGatherNarrow>(mx);
  AllowSplitLds<kGatherWide>(mx);
}

void Partition(const KArgs& a, hipStream_t s) {
  // one workgroup per CU: at most ~num_data / (kSplitSub * CUs) tile reservations each
  const int grid = std::max(1, std::min((a.num_data + kSplitSub - 1) / kSplitSub, NumCUs()));
  hipLaunchKernelGGL((k_split<4, 1, false, kGatherNarrow>), dim3(grid), dim3(kPartThreads), 0, s, a);
}

}  // namespace dev
}  // namespace lgbm_amd
