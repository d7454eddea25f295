// Round growth: speculative multi-leaf expansion of leaf-wise trees (device_types.h Round).
//
// The reference grows a tree one split at a time (serial_tree_learner.cpp:152-202: argmax over
// the leaves' best splits, split it, histogram + scan its children).  On the device every such
// step is a chain of dependent kernels whose latency (~50 us) does not shrink with the leaf, so
// a 63-leaf tree was 62 latency chains.  Expanding a leaf -- partitioning its rows by its best
// split, histogramming and scanning both children -- depends on that leaf's rows only, so a
// round expands the round_k current leaves of highest gain at once:
//
//   k_round_split   the fused partition + smaller-child histogram of every expansion; the
//                   round's rows are dealt out in row blocks of one common size, each block
//                   belongs to one expansion (partition_kernels.hip k_split, per expansion)
//   k_round_reduce  exact int64 sums of the partials of expansions with many row blocks
//   k_round_find    split scans of both children of every expansion, grid (features, 2 x
//                   round_k); the last workgroup of each child folds its per-feature results
//                   into the child's best split (cbest)
//   k_round_plan    one workgroup replays the sequential best-first order over the leaves:
//                   while the argmax leaf is expanded its split is accepted (split record,
//                   children become leaves 'leaf' and s + 1 with the expansion's statistics);
//                   the first argmax leaf that is not expanded ends the replay.  Then the next
//                   round's expansions are planned: the current unexpanded leaves of highest
//                   gain (the one that ended the replay first).  The plan runs in the last
//                   workgroup of k_round_find on one process; in distributed rounds the
//                   per-feature results are gathered first, and the last workgroup of
//                   k_round_childbest (the fold of the gathered results) runs it.
//
// The accepted sequence is the sequential one: a leaf's best split and its children's results
// depend only on its own rows, and the replay uses the host loop's argmax order (gain, real
// feature, leaf id).  Expansions not accepted before the tree is full cost work only.
// Pending expansions stay valid across rounds (leaves are only ever split by their best
// split), so no expansion is computed twice.
#include "hist_common.h"
#include "split_scan.h"

namespace lgbm_amd {
namespace dev {

namespace {

#ifndef LGBM_FIND_WAVE_OCC
#define LGBM_FIND_WAVE_OCC 2  // (one-wave scans without register spills: see split_kernels.hip)
#endif
#ifndef LGBM_ORACLE_SEQ
#define LGBM_ORACLE_SEQ 0  // A/B timing oracles only: 1 sequential (g, h) gathers, 2 also sequential row words
#endif
constexpr unsigned kRoundFlatMax = 128;  // split-scan grid rows up to this size count on one counter
constexpr int kRPartWaves = kPartThreads / kWave;
constexpr int kRGatherNarrow = 2, kRGatherWide = 8, kRGatherNarrowMaxWords = 8;
constexpr int kPlanThreads = 256;

__device__ __forceinline__ long long* RoundScratch(const KArgs& a, int parity, int j) {
  return a.scratch + (static_cast<size_t>(parity & 1) * a.round_k + j) * 2 * static_cast<size_t>(a.p.total_bins);
}

// a workgroup barrier ordering LDS only: nothing in the round's split kernel reads another
// wave's global stores, so the partition's stores (and the prefetched loads queued behind them
// on vmcnt) stay in flight across it -- __syncthreads' workgroup fence would drain them
__device__ __forceinline__ void LdsBarrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// the split column's bin of a row without branches (ColBin's source / width branches compile
// to divergent blocks whose waits drain every load in flight): one aligned dword load and a
// shift, from the column copy or the row-major matrix
struct ColSrc {
  const uint32_t* base;  // 4-byte aligned allocation (column copy or row-major matrix)
  int64_t off0;          // byte offset of row 0's bin
  int64_t stride;        // bytes between rows
  uint32_t mask;
  uint32_t shift;        // 4-bit groups in the row-major matrix: 4 for the high half of the byte
};
__device__ __forceinline__ ColSrc ColSource(const KArgs& a, int gbyte, int gwide, int64_t col_off) {
  ColSrc c;
  const bool col = a.bins_col != nullptr;
  c.base = col ? reinterpret_cast<const uint32_t*>(a.bins_col) : static_cast<const uint32_t*>(a.bins);
  c.off0 = col ? col_off : gbyte;
  c.stride = col ? (gwide == 1 ? 2 : 1) : 4 * static_cast<int64_t>(a.row_words);
  c.mask = gwide == 1 ? 0xffffu : (gwide >= 2 && !col ? 0xfu : 0xffu);
  c.shift = gwide == 3 && !col ? 4u : 0u;
  return c;
}
// (row < 0: none -- row 0 is read and the result dropped, so the load is unconditional)
__device__ __forceinline__ uint32_t ColBinNB(const ColSrc& c, int row) {
  const int64_t off = c.off0 + static_cast<int64_t>(max(row, 0)) * c.stride;
  const uint32_t wd = c.base[off >> 2];
  const uint32_t v = (wd >> ((static_cast<uint32_t>(off) & 3u) * 8u + c.shift)) & c.mask;
  return row < 0 ? 0u : v;
}

__device__ __forceinline__ int RValidInWave(int valid, int k, int w) {
  return min(kWave, max(0, valid - k * kPartThreads - w * kWave));
}

// per-expansion constants of the split kernel, staged in LDS once per workgroup
struct SplitExp {
  int pb, pc, src, dst, blk_off, nblk, hl, single;
  int fbyte, fwide;
  int sub_lo, sub_hi, offset, mfb;
  long long fcol;
  SplitRule r;
};

}  // namespace

// ---------------------------------------------------------------------------- k_round_split
// grid (split_grid, hist_tiles) of 1024-thread workgroups.  Row block kb of the round belongs
// to the expansion j with blk_off[j] <= kb < blk_off[j] + nblk[j]; it holds rows
// [(kb - blk_off[j]) * rpb, +rpb) of the expansion's parent range, processed in sub-tiles of
// kSplitSub rows exactly like k_split: sides by the split rule, per-wave ballots, one
// reservation per side and sub-tile on the expansion's cursors (lefts from the front of the
// range, rights from its back, in the other index buffer), the histogrammed child's rows
// compacted into an LDS row list and gathered into the tile's LDS histogram, stored as
// partial kb.  Only column tile 0 writes the partition.
#ifndef LGBM_SPLIT_WAVES
#define LGBM_SPLIT_WAVES 1  // waves per SIMD the register budget targets (A/B: 8 = two workgroups per CU)
#endif
template <int GPW, int UNITS, int GR, bool VOTE = false>
__global__ __launch_bounds__(kPartThreads) __attribute__((amdgpu_waves_per_eu(LGBM_SPLIT_WAVES))) void k_round_split(KArgs a) {
  extern __shared__ unsigned long long lds[];  // [UNITS * tile_bins] histogram, then the row list
  __shared__ SplitExp ex[kMaxRoundExp];
  __shared__ uint32_t cat_bits[kMaxRoundExp][kMaxCatWords];
  __shared__ int wl[kSplitRows][kRPartWaves];
  __shared__ int lpre[kSplitRows][kRPartWaves];
  __shared__ int hpre[kSplitRows][kRPartWaves];
  __shared__ int base[2];
  __shared__ int nh_s;
  Round* rd = a.rd;
  const int done = rd->done;
  const int nexp = rd->nexp, nblk = rd->nblk, rpb = rd->rpb;
  TileCtx t;
  InitTile<GPW>(a, &t);
  // the expansions' plans are loaded in the same batch as the round record (a slot past nexp
  // holds a stale plan that is never staged)
  SplitExp x;
  if (threadIdx.x < static_cast<unsigned>(kMaxRoundExp)) {
    const ExpPlan& e = rd->e[threadIdx.x];
    x.pb = e.part_begin;
    x.pc = e.part_count;
    x.src = e.src_buf;
    x.dst = e.dst_buf;
    x.blk_off = e.blk_off;
    x.nblk = e.nblk;
    x.hl = e.hist_left;
    x.single = e.nblk == 1 && e.part_count <= kSplitSub;
    x.fbyte = e.feat.gbyte;
    x.fwide = e.feat.gwide;
    x.fcol = e.feat.col_off;
    x.sub_lo = e.feat.sub_lo;
    x.sub_hi = e.feat.sub_hi;
    x.offset = e.feat.offset;
    x.mfb = e.feat.mfb;
    x.r.threshold = e.split.threshold;
    x.r.default_left = e.split.default_left;
    x.r.is_cat = e.split.is_categorical;
    x.r.missing_type = e.feat.missing_type;
    x.r.default_bin = e.feat.default_bin;
    x.r.max_bin = e.feat.num_bin - 1;
  }
  if (done || nexp <= 0 || static_cast<int>(blockIdx.x) >= nblk) return;
  if (threadIdx.x < static_cast<unsigned>(nexp)) ex[threadIdx.x] = x;
  for (int i = threadIdx.x; i < nexp * kMaxCatWords; i += kPartThreads) {
    const int j = i / kMaxCatWords;
    cat_bits[j][i % kMaxCatWords] = rd->e[j].split.is_categorical ? rd->e[j].split.cat_bits[i % kMaxCatWords] : 0u;
  }
  LdsBarrier();
  // LGBM_AMD_KTRACE: phase times of workgroup (0, 0) per round (wall clock, 10 ns ticks):
  // [stage, side, reserve, write, gather, tail, store, sub-tiles, rows, total]
  const bool tr = a.ktrace != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && rd->round < a.p.num_leaves;
  long long tacc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  long long tprev = 0, tstart = 0;
  if (tr) {
    tstart = wall_clock64();
    tprev = tstart;
  }
  auto stamp = [&](int k) {
    if (tr) {
      const long long now = wall_clock64();
      tacc[k] += now - tprev;
      tprev = now;
    }
  };
  stamp(0);
  // the expansion of row block kb
  auto exp_of = [&](int kb) {
    int j = 0;
    while (j + 1 < nexp && kb >= ex[j + 1].blk_off) ++j;
    return j;
  };
  int* rowlist = reinterpret_cast<int*>(lds + static_cast<size_t>(UNITS) * a.tile_bins);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  const bool writer = blockIdx.y == 0;
  // voting-parallel: the histogrammed rows' fixed-point (g, h), summed per row block by the
  // threads of word 0 of column tile 0 (each row once) -- that child's local sums
  // (a template flag: the accumulators cost the other variants registers -- Epsilon-shaped
  // wide rows 10.6 vs 11.8 ms/iter with a run-time flag)
  const bool loc_sums = VOTE && writer;
  long long loc_g = 0, loc_h = 0;
  int row[kSplitRows];
  uint32_t gb[kSplitRows];
  auto load_rows = [&](int jn, int t0n, int r1n, int* rr) {
    const int vn = min(kSplitSub, r1n - t0n);
    const int32_t* s = RowBuf(a, ex[jn].src);
    const int pbn = ex[jn].pb;
#pragma unroll
    for (int k = 0; k < kSplitRows; ++k) {
      const int i = k * kPartThreads + threadIdx.x;
      rr[k] = i < vn ? s[pbn + t0n + i] : -1;
    }
  };
  auto col_bins = [&](int jn, const int* rr, uint32_t* g) {
    const ColSrc c = ColSource(a, ex[jn].fbyte, ex[jn].fwide, ex[jn].fcol);
#pragma unroll
    for (int k = 0; k < kSplitRows; ++k) g[k] = ColBinNB(c, rr[k]);
  };
  {
    const int j = exp_of(blockIdx.x);
    const int r0 = (blockIdx.x - ex[j].blk_off) * rpb;
    load_rows(j, r0, min(ex[j].pc, r0 + rpb), row);
    col_bins(j, row, gb);
  }
  for (int kb = blockIdx.x; kb < nblk; kb += gridDim.x) {
    const int j = exp_of(kb);
    const SplitExp& X = ex[j];
    const int r0 = (kb - X.blk_off) * rpb, r1 = min(X.pc, r0 + rpb);
    const bool hl = X.hl != 0;
    Feature F;
    F.sub_lo = X.sub_lo;
    F.sub_hi = X.sub_hi;
    F.offset = X.offset;
    F.mfb = X.mfb;
    const SplitRule r = X.r;
    const uint32_t* cb = cat_bits[j];
    int32_t* dst = RowBuf(a, X.dst);
    for (int t0 = r0; t0 < r1; t0 += kSplitSub) {
      const int valid = min(kSplitSub, r1 - t0);
      // the next sub-tile of this workgroup: this block's next one, or the next block's first
      int nj = j, nt0 = t0 + kSplitSub, nr1 = r1;
      if (nt0 >= r1) {
        const int nkb = kb + gridDim.x;
        if (nkb < nblk) {
          nj = exp_of(nkb);
          nt0 = (nkb - ex[nj].blk_off) * rpb;
          nr1 = min(ex[nj].pc, nt0 + rpb);
        } else {
          nt0 = nr1 = 0;
        }
      }
      int nrow[kSplitRows];
      load_rows(nj, nt0, nr1, nrow);
      if (t0 == r0) {
        LdsBarrier();  // the previous block's partial was stored from this LDS
        for (int i = threadIdx.x; i < UNITS * t.nbins; i += kPartThreads) lds[i] = 0ull;
      }
      // ---- sides (this sub-tile's split-column bins were loaded during the previous one)
      bool left[kSplitRows];
      unsigned long long mask[kSplitRows];
#pragma unroll
      for (int k = 0; k < kSplitRows; ++k) {
        left[k] = row[k] >= 0 && GoesLeft(r, cb, FeatureBinOf(F, gb[k]));
        mask[k] = __ballot(left[k]);
      }
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < kSplitRows; ++k) wl[k][w] = __popcll(mask[k]);
      }
      LdsBarrier();
      stamp(1);
      if (tr) {
        tacc[7] += 1;
        tacc[8] += valid;
      }
      // ---- prefixes; the reservation is issued now and consumed after the gathers (its round
      // trip overlaps them)
      int res_l = 0, res_r = 0;
      int nl_w0 = 0;
      if (w == 0) {
        const int k = lane / kRPartWaves, jj = lane % kRPartWaves;
        const int c = wl[k][jj];
        const int hc = hl ? c : RValidInWave(valid, k, jj) - c;
        const int ci = WavePrefixIncl(c), hi = WavePrefixIncl(hc);
        lpre[k][jj] = ci - c;
        hpre[k][jj] = hi - hc;
        nl_w0 = __shfl(ci, kWave - 1, kWave);
        if (lane == kWave - 1) nh_s = hi;
      }
      LdsBarrier();
      stamp(2);
      const int nh = nh_s;
#pragma unroll
      for (int k = 0; k < kSplitRows; ++k) {
        const unsigned long long vm = __ballot(row[k] >= 0);
        const unsigned long long hm = hl ? mask[k] : (~mask[k] & vm);
        if (row[k] >= 0 && left[k] == hl) rowlist[hpre[k][w] + __popcll(hm & lt)] = row[k];
      }
      // the next sub-tile's split-column bins: in flight during the gathers
      uint32_t ngb[kSplitRows];
      col_bins(nj, nrow, ngb);
      // (issued after the column loads: a wait for those would otherwise cover the atomics)
      if (w == 0 && lane == 0 && writer && !X.single) {
        res_l = atomicAdd(&rd->cur[j][0], nl_w0);
        res_r = atomicAdd(&rd->cur[j][1], valid - nl_w0);
      }
      LdsBarrier();  // the row list is complete
      stamp(3);
      if (t.rs < t.rpp) {
        const int wi = t.w0 + t.q;
        const uint32_t* bins32 = static_cast<const uint32_t*>(a.bins);
        const int64_t wpr = a.row_words;
        if constexpr (GPW == kSparseGPW) {
          for (int j0 = t.rs; j0 < nh; j0 += GR * t.rpp) {
            int rr[GR];
#pragma unroll
            for (int k = 0; k < GR; ++k) {
              const int jr = j0 + k * t.rpp;
              rr[k] = jr < nh ? rowlist[jr] : -1;
            }
            float2 v[GR];
#pragma unroll
            for (int k = 0; k < GR; ++k) v[k] = GhAt(a, rr[k] >= 0 ? rr[k] : 0);
            AddSparseRows<GR, UNITS>(a, lds, t, rr, v);
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
        } else {
          // software-pipelined: the next batch's row words and (g, h) are in flight while this
          // batch's LDS atomics run
          const int step = GR * t.rpp;
          uint32_t wd[GR];
          float2 v[GR];
          auto fetch = [&](int j0, uint32_t* w_, float2* v_) {
#pragma unroll
            for (int k = 0; k < GR; ++k) {
              const int jr = j0 + k * t.rpp;
              const int x = jr < nh ? rowlist[jr] : -1;
#if LGBM_ORACLE_SEQ
              // timing oracle (wrong histograms): the gathers read the parent range's positions
              // instead of the rows, i.e. leaf-ordered copies that cost nothing to maintain
              const int xp = X.pb + t0 + jr;
              v_[k] = GhAt(a, x >= 0 ? xp : 0);
              w_[k] = x >= 0 ? bins32[static_cast<int64_t>(LGBM_ORACLE_SEQ >= 2 ? xp : x) * wpr + wi] : 0u;
#else
              v_[k] = GhAt(a, x >= 0 ? x : 0);
              w_[k] = x >= 0 ? bins32[static_cast<int64_t>(x) * wpr + wi] : 0u;  // word 0: every bin skipped
#endif
            }
          };
          if (t.rs < nh) fetch(t.rs, wd, v);
          for (int j0 = t.rs; j0 < nh; j0 += step) {
            uint32_t wn[GR];
            float2 vn[GR];
            if (j0 + step < nh) fetch(j0 + step, wn, vn);
#pragma unroll
            for (int k = 0; k < GR; ++k) AddRow<GPW, UNITS>(lds, t.goff, t.bits, wd[k], v[k], t.sg, t.sh);
            if (loc_sums && t.q == 0) {
#pragma unroll
              for (int k = 0; k < GR; ++k) {
                if (j0 + k * t.rpp < nh) {
                  loc_g += __float2ll_rn(v[k].x * t.sg);
                  loc_h += __float2ll_rn(v[k].y * t.sh);
                }
              }
            }
#pragma unroll
            for (int k = 0; k < GR; ++k) {
              wd[k] = wn[k];
              v[k] = vn[k];
            }
          }
        }
      }
      stamp(4);
      // ---- the partition (column tile 0): slots from the reservation
      if (w == 0 && lane == 0 && writer) {
        if (X.single) {
          base[0] = base[1] = 0;
          rd->cur[j][0] = nl_w0;
          rd->cur[j][1] = valid - nl_w0;
        } else {
          base[0] = res_l;
          base[1] = res_r;
        }
      }
      LdsBarrier();
      if (writer) {
        const int lbase = X.pb + base[0];
        const int rbase = X.pb + X.pc - 1 - base[1];
#pragma unroll
        for (int k = 0; k < kSplitRows; ++k) {
          if (row[k] >= 0) {
            const int lpos = lpre[k][w] + __popcll(mask[k] & lt);
            const int pos = k * kPartThreads + threadIdx.x;
            if (left[k]) dst[lbase + lpos] = row[k];
            else dst[rbase - (pos - lpos)] = row[k];
          }
        }
      }
#pragma unroll
      for (int k = 0; k < kSplitRows; ++k) {
        row[k] = nrow[k];
        gb[k] = ngb[k];
      }
      LdsBarrier();  // row list, wave counts, prefixes and bases are rewritten by the next sub-tile
      stamp(5);
    }
    if (r0 >= r1) {  // (an empty block still stores a zero partial)
      LdsBarrier();
      for (int i = threadIdx.x; i < UNITS * t.nbins; i += kPartThreads) lds[i] = 0ull;
      LdsBarrier();
    }
    unsigned long long* out = a.partials + static_cast<size_t>(kb) * UNITS * a.p.total_bins +
                              static_cast<size_t>(UNITS) * t.lo_bin;
    for (int i = threadIdx.x; i < UNITS * t.nbins; i += kPartThreads) out[i] = lds[i];
    if (loc_sums) {  // (uniform: every lane of every wave takes part in the sums)
      const long long bg = WaveSum(loc_g), bh = WaveSum(loc_h);
      if (lane == 0 && (bg != 0 || bh != 0)) {
        atomicAdd(&rd->loc_acc[j][0], static_cast<unsigned long long>(bg));
        atomicAdd(&rd->loc_acc[j][1], static_cast<unsigned long long>(bh));
      }
      loc_g = loc_h = 0;
    }
    stamp(6);
  }
  if (tr) {
    tacc[9] = wall_clock64() - tstart;
    long long* o = a.ktrace + static_cast<size_t>(rd->round) * kTraceSlots;
    for (int k = 0; k < 10; ++k) o[k] = tacc[k];
    o[10] = nexp;
    o[11] = nblk;
  }
}

// ----------------------------------------------------------------- k_round_part / k_round_hist
// The same round as k_round_split in two streaming kernels (KArgs::round_fused = 0): the
// partition alone (index + split-column byte per row, ballots, one reservation per side and
// sub-tile, no LDS histogram), then the histograms of the histogrammed children, whose rows
// are now one contiguous range of the other index buffer each -- row blocks of rpb rows read
// with kRowsInFlight independent gathers per thread, like the root histogram.  Block k of
// expansion j's child is partial blk_off[j] + k (blk_off reserves ceil(parent rows / rpb)).
__device__ __forceinline__ int RoundHistRows(const Round* rd, int j, int* begin) {
  const ExpPlan& e = rd->e[j];
  const int tl = rd->cur[j][0];
  *begin = e.part_begin + (e.hist_left ? 0 : tl);
  return e.hist_left ? tl : e.part_count - tl;
}
// row blocks of expansion j's histogram (fused: blocks of the parent's rows)
__device__ __forceinline__ int RoundHistBlocks(const KArgs& a, const Round* rd, int j) {
  if (a.round_fused) return rd->e[j].nblk;
  int b;
  const int h = RoundHistRows(rd, j, &b);
  return (h + rd->rpb - 1) / rd->rpb;
}

__global__ __launch_bounds__(kPartThreads) void k_round_part(KArgs a) {
  __shared__ SplitExp ex[kMaxRoundExp];
  __shared__ uint32_t cat_bits[kMaxRoundExp][kMaxCatWords];
  __shared__ int wl[kSplitRows][kRPartWaves];
  __shared__ int lpre[kSplitRows][kRPartWaves];
  __shared__ int base[2];
  Round* rd = a.rd;
  const int done = rd->done;
  const int nexp = rd->nexp, nblk = rd->nblk, rpb = rd->rpb;
  if (done || nexp <= 0 || static_cast<int>(blockIdx.x) >= nblk) return;
  if (threadIdx.x < static_cast<unsigned>(nexp)) {
    const ExpPlan& e = rd->e[threadIdx.x];
    SplitExp x;
    x.pb = e.part_begin;
    x.pc = e.part_count;
    x.src = e.src_buf;
    x.dst = e.dst_buf;
    x.blk_off = e.blk_off;
    x.nblk = e.nblk;
    x.hl = e.hist_left;
    x.single = e.nblk == 1 && e.part_count <= kSplitSub;
    x.fbyte = e.feat.gbyte;
    x.fwide = e.feat.gwide;
    x.fcol = e.feat.col_off;
    x.sub_lo = e.feat.sub_lo;
    x.sub_hi = e.feat.sub_hi;
    x.offset = e.feat.offset;
    x.mfb = e.feat.mfb;
    x.r.threshold = e.split.threshold;
    x.r.default_left = e.split.default_left;
    x.r.is_cat = e.split.is_categorical;
    x.r.missing_type = e.feat.missing_type;
    x.r.default_bin = e.feat.default_bin;
    x.r.max_bin = e.feat.num_bin - 1;
    ex[threadIdx.x] = x;
  }
  for (int i = threadIdx.x; i < nexp * kMaxCatWords; i += kPartThreads) {
    const int j = i / kMaxCatWords;
    cat_bits[j][i % kMaxCatWords] = rd->e[j].split.is_categorical ? rd->e[j].split.cat_bits[i % kMaxCatWords] : 0u;
  }
  __syncthreads();
  auto exp_of = [&](int kb) {
    int j = 0;
    while (j + 1 < nexp && kb >= ex[j + 1].blk_off) ++j;
    return j;
  };
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  int row[kSplitRows];
  uint32_t gb[kSplitRows];
  auto load_rows = [&](int jn, int t0n, int r1n, int* rr) {
    const int vn = min(kSplitSub, r1n - t0n);
    const int32_t* s = RowBuf(a, ex[jn].src);
    const int pbn = ex[jn].pb;
#pragma unroll
    for (int k = 0; k < kSplitRows; ++k) {
      const int i = k * kPartThreads + threadIdx.x;
      rr[k] = i < vn ? s[pbn + t0n + i] : -1;
    }
  };
  auto col_bins = [&](int jn, const int* rr, uint32_t* g) {
    const ColSrc c = ColSource(a, ex[jn].fbyte, ex[jn].fwide, ex[jn].fcol);
#pragma unroll
    for (int k = 0; k < kSplitRows; ++k) g[k] = ColBinNB(c, rr[k]);
  };
  {
    const int j = exp_of(blockIdx.x);
    const int r0 = (blockIdx.x - ex[j].blk_off) * rpb;
    load_rows(j, r0, min(ex[j].pc, r0 + rpb), row);
    col_bins(j, row, gb);
  }
  for (int kb = blockIdx.x; kb < nblk; kb += gridDim.x) {
    const int j = exp_of(kb);
    const SplitExp& X = ex[j];
    const int r0 = (kb - X.blk_off) * rpb, r1 = min(X.pc, r0 + rpb);
    Feature F;
    F.sub_lo = X.sub_lo;
    F.sub_hi = X.sub_hi;
    F.offset = X.offset;
    F.mfb = X.mfb;
    const SplitRule r = X.r;
    const uint32_t* cb = cat_bits[j];
    int32_t* dst = RowBuf(a, X.dst);
    for (int t0 = r0; t0 < r1; t0 += kSplitSub) {
      const int valid = min(kSplitSub, r1 - t0);
      int nj = j, nt0 = t0 + kSplitSub, nr1 = r1;
      if (nt0 >= r1) {
        const int nkb = kb + gridDim.x;
        if (nkb < nblk) {
          nj = exp_of(nkb);
          nt0 = (nkb - ex[nj].blk_off) * rpb;
          nr1 = min(ex[nj].pc, nt0 + rpb);
        } else {
          nt0 = nr1 = 0;
        }
      }
      int nrow[kSplitRows];
      load_rows(nj, nt0, nr1, nrow);
      bool left[kSplitRows];
      unsigned long long mask[kSplitRows];
#pragma unroll
      for (int k = 0; k < kSplitRows; ++k) {
        left[k] = row[k] >= 0 && GoesLeft(r, cb, FeatureBinOf(F, gb[k]));
        mask[k] = __ballot(left[k]);
      }
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < kSplitRows; ++k) wl[k][w] = __popcll(mask[k]);
      }
      __syncthreads();
      if (w == 0) {
        const int k = lane / kRPartWaves, jj = lane % kRPartWaves;
        const int c = wl[k][jj];
        const int ci = WavePrefixIncl(c);
        lpre[k][jj] = ci - c;
        const int nl = __shfl(ci, kWave - 1, kWave);
        if (lane == 0) {
          if (X.single) {
            base[0] = base[1] = 0;
            rd->cur[j][0] = nl;
            rd->cur[j][1] = valid - nl;
          } else {
            base[0] = atomicAdd(&rd->cur[j][0], nl);
            base[1] = atomicAdd(&rd->cur[j][1], valid - nl);
          }
        }
      }
      __syncthreads();
      const int lbase = X.pb + base[0];
      const int rbase = X.pb + X.pc - 1 - base[1];
#pragma unroll
      for (int k = 0; k < kSplitRows; ++k) {
        if (row[k] >= 0) {
          const int lpos = lpre[k][w] + __popcll(mask[k] & lt);
          const int pos = k * kPartThreads + threadIdx.x;
          if (left[k]) dst[lbase + lpos] = row[k];
          else dst[rbase - (pos - lpos)] = row[k];
        }
      }
#pragma unroll
      for (int k = 0; k < kSplitRows; ++k) row[k] = nrow[k];
      col_bins(nj, row, gb);
      __syncthreads();  // wave counts and bases are rewritten by the next sub-tile
    }
  }
}

template <int GPW, int UNITS>
__global__ __launch_bounds__(kHistThreads) void k_round_hist(KArgs a) {
  extern __shared__ unsigned long long lds[];
  __shared__ int s_off[kMaxRoundExp + 1], s_beg[kMaxRoundExp], s_rows[kMaxRoundExp], s_buf[kMaxRoundExp],
      s_cap[kMaxRoundExp];
  const Round* rd = a.rd;
  if (rd->done) return;
  const int nexp = rd->nexp, rpb = rd->rpb;
  if (nexp <= 0) return;
  TileCtx t;
  InitTile<GPW>(a, &t);
  if (threadIdx.x == 0) {
    int off = 0;
    for (int j = 0; j < nexp; ++j) {
      int b;
      const int h = RoundHistRows(rd, j, &b);
      s_off[j] = off;
      s_beg[j] = b;
      s_rows[j] = h;
      s_buf[j] = rd->e[j].dst_buf;
      s_cap[j] = rd->e[j].blk_off;
      off += (h + rpb - 1) / rpb;
    }
    s_off[nexp] = off;
  }
  __syncthreads();
  const int total = s_off[nexp];
  const size_t pstride = static_cast<size_t>(UNITS) * a.p.total_bins;
  for (int kb = blockIdx.x; kb < total; kb += gridDim.x) {
    int j = 0;
    while (j + 1 < nexp && kb >= s_off[j + 1]) ++j;
    const int k = kb - s_off[j];
    const int r0 = s_beg[j] + k * rpb, r1 = min(s_beg[j] + s_rows[j], r0 + rpb);
    HistBlock<false, GPW, UNITS>(a, lds, RowBuf(a, s_buf[j]), r0, r1, t,
                                 a.partials + static_cast<size_t>(s_cap[j] + k) * pstride + static_cast<size_t>(UNITS) * t.lo_bin);
  }
}

// --------------------------------------------------------------------------- k_round_reduce
// grid (bins / 256, kReduceRows, round_k): the partials of expansion blockIdx.z with more than
// kDirectChunk row blocks summed into its reduce buffer (pre-zeroed by the previous round's
// split scans when the chunks combine with atomics)
template <int UNITS>
__global__ __launch_bounds__(256) void k_round_reduce(KArgs a) {
  const Round* rd = a.rd;
  if (rd->done) return;
  const int j = blockIdx.z;
  if (j >= rd->nexp) return;
  const int nblk = RoundHistBlocks(a, rd, j);
  // data-parallel: every expansion reduced, into the owner-major send buffer (voting keeps
  // rank-local histograms: the single-process layout)
  const bool dp = a.p.data_parallel != 0 && !a.round_vote;
  if (!dp && nblk <= kDirectChunk) return;  // summed by the split scan
  if (static_cast<int>(blockIdx.y) * kReduceChunk >= nblk) return;
  const int bin = blockIdx.x * blockDim.x + threadIdx.x;
  const int nb = a.p.total_bins;
  if (bin >= nb) return;
  const size_t pstride = static_cast<size_t>(UNITS) * nb;
  const unsigned long long* part = a.partials + static_cast<size_t>(rd->e[j].blk_off) * pstride;
  long long g = 0, h = 0;
  for (int k0 = blockIdx.y * kReduceChunk; k0 < nblk; k0 += gridDim.y * kReduceChunk) {
    const unsigned long long* p = part + k0 * pstride + static_cast<size_t>(UNITS) * bin;
    const int kn = min(kReduceChunk, nblk - k0);
    unsigned long long v0[kReduceChunk], v1[kReduceChunk];
#pragma unroll
    for (int k = 0; k < kReduceChunk; ++k) {
      v0[k] = k < kn ? p[k * pstride] : 0ull;
      v1[k] = (UNITS == 2 && k < kn) ? p[k * pstride + 1] : 0ull;
    }
#pragma unroll
    for (int k = 0; k < kReduceChunk; ++k) {
      long long pg, ph;
      UnpackPartial(v0[k], v1[k], UNITS, &pg, &ph);
      g += pg;
      h += ph;
    }
  }
  long long* out = RoundScratch(a, rd->round, j);
  int pos = bin;
  if (dp) {
    const int rp = a.rs_pos[bin], owner = rp / a.rs_block;
    if (rp < 0) return;  // (a group no rank scans this tree)
    out = a.round_send;
    pos = (owner * a.round_k + j) * a.rs_block + (rp - owner * a.rs_block);
  }
  if (nblk <= kReduceChunk) {
    out[2 * pos] = g;
    out[2 * pos + 1] = h;
  } else {
    atomicAdd(reinterpret_cast<unsigned long long*>(&out[2 * pos]), static_cast<unsigned long long>(g));
    atomicAdd(reinterpret_cast<unsigned long long*>(&out[2 * pos + 1]), static_cast<unsigned long long>(h));
  }
}

// the plan's LDS tables (RoundPlanLds bytes): node tables (gain, -inf when the node has no
// split; real feature; first child or -1), leaf tables (gain, real feature, node; accepted
// leaves / nodes) and the prediction's copies of the leaf tables (+ levels below the leaf)
struct PlanTables {
  double *ng, *tg, *sg;
  unsigned long long* qkey;  // the bottleneck prediction's region: order keys and nodes (PredictBottleneck)
  int *nrf, *nch, *nfi, *trf, *tnode, *acc, *accn, *srf, *snode, *svd, *qn;
  __device__ PlanTables(unsigned char* lds, int NN, int L) {
    ng = reinterpret_cast<double*>(lds);
    tg = ng + NN;
    sg = tg + L;
    qkey = reinterpret_cast<unsigned long long*>(sg + L);
    nrf = reinterpret_cast<int*>(qkey + NN);
    nch = nrf + NN;
    nfi = nch + NN;  // the node's best split feature (inner index; -1: none)
    trf = nfi + NN;
    tnode = trf + L;
    acc = tnode + L;
    accn = acc + L;
    srf = accn + L;
    snode = srf + L;
    svd = snode + L;
    qn = svd + L;
  }
};

template <bool ROOT, int NT, bool XT = false>
__device__ void RoundPlanBody(const KArgs& a, unsigned char* plan_lds);

// ----------------------------------------------------------------------------- k_round_find
template <int KIND, int NT>
struct RoundFindShared {
  BlockScratch<NT> sc;
  ScanScratch<NT> ssc;
  Cand sc2[NT / kWave];
  typename std::conditional<KIND == 2, CatScratchT<kFindCatNarrow>,
                            typename std::conditional<KIND == 3, CatScratchT<kFindMaxCatBins>, int>::type>::type cat_sc;
  unsigned long long s_red[2 * NT];
  ArgC arg[NT / kWave];
};

// per-feature result slot of child y, inner feature f (distributed: rank-major blocks)
__device__ __forceinline__ size_t RoundFbIndex(const KArgs& a, int y, int f) {
  if (!a.round_dist || a.round_vote) return static_cast<size_t>(y) * a.p.num_features + f;
  const int fi = a.fb_index[f], per = 2 * a.max_owned;
  const int owner = fi / per, local = fi - owner * per;
  return (static_cast<size_t>(owner) * 2 * a.round_k + y) * a.max_owned + local;
}

// the best split of child y (2j + lr) of the round, node `node`, from its per-feature
// results, by the child's last split-scan workgroup (SplitInfo order: larger gain, then
// smaller real feature)
template <int KIND, int NT>
__device__ void ChildBest(const KArgs& a, int y, int node, RoundFindShared<KIND, NT>& sh) {
  const int NF = a.p.num_features, tid = threadIdx.x;
  const FeatureBest* fb0 = a.feat_best;
  constexpr int kB = 8;
  ArgC c = ArgNone();
#pragma unroll 1
  for (int i0 = tid; i0 < NF; i0 += kB * NT) {
    double cg[kB];
    int crf[kB], cf[kB];
#pragma unroll
    for (int k = 0; k < kB; ++k) {
      const int i = i0 + k * NT;
      cf[k] = -1;
      if (i < NF) {
        const FeatureBest& r = fb0[RoundFbIndex(a, y, i)];
        cg[k] = r.gain;
        crf[k] = r.real_feature;
        cf[k] = r.feature;
      }
    }
#pragma unroll
    for (int k = 0; k < kB; ++k) {
      if (cf[k] >= 0 && (c.idx < 0 || SplitBetter(cg[k], crf[k], c.g, c.rf))) {
        c.g = cg[k];
        c.rf = crf[k];
        c.idx = i0 + k * NT;
      }
    }
  }
  c = ArgWaveBest(c);
  if ((tid & 63) == 0) sh.arg[tid >> 6] = c;
  __syncthreads();
  ArgC b = sh.arg[0];
#pragma unroll
  for (int k = 1; k < NT / kWave; ++k) ArgTake(&b, sh.arg[k]);
  const size_t ci = static_cast<size_t>(node);
  FeatureBest* dst = a.cbest + ci;
  // (write-through: with KArgs::plan_in_find another workgroup of this launch plans from them)
  if (tid == 0) {
    if (b.idx >= 0 && b.g != -INFINITY) {
      const size_t wi = RoundFbIndex(a, y, b.idx);
      const FeatureBest w = fb0[wi];
      PublishRecord(dst, w);
      if (w.ncat > 0) {
        PublishCatCopy(a.cbest_cat + ci * kMaxCatWords, a.feat_cat + wi * kMaxCatWords);
      }
    } else {
      FeatureBest none = {};
      none.gain = -INFINITY;
      none.feature = none.real_feature = -1;
      PublishRecord(dst, none);
    }
  }
}

// split scan of one (feature, child of expansion j): grid (num_scan or categorical features,
// 2 x round_k); child y = 2j + lr (0 left, 1 right).  The histogrammed child takes the
// expansion's reduced histogram (or sums its few partials itself) into its new slot; the
// other one subtracts it from the parent's slot in place (exact int64).  Children of an
// expansion that cannot be split (max_depth, min_data_in_leaf) are not scanned.
template <int KIND, bool SIMPLE, int NT, bool VG = false, bool PIF = true>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT == kWave ? LGBM_FIND_WAVE_OCC : 1))) void k_round_find(KArgs a) {
  constexpr bool CAT = KIND >= 2;  // (3: the wide categorical variant)
  extern __shared__ double s_bins[];  // [2][max_feature_bins] dequantised (g, h), if they fit
  __shared__ RoundFindShared<KIND, NT> sh;
  __shared__ int s_last;
  Round* rd = a.rd;
  const long long t_entry = a.ktrace != nullptr ? wall_clock64() : 0;
  const int by = static_cast<int>(blockIdx.y);
  const int y = by, j = y >> 1, lr = y & 1;
  // voting-parallel rounds (KArgs::round_vote): Params::vote_phase 1 scans every feature on this
  // rank's histograms, sums and counts; 2 scans the features the vote elected for child y
  // (KArgs::vote_list) on their all-reduced histograms (KArgs::vote_hist)
  // (VG: the global scan is an instantiation of its own -- a run-time flag put the elected
  // feature's load in front of every scan's feature load: +10% on wide data)
  const bool vote_local = a.round_vote && a.p.vote_phase == 1;
  constexpr bool vote_global = VG;
  int f = CAT ? a.cat_list[blockIdx.x] : (a.feat_list != nullptr ? a.feat_list[blockIdx.x] : static_cast<int>(blockIdx.x));
  if constexpr (VG) f = a.vote_list[y * a.p.vote_k + blockIdx.x];
  const bool vote_empty = f < 0;  // (an empty elected slot, or a padded owner slot)
  if (vote_empty) f = 0;
  const int tid = threadIdx.x;
  const int NF = a.p.num_features;
  const int units = a.hist_units;
  // the round record, the expansion's plan and the feature in one batch of loads, the
  // finished-tree check included (it used to cost a round trip of its own)
  const int done = rd->done, nexp = rd->nexp, rround = rd->round;
  const ExpPlan& E = rd->e[j];
  const int pc = E.part_count, tl = rd->cur[j][0];
  const int e_gl0 = E.lr[0].global_count, e_gl1 = E.lr[1].global_count, e_hl = E.hist_left;
  const int e_slot_new = E.slot_new, e_slot_parent = E.slot_parent, e_frow = E.frow_child[lr];
  const int e_frow_parent = E.frow_parent, blk_off = E.blk_off, e_nblk = E.nblk;
  const ChildStats cl = E.lr[lr];
  const Feature F = a.feat[f];
  const int8_t tree_used = a.tree_mask[f];
  if (done) return;
  if (a.ktrace != nullptr && blockIdx.x == 0 && by == 0 && threadIdx.x == 0 && rround < a.p.num_leaves) {
    a.ktrace[static_cast<size_t>(rround) * kTraceSlots + 25] = wall_clock64();
  }
  const int parity = rround & 1;
  const int nbf = F.num_bin - F.offset;
  const double ig = a.scales[2], ih = a.scales[3];
  // LGBM_AMD_KTRACE: the planning workgroup's own path through the scan (slots 26..31: entry,
  // inputs loaded, histogram staged, scan done, child's arrival, child's fold done)
  const bool ktw = a.ktrace != nullptr && tid == 0 && rround < a.p.num_leaves;
  long long kt[6] = {0, 0, 0, 0, 0, 0};
  if (ktw) {
    kt[0] = t_entry;
    kt[1] = wall_clock64();
  }
  // this feature's bins of expansion j's reduce buffer for the next round (every expansion
  // slot: the next round may use any)
  const bool dp = a.p.data_parallel != 0;
  const bool owner = dp && !a.round_vote;  // (data-parallel: reduce-scattered to the feature owners)
  if (!CAT && lr == 0 && !owner && !vote_global) {
    long long* nxt = RoundScratch(a, parity + 1, j);
    for (int i = tid; i < 2 * nbf; i += NT) nxt[2 * F.hist_offset + i] = 0;
  }
  if (!CAT && owner && a.round_send != nullptr) {
    // data-parallel: the next round's owner-major send buffer, cleared by every workgroup's
    // share (this round's reduce-scatter has read it) -- no memset node per round
    const size_t total = static_cast<size_t>(a.p.world) * a.round_k * a.rs_block * 2;
    const size_t nwg = static_cast<size_t>(gridDim.x) * gridDim.y;
    const size_t per = (total + nwg - 1) / nwg;
    const size_t b0 = (static_cast<size_t>(by) * gridDim.x + blockIdx.x) * per;
    const size_t b1 = min(total, b0 + per);
    for (size_t i = b0 + tid; i < b1; i += NT) a.round_send[i] = 0;
  }
  if (j >= nexp || vote_empty) return;
  if (vote_global && CAT && !F.is_cat) return;  // (an elected numerical feature)
  // data-parallel: the children's global counts from the split's estimates (reference
  // data_parallel_tree_learner.cpp: global leaf counts from the SplitInfo)
  const int lc = dp ? e_gl0 : tl, rc = dp ? e_gl1 : pc - tl;
  const int md = SkipMinData(a);
  const bool skip = (a.p.max_depth > 0 && cl.depth >= a.p.max_depth) || (lc < 2 * md && rc < 2 * md);
  const bool is_hist = (lr == 0) == (e_hl != 0);
  const int slot = is_hist ? e_slot_new : e_slot_parent;
  const int frow = e_frow;
  const int nblk = a.round_fused ? e_nblk : RoundHistBlocks(a, rd, j);
  // (per-node sampling: the parent leaf's row of the reference's flags, KArgs::leaf_rows)
  // (voting: every feature is scanned and its local histogram built -- the vote may elect a
  // feature the parent's local scan could not split, whose local histogram the reference's
  // learner would not have built (VotingParallelTreeLearner::FindBestSplits builds the tree's
  // sample minus those, then copies the elected ones' histograms))
  const int8_t parent_flag = a.leaf_rows != nullptr ? a.leaf_rows[static_cast<size_t>(e_frow_parent) * NF + f]
                                                    : a.splittable[static_cast<size_t>(e_frow_parent) * NF + f];
  const int8_t parent_ok = a.round_vote ? 1 : parent_flag;
  FeatureBest* fb_out = &a.feat_best[RoundFbIndex(a, y, f)];
  int8_t* flags = a.splittable + static_cast<size_t>(frow) * NF;
  const SplitParams& p = a.p.sp;
  FeatureBest o;
  o.gain = -INFINITY;
  o.feature = -1;
  o.real_feature = -1;
  o.thr = 0;
  o.default_left = 1;
  o.lc = o.rc = 0;
  o.mono = 0;
  o.ncat = 0;
  o.flag = -1;
  o.pad = 0;
  o.lg = o.lh = o.rg = o.rh = o.lo = o.ro = 0.0;
  bool write = true;
  if (KIND == 1 && F.is_cat) {
    write = false;  // the categorical kernel scans it
  } else if (skip) {
    // (both children keep gain -inf: never split)
  } else if (tree_used && !parent_ok) {
    // the parent could not split on f: neither child evaluates it (SerialTreeLearner::FindBestSplits)
    if (tid == 0) flags[f] = 0;
    o.flag = 0;
  } else if (tree_used && (!F.is_cat || F.num_bin <= kFindMaxCatBins)) {
    // interaction constraints: like a sampled-out feature, a disallowed one is not evaluated
    // but keeps its histogram (descendants subtract it); voting's local scan evaluates it (its
    // features are the tree's sample and the parent's flags only)
    bool used = true;
    if (a.feat_icmask != nullptr && !vote_local && !IcAny(cl.icmask & a.feat_icmask[f])) used = false;
    LeafCtx L;
    L.sg = cl.sum_g;
    L.sh = cl.sum_h + 2 * kEpsilon;
    L.n = lr == 0 ? lc : rc;
    L.parent_out = cl.output;
    L.c.min = cl.cmin;
    L.c.max = cl.cmax;
    if (vote_local) {
      // this rank's rows of the child: the histogrammed child's sums from k_round_split, the
      // other one's as the parent's minus those (loaded here only: the extra loads in the
      // common batch cost the narrow one-wave scans of wide data ~20%)
      const unsigned long long loc0 = rd->loc_acc[j][0], loc1 = rd->loc_acc[j][1];
      const double pl_g = a.rnode_lsum[2 * E.node], pl_h = a.rnode_lsum[2 * E.node + 1];
      const double hg = static_cast<double>(static_cast<long long>(loc0)) * ig;
      const double hh = static_cast<double>(static_cast<long long>(loc1)) * ih;
      L.sg = is_hist ? hg : pl_g - hg;
      L.sh = (is_hist ? hh : pl_h - hh) + 2 * kEpsilon;
      L.n = lr == 0 ? tl : pc - tl;
    }
    const int nh = 2 * a.p.total_bins;
    long long* dst = vote_global ? a.vote_hist + static_cast<size_t>(y * a.p.vote_k + blockIdx.x) * 2 * a.p.max_feature_bins
                                 : a.hist + static_cast<size_t>(slot) * nh + 2 * F.hist_offset;
    const long long* src = vote_global ? dst
                           : owner ? a.round_owned + 2 * (static_cast<size_t>(j) * a.rs_block + a.owned_off[f])
                                   : RoundScratch(a, parity, j) + 2 * F.hist_offset;
    const size_t pstride = static_cast<size_t>(units) * a.p.total_bins;
    const unsigned long long* part = a.partials + static_cast<size_t>(blk_off) * pstride + static_cast<size_t>(units) * F.hist_offset;
    const bool stage = a.p.max_feature_bins <= kFindLdsBins;
    double* sgv = s_bins;
    double* shv = s_bins + (stage ? a.p.max_feature_bins : 0);
    const bool subtract = !is_hist && !vote_global;
    const int nblk_direct = (!owner && !vote_global && nblk <= kDirectChunk) ? nblk : -1;
    const bool spread = nblk_direct > 1 && 2 * nbf <= NT;
    long long pg0 = 0, ph0 = 0;
    if (subtract && tid < nbf) {
      pg0 = dst[2 * tid];
      ph0 = dst[2 * tid + 1];
    }
    if (spread) {
      for (int i = tid; i < 2 * nbf; i += NT) sh.s_red[i] = 0ull;
      __syncthreads();
      const int per = NT / nbf;
      const int i = tid % nbf, r = tid / nbf;
      if (r < per) {
        constexpr int kC = 8;
        long long g = 0, h = 0;
        for (int k0 = r; k0 < nblk_direct; k0 += per * kC) {
          unsigned long long v0[kC], v1[kC];
#pragma unroll
          for (int cc = 0; cc < kC; ++cc) {
            const int k = k0 + cc * per;
            const unsigned long long* q = part + k * pstride + static_cast<size_t>(units) * i;
            v0[cc] = k < nblk_direct ? q[0] : 0ull;
            v1[cc] = (k < nblk_direct && units == 2) ? q[1] : 0ull;
          }
#pragma unroll
          for (int cc = 0; cc < kC; ++cc) {
            long long pgv, phv;
            UnpackPartial(v0[cc], v1[cc], units, &pgv, &phv);
            g += pgv;
            h += phv;
          }
        }
        atomicAdd(&sh.s_red[2 * i], static_cast<unsigned long long>(g));
        atomicAdd(&sh.s_red[2 * i + 1], static_cast<unsigned long long>(h));
      }
      __syncthreads();
    }
    for (int i = tid; i < nbf; i += NT) {
      long long g = 0, h = 0;
      if (spread) {
        g = static_cast<long long>(sh.s_red[2 * i]);
        h = static_cast<long long>(sh.s_red[2 * i + 1]);
      } else if (nblk_direct >= 0) {
        for (int k0 = 0; k0 < nblk_direct; k0 += kDirectChunk) {
          unsigned long long v0[kDirectChunk], v1[kDirectChunk];
#pragma unroll
          for (int k = 0; k < kDirectChunk; ++k) {
            const unsigned long long* q = part + (k0 + k) * pstride + static_cast<size_t>(units) * i;
            v0[k] = k0 + k < nblk_direct ? q[0] : 0ull;
            v1[k] = (k0 + k < nblk_direct && units == 2) ? q[1] : 0ull;
          }
#pragma unroll
          for (int k = 0; k < kDirectChunk; ++k) {
            long long pgv, phv;
            UnpackPartial(v0[k], v1[k], units, &pgv, &phv);
            g += pgv;
            h += phv;
          }
        }
      } else {
        g = src[2 * i];
        h = src[2 * i + 1];
      }
      if (subtract) {
        g = (i == tid ? pg0 : dst[2 * i]) - g;
        h = (i == tid ? ph0 : dst[2 * i + 1]) - h;
      }
      if (!vote_global) {
        dst[2 * i] = g;
        dst[2 * i + 1] = h;
      }
      if (stage) {
        sgv[i] = static_cast<double>(g) * ig;
        shv[i] = static_cast<double>(h) * ih;
      }
    }
    __syncthreads();
    if (ktw) kt[2] = wall_clock64();
    if (used) {
      L.cnt_factor = L.n / L.sh;
      const double gain_shift = LeafGain(L.sg, L.sh, p.lambda_l1, p.lambda_l2, p.max_delta_step, p.path_smooth, L.n,
                                         L.parent_out, p.use_l1, p.use_max_output, p.use_smoothing);
      L.min_gain_shift = gain_shift + p.min_gain_to_split;
      o.feature = f;
      o.real_feature = F.real_index;
      HistView hv;
      hv.lg = stage ? sgv : nullptr;
      hv.lh = stage ? shv : nullptr;
      hv.h = dst;
      hv.inv_g = ig;
      hv.inv_h = ih;
      bool splittable;
      if constexpr (!CAT) {
        if (a.round_xt) {  // (extra_trees: the prefixes the replay evaluates its drawn thresholds from)
          XtStorePrefix<NT>(F, hv, L, a.node_pre + static_cast<size_t>(frow) * a.p.total_bins + F.hist_offset, &sh.ssc);
        }
      }
      if constexpr (CAT) {
        splittable = FindCategoricalBlock(F, hv, L, p, &o, a.feat_cat + RoundFbIndex(a, y, f) * kMaxCatWords,
                                          &sh.sc, &sh.cat_sc);
      } else {
        splittable = FindNumericalBlock<SIMPLE, NT>(F, hv, L, p, cl.depth, a.p.monotone_penalty, &o, &sh.sc, &sh.ssc,
                                                    sh.sc2, kNoRandThr);
      }
      if (tid == 0 && !vote_global) {  // (voting: the local scan's flags; categorical: thread 0 decides)
        flags[f] = splittable ? 1 : 0;
        o.flag = splittable ? 1 : 0;
      }
      // CEGB (GPUTreeLearner::CegbRounds: no refunds in a round tree), before the monotone
      // penalty as SerialTreeLearner::ComputeBestSplitForFeature
      if (a.p.cegb && !a.round_cegb) {  // (KArgs::round_cegb: the replay subtracts them)
        double delta = a.p.cegb_split * L.n;
        if (a.cegb_coupled != nullptr && !a.cegb_used[f]) delta += a.cegb_coupled[f];
        o.gain -= delta;
      }
      if (!CAT && !SIMPLE && F.monotone != 0) o.gain *= MonotonePenalty(cl.depth, a.p.monotone_penalty);
      if (o.gain == -INFINITY) o.feature = -1;
    }
  }
  if (ktw) kt[3] = wall_clock64();
  if (write && tid == 0) {
    PublishRecord(fb_out, o);
    if (a.node_fb != nullptr) PublishRecord(&a.node_fb[static_cast<size_t>(frow) * NF + f], o);
  }
  if constexpr (CAT) {
    // (per-node sampling: the category set kept per node, from this scan's slot)
    if (write && a.node_fb_cat != nullptr && a.node_cat_slot[f] >= 0) {
      __syncthreads();
      if (tid == 0 && o.ncat > 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        PublishCatCopy(a.node_fb_cat + (static_cast<size_t>(frow) * a.node_cat_slots + a.node_cat_slot[f]) * kMaxCatWords,
                       a.feat_cat + RoundFbIndex(a, y, f) * kMaxCatWords);
      }
    }
  }
  // (distributed: the results are gathered from every rank first, k_round_childbest folds them)
  if (KIND == 1 || a.round_dist) return;  // (the categorical kernel counts the arrivals)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  ArrivalRelease();
  __syncthreads();
  // arrival: the child's last workgroup folds the child's per-feature results
  if (tid == 0) {
    if (ktw) kt[4] = wall_clock64();
    const unsigned nwg = gridDim.x;
    uint32_t* cc = a.child_cnt + static_cast<size_t>(y) * (kFindSub + 1) * kFindSubStride;
    int last = 0;
    if (nwg <= kRoundFlatMax) {
      if (atomicAdd(cc, 1u) == nwg - 1) {
        last = 1;
        *cc = 0u;  // (every other workgroup of the child has counted)
      }
    } else {
      const unsigned g = blockIdx.x % kFindSub;
      const unsigned members = (nwg - g + kFindSub - 1) / kFindSub;
      uint32_t* sub = cc + g * kFindSubStride;
      if (atomicAdd(sub, 1u) == members - 1) {
        *sub = 0u;
        uint32_t* top = cc + kFindSub * kFindSubStride;
        if (atomicAdd(top, 1u) == kFindSub - 1) {
          last = 1;
          *top = 0u;
        }
      }
    }
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  ChildBest<KIND, NT>(a, y, frow, sh);
  if (ktw) kt[5] = wall_clock64();
  // (PIF: an instantiation without the plan when the plan has its own kernel -- the replay's
  // registers otherwise set the occupancy of every scan workgroup)
  if (!PIF || !a.plan_in_find) return;
  // the last child of the round to finish plans the next round (its scans' results were
  // published write-through; one agent-scope acquire)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  ArrivalRelease();
  __syncthreads();
  if (tid == 0) {
    const unsigned n = 2u * static_cast<unsigned>(nexp);
    int last = 0;
    if (atomicAdd(&rd->child_done, 1u) == n - 1) {
      last = 1;
      rd->child_done = 0u;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  if (ktw) {
    for (int k = 0; k < 6; ++k) a.ktrace[static_cast<size_t>(rround) * kTraceSlots + 26 + k] = kt[k];
#if LGBM_FIND_PHASES
    for (int k = 0; k < 4; ++k) a.ktrace[static_cast<size_t>(rround) * kTraceSlots + 12 + k] = g_find_phase[k];
#endif
  }
  if constexpr (PIF) RoundPlanBody<false, NT>(a, reinterpret_cast<unsigned char*>(s_bins));
}

// ----------------------------------------------------------------------------- k_round_plan
// ordered keys of the replay's argmax (SplitInfo order over leaves): larger gain first (NaN =
// -inf), then smaller real feature, then lower leaf id -- two wave max-reductions over DPP
// lane moves instead of a shuffle butterfly carrying five values
__device__ __forceinline__ uint32_t TieKey(int rf, int leaf) {
  const uint32_t r = rf < 0 ? 0x3fffffu : min(static_cast<uint32_t>(rf), 0x3ffffeu);
  return ~((r << 10) | static_cast<uint32_t>(leaf));
}
// the argmax leaf among l <= s with take(l) (one wave; -1: none)
template <typename Take>
__device__ __forceinline__ int WaveArgmaxLeaf(const double* tg, const int* trf, int s, Take take) {
  const int lane = threadIdx.x & 63;
  unsigned long long gk = 0;
  uint32_t tk = 0;
  for (int l = lane; l <= s; l += kWave) {
    if (!take(l)) continue;
    const unsigned long long k = GainKey(tg[l]);
    const uint32_t t = TieKey(trf[l], l);
    if (k > gk || (k == gk && t > tk)) {
      gk = k;
      tk = t;
    }
  }
  const unsigned long long gm = WaveMaxDpp(gk);
  if (gm == 0) return -1;
  const uint32_t tm = WaveMaxDpp(gk == gm ? tk : 0u);
  return static_cast<int>((~tm) & 1023u);
}
__device__ __forceinline__ void WaveLdsSync() {  // lane 0's LDS stores before the wave's next loads
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#ifndef LGBM_REPLAY_KEY32
#define LGBM_REPLAY_KEY32 1
#endif
#ifndef LGBM_REPLAY_PREFETCH
#define LGBM_REPLAY_PREFETCH 0  // (A/B: children loaded ahead -- 2.356 vs 2.343 ms/iter, not kept)
#endif
// Replay + prediction with one leaf per lane in registers (num_leaves <= 64, wave 0): a step
// is one 64-bit DPP max over the gain keys (the tie key's max only when gains tie exactly),
// reads of the winner's lane, and LDS reads of the node tables by the two lanes whose leaf
// changes -- no LDS round trip through every lane per step.  Same order and picks as the LDS
// tables' loop below.
struct RegLeaf {
  double g;
  int rf, node, ch;
  uint32_t k32;  // GainKey32(g): the argmax's first, 32-bit pass
#if LGBM_REPLAY_PREFETCH
  // the node's children (ch >= 0), loaded ahead: gain, real feature, first child of each
  double g0, g1;
  int rf0, rf1, ch0, ch1;
#endif
};
// order-preserving 32-bit key of a gain (NaN = -inf): the gain rounded to float, whose
// rounding is monotone -- a larger float key means a larger gain; equal float keys are
// resolved by the exact 64-bit keys
__device__ __forceinline__ uint32_t GainKey32(double g) {
  if (g != g) g = -INFINITY;
  const uint32_t b = __float_as_uint(static_cast<float>(g));
  return (b >> 31) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ int RegArgmax(const RegLeaf& x, bool live) {
  const int lane = threadIdx.x & 63;
  // one 32-bit DPP max; the exact 64-bit / tie passes only when the float keys tie
#if LGBM_REPLAY_KEY32
  const uint32_t k = live ? x.k32 : 0u;
#else
  const uint32_t k = live ? 1u : 0u;  // (A/B: every live lane into the 64-bit pass)
#endif
  const uint32_t km = WaveMaxDpp(k);
  const unsigned long long t32 = __ballot(live && k == km);
  if (__popcll(t32) == 1) return __builtin_amdgcn_readfirstlane(static_cast<int>(__builtin_ctzll(t32)));
  const bool in = live && k == km;
  const unsigned long long gk = in ? GainKey(x.g) : 0ull;
  const unsigned long long gm = WaveMaxDpp(gk);
  const unsigned long long tied = __ballot(in && gk == gm);
  if (__popcll(tied) == 1) return __builtin_amdgcn_readfirstlane(static_cast<int>(__builtin_ctzll(tied)));
  const uint32_t tm = WaveMaxDpp((in && gk == gm) ? TieKey(x.rf, lane) : 0u);
  return static_cast<int>((~tm) & 1023u);
}
#if LGBM_REPLAY_PREFETCH
// the children of the lane's node, loaded now and used only when the lane next wins: the
// winner's children come from its registers (readlane) instead of an LDS round trip that the
// next argmax would wait for
__device__ __forceinline__ void RegPrefetch(RegLeaf* x, const double* ng, const int* nrf, const int* nch) {
  const int c = x->ch;
  x->g0 = c >= 0 ? ng[c] : -INFINITY;
  x->rf0 = c >= 0 ? nrf[c] : -1;
  x->ch0 = c >= 0 ? nch[c] : -1;
  x->g1 = c >= 0 ? ng[c + 1] : -INFINITY;
  x->rf1 = c >= 0 ? nrf[c + 1] : -1;
  x->ch1 = c >= 0 ? nch[c + 1] : -1;
}
__device__ __forceinline__ void RegSet(RegLeaf* x, int node, double g, int rf, int ch, const double* ng, const int* nrf,
                                       const int* nch) {
  x->node = node;
  x->g = g;
  x->k32 = GainKey32(g);
  x->rf = rf;
  x->ch = ch;
  RegPrefetch(x, ng, nrf, nch);
}
#endif
__device__ __forceinline__ void RegLoad(RegLeaf* x, int node, const double* ng, const int* nrf, const int* nch) {
  x->node = node;
  x->g = node >= 0 ? ng[node] : -INFINITY;
  x->k32 = GainKey32(x->g);
  x->rf = node >= 0 ? nrf[node] : -1;
  x->ch = node >= 0 ? nch[node] : -1;
#if LGBM_REPLAY_PREFETCH
  RegPrefetch(x, ng, nrf, nch);
#endif
}
// lanes w and nl take the children of lane w's node (c, c + 1)
__device__ __forceinline__ void RegTakeChildren(RegLeaf* x, int lane, int w, int nl, int c, const double* ng,
                                                const int* nrf, const int* nch) {
#if LGBM_REPLAY_PREFETCH
  const double g0 = ReadLane(x->g0, w), g1 = ReadLane(x->g1, w);
  const int rf0 = ReadLane(x->rf0, w), rf1 = ReadLane(x->rf1, w);
  const int ch0 = ReadLane(x->ch0, w), ch1 = ReadLane(x->ch1, w);
  if (lane == w) RegSet(x, c, g0, rf0, ch0, ng, nrf, nch);
  if (lane == nl) RegSet(x, c + 1, g1, rf1, ch1, ng, nrf, nch);
#else
  if (lane == w) RegLoad(x, c, ng, nrf, nch);
  if (lane == nl) RegLoad(x, c + 1, ng, nrf, nch);
#endif
}
// extra_trees on round growth (KArgs::round_xt), one lane: feature f's split of node `node` at
// the drawn threshold rthr, from the node's prefix table -- FindNumericalBlock's candidates at
// that threshold (the reverse one at bin rthr + 1 - offset, the forward one at rthr - offset,
// the forward start for a NaN bin without bin 0), the same sums (exact) and selection, then the
// scan's feature and depth penalties.  Returns the splittable flag.
__device__ bool XtEvalNum(const KArgs& a, const Feature& F, int f, int node, const ChildStats& cs, int n, int rthr,
                          FeatureBest* out) {
  const SplitParams& p = a.p.sp;
  const bool simple = !p.use_l1 && !p.use_max_output && !p.use_smoothing && !p.use_mc;
  const XtPre* pre = a.node_pre + static_cast<size_t>(node) * a.p.total_bins + F.hist_offset;
  const int nb = F.num_bin - F.offset, offset = F.offset;
  const bool two = F.num_bin > 2 && F.missing_type != 0;
  const bool skip_def = two && F.missing_type == 1;
  const bool na = two && F.missing_type == 2;
  const int def_t = skip_def ? F.default_bin - offset : -1;
  LeafCtx L;
  L.sg = cs.sum_g;
  L.sh = cs.sum_h + 2 * kEpsilon;
  L.n = n;
  L.parent_out = cs.output;
  L.c.min = cs.cmin;
  L.c.max = cs.cmax;
  L.cnt_factor = L.n / L.sh;
  L.min_gain_shift = LeafGain(L.sg, L.sh, p.lambda_l1, p.lambda_l2, p.max_delta_step, p.path_smooth, L.n, L.parent_out,
                              p.use_l1, p.use_max_output, p.use_smoothing) +
                     p.min_gain_to_split;
  // the entries (one batch of loads): the last (every stored bin), the one before it (the NaN
  // bin), the default bin and the one before it (the default bin's own sums, taken out of every
  // prefix past it as the scan leaves it out), the reverse candidate's exclusive prefix and the
  // forward candidate's inclusive one.  P[t]: stored bins <= t, the rebuilt one left out
  const int fix_t = F.mfb > 0 ? F.mfb : -1;
  const int t_r = rthr + 1 - offset, t_f = rthr - offset;
  // (unconditional loads at clamped indices, the unused ones zeroed after: one round trip)
  const XtPre zero = {0.0, 0.0, 0, 0};
  auto at = [&](int t) { return pre[min(max(t, 0), nb - 1)]; };
  const XtPre T = pre[nb - 1];
  XtPre T2 = at(nb - 2), D = at(def_t), D2 = at(def_t - 1), R = at(t_r - 1), W = at(t_f);
  if (nb < 2) T2 = zero;
  if (def_t < 0) D = zero;
  if (def_t < 1) D2 = zero;
  if (!(t_r >= 1 && t_r - 1 < nb)) R = zero;
  if (!(t_f >= 0 && t_f < nb)) W = zero;
  const double dg = D.g - D2.g, dh = D.h - D2.h;  // (exact: grid values)
  const int dc = D.c - D2.c;
  // prefix without the default bin (exact) of the bins <= t
  auto wo_def = [&](const XtPre& e, int t, double* g, double* h, int* c) {
    const bool sub = def_t >= 0 && def_t <= t;
    *g = sub ? e.g - dg : e.g;
    *h = sub ? e.h - dh : e.h;
    *c = sub ? e.c - dc : e.c;
  };
  // FixHistogram: the most frequent bin from the leaf totals (every stored bin: T), added last
  const bool fix_in = fix_t >= 0 && fix_t != def_t;
  double fix_g = 0.0, fix_h = 0.0;
  int fix_c = 0;
  if (fix_t >= 0) {
    fix_g = L.sg - T.g;
    fix_h = (L.sh - 2 * kEpsilon) - T.h;
    fix_c = RoundIntD(fix_h * L.cnt_factor);
  }
  double tot_g, tot_h;
  int tot_c;
  wo_def(T, nb - 1, &tot_g, &tot_h, &tot_c);
  if (fix_in) {
    tot_g += fix_g;
    tot_h += fix_h;
    tot_c += fix_c;
  }
  // (na: no default bin; the NaN bin is the last one -- rebuilt, or the last entry's step)
  const bool nan_fix = fix_t == nb - 1;
  const double ng = !na ? 0.0 : nan_fix ? fix_g : T.g - T2.g;
  const double nh = !na ? 0.0 : nan_fix ? fix_h : T.h - T2.h;
  const int nc = !na ? 0 : nan_fix ? fix_c : T.c - T2.c;
  const int t_start_r = nb - 1 - (na ? 1 : 0), t_end_r = 1 - offset, t_end_f = nb - 2;
  const double pr_g = na ? tot_g - ng : tot_g, pr_h = na ? tot_h - nh : tot_h;
  const int pr_c = na ? tot_c - nc : tot_c;
  const bool minus_one = na && offset == 1;
  const double lg0 = minus_one ? L.sg - T.g : 0.0;
  const double lh0 = minus_one ? L.sh - kEpsilon - T.h : kEpsilon;
  const int lc0 = minus_one ? L.n - tot_c : 0;
  const double min_h = p.min_sum_hessian_in_leaf;
  const int min_n = p.min_data_in_leaf;
  const int8_t mono = static_cast<int8_t>(F.monotone);
  double rb_gain = -INFINITY, fb_gain = -INFINITY, rb_lg = 0.0, rb_lh = 0.0, fb_lg = 0.0, fb_lh = 0.0;
  int rb_thr = -1, fb_thr = 0x7fffffff, rb_lc = 0, fb_lc = 0;
  bool any = false;
  for (int c = 0; c < 3; ++c) {  // 0: the forward start, 1: reverse, 2: forward
    bool ok;
    double xg, xh;
    int xc, thr;
    if (c == 0) {
      ok = minus_one && rthr == offset - 1;
      xg = lg0;
      xh = lh0;
      xc = lc0;
      thr = offset - 1;
    } else if (c == 1) {
      ok = t_r != def_t && t_r >= t_end_r && t_r <= t_start_r;
      double pg, ph;
      int pc;
      wo_def(R, t_r - 1, &pg, &ph, &pc);
      const bool fx = fix_in && fix_t < t_r;
      const double eg = fx ? pg + fix_g : pg, eh = fx ? ph + fix_h : ph;
      const int ec = fx ? pc + fix_c : pc;
      xg = L.sg - (pr_g - eg);
      xh = L.sh - (pr_h - eh + kEpsilon);
      xc = L.n - (pr_c - ec);
      thr = t_r - 1 + offset;
    } else {
      ok = two && t_f >= 0 && t_f != def_t && t_f <= t_end_f;
      double pg, ph;
      int pc;
      wo_def(W, t_f, &pg, &ph, &pc);
      const bool fx = fix_in && fix_t <= t_f;
      xg = lg0 + (fx ? pg + fix_g : pg);
      xh = lh0 + (fx ? ph + fix_h : ph);
      xc = lc0 + (fx ? pc + fix_c : pc);
      thr = t_f + offset;
    }
    if (!ok || xc < min_n || xh < min_h) continue;
    const int rc = L.n - xc;
    const double rh = L.sh - xh;
    if (rc < min_n || rh < min_h) continue;
    const double gain = simple ? GainOf<true>(xg, xh, L.sg - xg, rh, p.lambda_l2, p, L.c, mono, xc, rc, L.parent_out)
                               : GainOf<false>(xg, xh, L.sg - xg, rh, p.lambda_l2, p, L.c, mono, xc, rc, L.parent_out);
    if (!(gain > L.min_gain_shift)) continue;
    any = true;
    if (c == 1) {
      rb_gain = gain;
      rb_thr = thr;
      rb_lg = xg;
      rb_lh = xh;
      rb_lc = xc;
    } else {
      fb_gain = gain;
      fb_thr = thr;
      fb_lg = xg;
      fb_lh = xh;
      fb_lc = xc;
    }
  }
  FeatureBest o;
  o.gain = -INFINITY;
  o.feature = f;
  o.real_feature = F.real_index;
  o.thr = 0;
  o.default_left = two ? 1 : (F.missing_type == 2 ? 0 : 1);
  o.lc = o.rc = 0;
  o.mono = F.monotone;
  o.ncat = 0;
  o.flag = -1;
  o.pad = 0;
  o.lg = o.lh = o.rg = o.rh = o.lo = o.ro = 0.0;
  for (int d = 0; d < (two ? 2 : 1); ++d) {
    const double bg = d == 0 ? rb_gain : fb_gain;
    if (any && bg > o.gain + L.min_gain_shift) {
      const double blg = d == 0 ? rb_lg : fb_lg, blh = d == 0 ? rb_lh : fb_lh;
      const int blc = d == 0 ? rb_lc : fb_lc;
      o.thr = d == 0 ? rb_thr : fb_thr;
      o.lo = simple ? OutputOf<true>(blg, blh, p.lambda_l2, p, L.c, blc, L.parent_out)
                    : OutputOf<false>(blg, blh, p.lambda_l2, p, L.c, blc, L.parent_out);
      o.lc = blc;
      o.lg = blg;
      o.lh = blh - kEpsilon;
      o.ro = simple ? OutputOf<true>(L.sg - blg, L.sh - blh, p.lambda_l2, p, L.c, L.n - blc, L.parent_out)
                    : OutputOf<false>(L.sg - blg, L.sh - blh, p.lambda_l2, p, L.c, L.n - blc, L.parent_out);
      o.rc = L.n - blc;
      o.rg = L.sg - blg;
      o.rh = L.sh - blh - kEpsilon;
      o.gain = bg - L.min_gain_shift;
      o.default_left = d == 1 ? 0 : (!two && F.missing_type == 2 ? 0 : 1);
    }
  }
  o.gain *= F.penalty;
  if (!simple && F.monotone != 0) o.gain *= MonotonePenalty(cs.depth, a.p.monotone_penalty);
  if (o.gain == -INFINITY) o.feature = -1;
  *out = o;
  return any;
}

// (extra_trees: draw k of a feature's generator, k >= 1, as the step scans draw)
__device__ __forceinline__ int XtThreshold(const KArgs& a, const Feature& F, int f, int k) {
  const uint32_t x = LcgSkip(a.xt_base[f], k);
  return static_cast<int>(x & 0x7fffffffu) % (F.num_bin - 2);
}

// Deferred fold (per-node sampling, KArgs::round_bynode; extra_trees, KArgs::round_xt), wave 0,
// when the replay accepts split s of leaf w (node n, children c = left and c + 1 = right; the
// left keeps leaf id w, the right is leaf s + 1).  SerialTreeLearner::BeforeFindBestSplit /
// FindBestSplits / FindBestSplitsFromHistograms in the sequential order: unless the children
// are not scanned (depth, min_data, the tree's last split), the smaller child (fewer rows; a
// tie: the right one) is evaluated first -- per-node sampling: it takes draw d, the larger
// d + 1; extra_trees: per feature, its threshold draw comes first.  The parent's flag row moves
// to the larger child's leaf id (the smaller one keeps the stale row of its id), a feature the
// parent could not split is 0 for the smaller child and skipped, and a feature a child
// evaluates takes the child's flag and competes for its best split (per-node sampling: the
// scan's result, KArgs::node_fb; extra_trees: the drawn threshold's, XtEvalNum).  The
// children's bests go to cbest and the node tables.  xcnt: extra_trees draw counts per feature
// (LDS, at most kXtLaneFeatures * 64 features).
// (XT: compiled in only where the extra_trees replay runs -- k_round_plan; the replay's
// registers would otherwise set the occupancy of every scan workgroup of k_round_find)
constexpr int kXtLaneFeatures = 4;
template <bool XT>
__device__ bool DeferAccept(const KArgs& a, int s, int w, int n, int c, int* draw, double* ng, int* nrf, int* nfi,
                            int* xcnt, int my_node, const int* tnode) {
  const int lane = threadIdx.x & 63;
  const int L = a.p.num_leaves, NF = a.p.num_features, md = a.p.sp.min_data_in_leaf;
  // CEGB coupled penalties (KArgs::round_cegb): the split's feature, if the model had not used
  // it, refunds its coupled penalty to the other leaves' remembered candidates first
  // (CostEfficientGradientBoosting::UpdateLeafBestSplits, at SplitInner's start).  A refunded
  // leaf is never an expanded one: the plan expands only leaves no refund can change (below).
  // Leaf l's node: this lane's my_node (register replay, leaf = lane) or tnode[l].
  bool refunded = false;
  if (a.round_cegb && a.cegb_coupled != nullptr) {
    const int fsplit = nfi[n];
    if (fsplit >= 0 && !a.cegb_used[fsplit]) {
      refunded = true;
      const double refund = a.cegb_coupled[fsplit];
      for (int l = lane; l <= s; l += kWave) {
        if (l == w) continue;
        const int nd = tnode != nullptr ? tnode[l] : my_node;
        FeatureBest cand = a.cegb_mem[static_cast<size_t>(l) * NF + fsplit];
        cand.gain += refund;
        const double cg = ng[nd];
        const int crf = nrf[nd] < 0 ? 0x7fffffff : nrf[nd];
        const int nrf_c = cand.feature < 0 ? 0x7fffffff : cand.real_feature;
        if (cg > -INFINITY && (cand.gain > cg || (cand.gain == cg && nrf_c < crf))) {
          a.cbest[nd] = cand;
          ng[nd] = cand.gain;
          nrf[nd] = cand.real_feature;
          nfi[nd] = cand.feature;
        }
      }
      if (lane == 0) a.cegb_used[fsplit] = 1;
      __threadfence_block();  // (the children's folds below and later splits read the flag)
      WaveLdsSync();
    }
  }
  const RNode& P = a.rnode[n];
  // (data-parallel: the children's global counts -- the split's estimates -- as the reference's
  // GetGlobalDataCountInLeaf; this rank's rows otherwise)
  const bool dpc = a.p.data_parallel != 0;
  const int nl = dpc ? a.rnode[c].st.global_count : P.total_left;
  const int nr = dpc ? a.rnode[c + 1].st.global_count : P.count - P.total_left;
  const int depth = a.rnode[c].st.depth;
  const bool scanned = s + 1 < L - 1 && !(a.p.max_depth > 0 && depth >= a.p.max_depth) && !(nl < 2 * md && nr < 2 * md);
  if (!scanned) {
    if (lane < 2) {
      FeatureBest none = {};
      none.gain = -INFINITY;
      none.feature = none.real_feature = -1;
      a.cbest[c + lane] = none;
      ng[c + lane] = -INFINITY;
      nrf[c + lane] = -1;
      nfi[c + lane] = -1;
    }
    WaveLdsSync();
    return refunded;
  }
  const bool bn = a.round_bynode != 0, xt = XT && a.round_xt != 0;
  int d0 = 0;
  if (bn) {
    d0 = *draw;
    *draw = d0 + 2;
  }
  const bool small_left = nl < nr;
  const int small_leaf = small_left ? w : s + 1, large_leaf = small_left ? s + 1 : w;
  const int small_node = small_left ? c : c + 1, large_node = small_left ? c + 1 : c;
  int8_t* rw = a.leaf_rows + static_cast<size_t>(w) * NF;
  int8_t* rn = a.leaf_rows + static_cast<size_t>(s + 1) * NF;
  int8_t* rs = a.leaf_rows + static_cast<size_t>(small_leaf) * NF;
  int8_t* rl = a.leaf_rows + static_cast<size_t>(large_leaf) * NF;
  const int8_t* ms = bn ? a.node_mask + static_cast<size_t>(d0) * NF : nullptr;
  const int8_t* ml = bn ? ms + NF : nullptr;
  const int8_t* fs = a.splittable + static_cast<size_t>(small_node) * NF;
  const int8_t* fl = a.splittable + static_cast<size_t>(large_node) * NF;
  const bool cg = a.round_cegb != 0;
  const FeatureBest* bs = (bn || cg) ? a.node_fb + static_cast<size_t>(small_node) * NF : nullptr;
  const FeatureBest* bl = (bn || cg) ? a.node_fb + static_cast<size_t>(large_node) * NF : nullptr;
  const int ns = small_left ? nl : nr, nlg = small_left ? nr : nl;
  ChildStats css, csl;
  if (xt) {
    css = a.rnode[small_node].st;
    csl = a.rnode[large_node].st;
  }
  // (CEGB: the scans published the raw candidates -- remembered per leaf id for later refunds
  // -- and the penalties of the model's used set now are subtracted here)
  auto cegb_take = [&](FeatureBest* o, int leaf, int f, int rows) {
    a.cegb_mem[static_cast<size_t>(leaf) * NF + f] = *o;
    double delta = a.p.cegb_split * rows;
    if (a.cegb_coupled != nullptr && !a.cegb_used[f]) delta += a.cegb_coupled[f];
    o->gain -= delta;
  };
  ArgC cs = ArgNone(), cl = ArgNone();
  FeatureBest rec_s, rec_l;  // (extra_trees: this lane's best records of the two children)
  // (the flag rows are read before any is written: the children's rows are the parent's and the
  // new leaf's)
  if constexpr (XT) {
    if (xt) {
      // extra_trees, one child's evaluation live at a time: pass 0 the smaller child (its flags
      // kept in LDS), pass 1 the larger one and the rows
      __shared__ int8_t s_gs[kXtLaneFeatures * kWave];
      for (int pass = 0; pass < 2; ++pass) {
        const bool small = pass == 0;
        for (int f = lane; f < NF; f += kWave) {
          const int8_t parent = rw[f], stale = rn[f];
          const bool live = a.tree_mask[f] && parent;
          const bool es = !bn || ms[f], el = !bn || ml[f];
          const Feature F = a.feat[f];
          const bool drawn = F.num_bin - 2 > 0;
          const int cnt = xcnt[f];  // (the smaller child draws first)
          int8_t g = -1;
          if (live && (small ? es : el)) {
            const int k = cnt + 1 + (!small && es && drawn ? 1 : 0);
            const int thr = drawn ? XtThreshold(a, F, f, k) : 0;
            FeatureBest o;
            g = XtEvalNum(a, F, f, small ? small_node : large_node, small ? css : csl, small ? ns : nlg, thr, &o) ? 1 : 0;
            ArgC& cc = small ? cs : cl;
            if (o.feature >= 0 && (cc.idx < 0 || SplitBetter(o.gain, o.real_feature, cc.g, cc.rf))) {
              cc.g = o.gain;
              cc.rf = o.real_feature;
              cc.idx = f;
              if (small) rec_s = o;
              else rec_l = o;
            }
          }
          if (small) {
            s_gs[f] = g;
            continue;
          }
          int8_t vs = stale, vl = parent;
          if (a.tree_mask[f]) {
            if (!parent) {
              vs = 0;
            } else {
              if (s_gs[f] >= 0) vs = s_gs[f];
              if (g >= 0) vl = g;
            }
          }
          if (live) xcnt[f] = cnt + ((es && drawn) ? 1 : 0) + ((el && drawn) ? 1 : 0);
          rs[f] = vs;
          rl[f] = vl;
        }
        WaveLdsSync();
      }
    }
  }
  if (!xt) {
    for (int f = lane; f < NF; f += kWave) {
      const int8_t parent = rw[f], stale = rn[f];
      int8_t vs = stale, vl = parent;  // (the rows after the move: the larger child holds the parent's)
      if (a.tree_mask[f]) {
        if (!parent) {
          vs = 0;
        } else {
          // (the fold reads three fields of a record; CEGB copies it into the leaf's memory)
          if (!bn || ms[f]) {
            vs = fs[f];
            const FeatureBest& r = bs[f];
            double og = r.gain;
            const int orf = r.real_feature, ofe = r.feature;
            if (cg) {
              FeatureBest o = r;
              cegb_take(&o, small_leaf, f, ns);
              og = o.gain;
            }
            if (ofe >= 0 && (cs.idx < 0 || SplitBetter(og, orf, cs.g, cs.rf))) {
              cs.g = og;
              cs.rf = orf;
              cs.idx = f;
            }
          }
          if (!bn || ml[f]) {
            vl = fl[f];
            const FeatureBest& r = bl[f];
            double og = r.gain;
            const int orf = r.real_feature, ofe = r.feature;
            if (cg) {
              FeatureBest o = r;
              cegb_take(&o, large_leaf, f, nlg);
              og = o.gain;
            }
            if (ofe >= 0 && (cl.idx < 0 || SplitBetter(og, orf, cl.g, cl.rf))) {
              cl.g = og;
              cl.rf = orf;
              cl.idx = f;
            }
          }
        }
      }
      rs[f] = vs;
      rl[f] = vl;
    }
  }
  const ArgC bcs = ArgWaveBest(cs), bcl = ArgWaveBest(cl);
  FeatureBest none = {};
  none.gain = -INFINITY;
  none.feature = none.real_feature = -1;
  if (xt) {
    // the lane holding a child's winner hands its record over through LDS; lanes 0 / 1 store
    // the children's bests (a uniform-address store from a lane picked at run time lost its
    // value to the other lanes' masked copies)
    __shared__ FeatureBest s_rec[2];
    if (bcs.idx >= 0 && (bcs.idx & (kWave - 1)) == lane) s_rec[0] = rec_s;
    if (bcl.idx >= 0 && (bcl.idx & (kWave - 1)) == lane) s_rec[1] = rec_l;
    WaveLdsSync();
    if (lane < 2) {
      const ArgC& b = lane == 0 ? bcs : bcl;
      const int node = lane == 0 ? small_node : large_node;
      const bool ok = b.idx >= 0 && b.g != -INFINITY;
      a.cbest[node] = ok ? s_rec[lane] : none;
      ng[node] = ok ? b.g : -INFINITY;
      nrf[node] = ok ? b.rf : -1;
      nfi[node] = ok ? b.idx : -1;
    }
  } else if (lane < 2) {
    const ArgC& b = lane == 0 ? bcs : bcl;
    const int node = lane == 0 ? small_node : large_node;
    FeatureBest o = none;
    if (b.idx >= 0 && b.g != -INFINITY) {
      o = (lane == 0 ? bs : bl)[b.idx];
      if (cg) o.gain = b.g;  // (the penalised gain)
    }
    a.cbest[node] = o;
    ng[node] = o.feature >= 0 ? o.gain : -INFINITY;
    nrf[node] = o.real_feature;
    nfi[node] = o.feature;
  }
  if (!xt && a.node_fb_cat != nullptr) {
    // a categorical winner's category set, from the node's copy (the whole wave)
    for (int side = 0; side < 2; ++side) {
      const ArgC& b = side == 0 ? bcs : bcl;
      if (b.idx < 0 || b.g == -INFINITY || a.node_cat_slot[b.idx] < 0) continue;
      const int node = side == 0 ? small_node : large_node;
      const uint32_t* src = a.node_fb_cat + (static_cast<size_t>(node) * a.node_cat_slots + a.node_cat_slot[b.idx]) * kMaxCatWords;
      uint32_t* dst = a.cbest_cat + static_cast<size_t>(node) * kMaxCatWords;
      for (int i = lane; i < kMaxCatWords; i += kWave) dst[i] = src[i];
    }
  }
  WaveLdsSync();
  return refunded;
}

// The replay (wave 0): returns s, the splits after it, and *done; acc / accn / tnode as the LDS
// path.  x keeps the replayed leaves for the prediction.
template <bool XT>
__device__ int ReplayRegs(const KArgs& a, int L, int s0, double* ng, int* nrf, const int* nch, int* nfi, int* tnode,
                          int* acc, int* accn, RegLeaf* xp, int* done_out, int* draw, int* xcnt, int* blocker) {
  const int lane = threadIdx.x & 63;
  RegLeaf& x = *xp;
  RegLoad(&x, lane <= s0 ? tnode[lane] : -1, ng, nrf, nch);
  int s = s0, done = 0;
  *blocker = -1;
  for (;;) {
    if (s >= L - 1) {
      done = 1;
      break;
    }
    const int w = RegArgmax(x, lane <= s);
    if (!(ReadLane(x.g, w) > 0.0)) {
      done = 1;
      break;
    }
    const int c = ReadLane(x.ch, w);
    if (c < 0) {
      *blocker = ReadLane(x.node, w);
      break;
    }
    const int nl = s + 1;
    if (lane == 0) {
      acc[s - s0] = w;
      accn[s - s0] = ReadLane(x.node, w);
    }
    bool refunded = false;
    if (a.round_bynode || a.round_cegb || (XT && a.round_xt)) {
      refunded = DeferAccept<XT>(a, s, w, ReadLane(x.node, w), c, draw, ng, nrf, nfi, xcnt, x.node, nullptr);
    }
    RegTakeChildren(&x, lane, w, nl, c, ng, nrf, nch);
    if (refunded) RegLoad(&x, lane <= nl ? x.node : -1, ng, nrf, nch);  // (refunded leaves' new bests)
    ++s;
  }
  if (lane <= s) tnode[lane] = x.node;
  *done_out = done;
  return s;
}

// the next round's expansions predicted past the blocker (wave 0, after ReplayRegs): returns
// the picks' count (s_pick); *done when the tree cannot go on
__device__ int PredictRegs(const KArgs& a, int L, int s, int used, int kround, const double* ng, const int* nrf,
                           const int* nch, int* s_pick, RegLeaf* xp, int* done_io) {
  const int lane = threadIdx.x & 63;
  RegLeaf& x = *xp;
  int done = *done_io, n = 0;
  if (!done) {
    const int need = L - 1 - s;
    int kmax = min(kround, a.round_need_div > 0 ? max(1, need / a.round_need_div) : need);
    kmax = min(kmax, a.round_emax - used - (need - 1));
    kmax = max(kmax, min(1, a.round_emax - used));
    if (kmax <= 0) done = 1;
    const int vmax = (a.round_bynode || a.round_xt || a.round_cegb) ? 0 : a.round_vmax;  // (deferred folds: the current leaves only)
    int vd = 0;
    for (int ss = s; !done && n < kmax && ss < L - 1; ++ss) {
      const int w = RegArgmax(x, lane <= ss);
      if (!(ReadLane(x.g, w) > 0.0)) break;
      const int c = ReadLane(x.ch, w), v = ReadLane(vd, w);
      const int nl = ss + 1;
      if (c >= 0) {
        RegTakeChildren(&x, lane, w, nl, c, ng, nrf, nch);
        if (lane == w || lane == nl) vd = v + 1;
      } else {
        if (v <= vmax) {
          if (lane == 0) s_pick[n] = ReadLane(x.node, w);
          ++n;
        }
        if (lane == w || lane == nl) RegLoad(&x, -1, ng, nrf, nch);
      }
    }
    if (n == 0) done = 1;
  }
  *done_io = done;
  return n;
}

// The next round's picks from order keys instead of the step walk (KArgs::round_predict; wave
// 0 after the replay, any num_leaves; the blocker is the first pick).  Best-first order pops a
// node only after its ancestors below the current leaf, so the known nodes come out by
// decreasing bottleneck m(v) -- the least gain on the path from the leaf to v: the frontier
// falls below m(v) only after v is reached -- and, within one bottleneck, by the least gain
// below it (m2), ancestors first.  Keys (m, m2, -depth) of float-rounded gains: ties and deeper
// bottleneck levels order approximately, which only changes the nodes expanded ahead, never
// the tree (the replay is exact).  A pick's pops before it are the region's nodes with gain > 0
// on the path and a larger key; picks stop at kmax or when the tree's remaining splits are used
// up, as the walk's.  Cost: one pass per level of the known region and two wave passes per pick
// instead of one argmax step per pop (the walk's 3 -> 18 us per plan late in a 63-leaf tree).
__device__ int PredictBottleneck(const KArgs& a, int L, int s, int used, int kround, const double* ng, const int* nch,
                                 const int* tnode, int blocker, unsigned long long* qkey, int* qn, int* s_pick,
                                 int* done_io) {
  const int lane = threadIdx.x & 63;
  int done = *done_io, n = 0;
  const int need = L - 1 - s;
  int kmax = 0;
  if (!done) {
    kmax = min(kround, a.round_need_div > 0 ? max(1, need / a.round_need_div) : need);
    kmax = min(kmax, a.round_emax - used - (need - 1));
    kmax = max(kmax, min(1, a.round_emax - used));
    if (kmax <= 0 || blocker < 0) done = 1;  // (unreachable: the budget keeps room for the blocker)
  }
  if (!done) {
    const int vmax = (a.round_bynode || a.round_xt || a.round_cegb) ? 0 : min(a.round_vmax, 14);
    constexpr uint32_t kPos = 0x80000000u;   // GainKey32(0.0): keys above are gains > 0
    constexpr uint32_t kNone = 0xfffffff0u;  // m2 before a gain below the bottleneck (low 4 bits: 15 - depth)
    for (int l = lane; l <= s; l += kWave) {  // the region's first level: the leaves' nodes
      const int nd = tnode[l];
      qn[l] = nd;
      qkey[l] = (static_cast<unsigned long long>(GainKey32(ng[nd])) << 32) | kNone | 15u;
    }
    WaveLdsSync();
    // the region level by level: an expanded node with m > 0 appends its children
    int head = 0, tail = s + 1;
    while (head < tail) {
      const int i = head + lane, t0 = tail;
      unsigned long long k = 0;
      int c = -1;
      if (i < t0) {
        k = qkey[i];
        c = nch[qn[i]];
      }
      const uint32_t km = static_cast<uint32_t>(k >> 32);
      const bool grow = i < t0 && c >= 0 && km > kPos;
      const unsigned long long bm = __ballot(grow);
      if (grow) {
        const int q = t0 + 2 * __popcll(bm & ((1ull << lane) - 1));
        const uint32_t km2 = static_cast<uint32_t>(k) & kNone;
        const uint32_t d = min(16u - (static_cast<uint32_t>(k) & 15u), 15u);  // the children's depth
        for (int j = 0; j < 2; ++j) {
          const uint32_t kc = GainKey32(ng[c + j]);
          const uint32_t m1 = kc <= km ? kc : km;
          const uint32_t m2 = kc <= km ? kNone : min(km2, kc & kNone);
          qn[q + j] = c + j;
          qkey[q + j] = (static_cast<unsigned long long>(m1) << 32) | m2 | (15u - d);
        }
      }
      tail = t0 + 2 * __popcll(bm);
      head = min(head + kWave, t0);
      WaveLdsSync();
    }
    const int R = tail;
    if (lane == 0) s_pick[0] = blocker;
    n = 1;
    for (; n < kmax; ++n) {
      // the best candidate left: unexpanded, within vmax levels, m > 0, not picked
      unsigned long long bk = 0;
      int bi = -1;
      for (int i = lane; i < R; i += kWave) {
        const int nd = qn[i];
        const unsigned long long k = qkey[i];
        if (nd < 0 || nd == blocker || static_cast<uint32_t>(k >> 32) <= kPos) continue;
        if (15 - static_cast<int>(k & 15u) > vmax || nch[nd] >= 0) continue;
        if (k > bk) {
          bk = k;
          bi = i;
        }
      }
      const unsigned long long gm = WaveMaxDpp(bk);
      if (gm == 0) break;
      // its pops before it: the region's nodes with m > 0 and a larger key
      int cnt = 0;
      for (int i = lane; i < R; i += kWave) {
        const unsigned long long k = qkey[i];
        cnt += (static_cast<uint32_t>(k >> 32) > kPos && k > gm) ? 1 : 0;
      }
      if (WaveSum(cnt) >= need) break;
      const unsigned long long own = __ballot(bi >= 0 && bk == gm);
      const int idx = ReadLane(bi, static_cast<int>(__builtin_ctzll(own)));
      if (lane == 0) {
        const int nd = qn[idx];
        s_pick[n] = nd;
        qn[idx] = -1 - nd;
      }
      WaveLdsSync();
    }
  }
  *done_io = done;
  return done ? 0 : n;
}

// One workgroup.  ROOT: the root's best split from its per-feature results (FindRoot), then
// the first plan.  Otherwise: fold the round's partition counts into its nodes, replay the
// best-first order over the leaves (wave 0, LDS tables): while the argmax leaf's node is
// expanded its split is accepted and its children nodes become the leaves w and s + 1 -- so a
// chain of speculative expansions is accepted in one replay.  Then the next round: the nodes
// the sequential order is predicted to need next, the leaf that ended the replay first,
// within the tree's expansion budget.
// Global loads are issued in few independent batches: every one is a ~1-2 us round trip.
// The finished tree to the host (KArgs::host_out): every split record in order (a numerical
// split's category words skipped), then the scalars with a system-scope release, so the host
// sees them only after the records.
__device__ void HostTreeOut(const KArgs& a, int nsplit, int rounds, int nodes, int draws) {
  constexpr int kRecWords = static_cast<int>(sizeof(SplitRecord) / 8);
  constexpr int kCatWord0 =
      static_cast<int>((__builtin_offsetof(SplitRecord, split) + __builtin_offsetof(DeviceSplit, cat_bits) + 7) / 8);
  static_assert(sizeof(SplitRecord) % 8 == 0, "8-byte words");
  unsigned long long* dst = reinterpret_cast<unsigned long long*>(a.host_out + kHostOutHeaderWords);
  const unsigned long long* src = reinterpret_cast<const unsigned long long*>(a.rec);
  for (int i = threadIdx.x; i < nsplit * kRecWords; i += blockDim.x) {
    const int r = i / kRecWords, w = i - r * kRecWords;
    if (w >= kCatWord0 && !a.rec[r].split.is_categorical) continue;
    dst[i] = src[i];
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_store(&a.host_out[1], nsplit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&a.host_out[2], rounds, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&a.host_out[3], nodes, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&a.host_out[4], draws, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&a.host_out[0], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <bool ROOT, int NT, bool XT>
__device__ void RoundPlanBody(const KArgs& a, unsigned char* plan_lds) {
  constexpr int kPlanThreads = NT;
  __shared__ int s_done, s_s1, s_nexp, s_draw;
  __shared__ ArgC s_arg[kPlanThreads / kWave];
  __shared__ int s_pick[kMaxRoundExp];
  __shared__ int s_pc[kMaxRoundExp];
  // the next round's expansion plans and their children's nodes, composed in LDS by one thread
  // each and stored by every thread in 8-byte words (one thread storing a ~0.9 KB plan field by
  // field took ~3.5 us)
  __shared__ ExpPlan s_e[kMaxRoundExp];
  __shared__ RNode s_c[2 * kMaxRoundExp];
  Round* rd = a.rd;
  const int L = a.p.num_leaves, NF = a.p.num_features, NN = a.round_nodes, tid = threadIdx.x, lane = tid & 63;
  // node tables (gain, -inf when the node has no split; real feature; first child or -1),
  // leaf tables (gain, real feature, node; accepted leaves / nodes) and the prediction's copies
  // of the leaf tables (+ levels below the real leaf)
  const PlanTables T(plan_lds, NN, L);
  double *ng = T.ng, *tg = T.tg, *sg = T.sg;
  int *nrf = T.nrf, *nch = T.nch, *nfi = T.nfi, *trf = T.trf, *tnode = T.tnode, *acc = T.acc, *accn = T.accn,
      *srf = T.srf, *snode = T.snode, *svd = T.svd;
  const int s0 = rd->nsplit;
  const int nexp_prev = rd->nexp;
  const int round0 = rd->round, rounds0 = rd->rounds, accmax0 = rd->accepted_max;
  const int kcur = rd->k_cur;
  const int kround = (kcur > 0 && kcur < a.round_k) ? kcur : a.round_k;  // this tree's round width
  const int nn = rd->next_frow;  // nodes of the tree so far
  const int next_slot = rd->next_slot;
  const bool dp = a.p.data_parallel != 0;  // (global counts: the split's estimates)
  // LGBM_AMD_KTRACE: phase times of the plan (slots 16..24 of the round it ends)
  long long* ktr = (a.ktrace != nullptr && tid == 0 && rd->round < L) ? a.ktrace + static_cast<size_t>(rd->round) * kTraceSlots : nullptr;
  long long tprev = ktr != nullptr ? wall_clock64() : 0;
  if (ktr != nullptr) ktr[16] = tprev;
  auto stamp = [&](int k) {
    if (ktr != nullptr) {
      const long long now = wall_clock64();
      ktr[k] = now - tprev;
      tprev = now;
    }
  };
  if (ROOT) {
    ArgC c = ArgNone();
    for (int f = tid; f < NF; f += kPlanThreads) {
      const FeatureBest& fb = a.feat_best[FeatBestIndex(a, 0, f)];
      if (fb.feature >= 0 && (c.idx < 0 || SplitBetter(fb.gain, fb.real_feature, c.g, c.rf))) {
        c.g = fb.gain;
        c.rf = fb.real_feature;
        c.idx = f;
      }
    }
    c = ArgWaveBest(c);
    if (lane == 0) s_arg[tid >> 6] = c;
    // per-node sampling: the root leaf's row of the reference's flags takes the root scan's flags
    // of the features its sample (draw 0) evaluated; the others keep their (stale) values
    if (a.leaf_rows != nullptr && static_cast<int>(a.root[2]) >= 2 * a.p.sp.min_data_in_leaf) {
      const int8_t* rf0 = a.splittable + static_cast<size_t>(a.leaves[0].frow) * NF;
      for (int f = tid; f < NF; f += kPlanThreads) {
        if (!(a.tree_mask[f] && (a.node_mask == nullptr || a.node_mask[f]))) continue;
        if (a.round_dist) {  // (each rank wrote its own features' flags: the gathered records carry them all)
          const int fl = a.feat_best[FeatBestIndex(a, 0, f)].flag;
          if (fl >= 0) a.leaf_rows[f] = static_cast<int8_t>(fl);
        } else {
          a.leaf_rows[f] = rf0[f];
        }
      }
    }
    __syncthreads();
    ArgC b = s_arg[0];
    for (int k = 1; k < kPlanThreads / kWave; ++k) ArgTake(&b, s_arg[k]);
    if (b.idx >= 0 && b.g == -INFINITY) b.idx = -1;
    if (tid == 0) {
      // node 0: the root leaf and its best split
      FeatureBest fb = {};
      fb.gain = -INFINITY;
      fb.feature = fb.real_feature = -1;
      if (b.idx >= 0) {
        fb = a.feat_best[FeatBestIndex(a, 0, b.idx)];
        const uint32_t* cat = FeatCat(a, 0, b.idx);
        if (fb.ncat > 0) {
          for (int w = 0; w < kMaxCatWords; ++w) a.cbest_cat[w] = cat[w];
        }
        ToDeviceSplit(fb, cat, &a.best[0]);
      } else {
        NoSplit(&a.best[0]);
      }
      a.cbest[0] = fb;
      // (per-node sampling: a root the reference learner does not scan makes no draw -- the
      // host advances its sampler by Round::bynode_next draws)
      if (a.round_bynode && static_cast<int>(a.root[2]) < 2 * a.p.sp.min_data_in_leaf) rd->bynode_next = 0;
      const Leaf R = a.leaves[0];
      RNode r;
      r.begin = R.begin;
      r.count = R.count;
      r.buf = R.buf;
      r.expanded = 0;
      r.child = -1;
      r.total_left = 0;
      r.st.sum_g = R.sum_g;
      r.st.sum_h = R.sum_h;
      r.st.output = R.output;
      r.st.cmin = R.cmin;
      r.st.cmax = R.cmax;
      r.st.global_count = R.global_count;
      r.st.depth = R.depth;
      r.st.slot = R.slot;
      r.st.leaf = 0;
      r.st.frow = 0;
      r.st.icmask = R.icmask;
      a.rnode[0] = r;
      if (a.round_vote) {  // (voting: the local root scan's sums)
        a.rnode_lsum[0] = R.lsum_g;
        a.rnode_lsum[1] = R.lsum_h;
      }
      ng[0] = b.idx >= 0 ? b.g : -INFINITY;
      nrf[0] = b.idx >= 0 ? b.rf : -1;
      nch[0] = -1;
      nfi[0] = b.idx >= 0 ? fb.feature : -1;
      tnode[0] = 0;
      tg[0] = ng[0];
      trf[0] = nrf[0];
    }
  } else {
    // the previous round's partition counts: its children's rows
    if (tid < nexp_prev) {
      const ExpPlan& E = rd->e[tid];
      const int tl = rd->cur[tid][0];
      const int pb = E.part_begin, pc = E.part_count, db = E.dst_buf, c = E.frow_child[0];
      a.rnode[E.node].total_left = tl;
      RNode* cn = a.rnode + c;
      cn[0].begin = pb;
      cn[0].count = tl;
      cn[0].buf = db;
      cn[1].begin = pb + tl;
      cn[1].count = pc - tl;
      cn[1].buf = db;
      if (a.round_vote) {
        // this rank's sums of the children (the local scan's, from k_round_split's fixed point)
        const double hg = static_cast<double>(static_cast<long long>(rd->loc_acc[tid][0])) * a.scales[2];
        const double hh = static_cast<double>(static_cast<long long>(rd->loc_acc[tid][1])) * a.scales[3];
        const int h = E.hist_left ? 0 : 1;
        double* pl = a.rnode_lsum + 2 * E.node;
        double* cl = a.rnode_lsum + 2 * c;
        cl[2 * h] = hg;
        cl[2 * h + 1] = hh;
        cl[2 * (1 - h)] = pl[0] - hg;
        cl[2 * (1 - h) + 1] = pl[1] - hh;
      }
    }
    // one batch of independent loads: every node's best and children, every leaf's node
    for (int n = tid; n < nn; n += kPlanThreads) {
      const FeatureBest& cb = a.cbest[n];
      const double g = cb.gain;
      const int rf = cb.real_feature, fi = cb.feature;
      const int ex = a.rnode[n].expanded, ch = a.rnode[n].child;
      ng[n] = fi >= 0 ? g : -INFINITY;
      nrf[n] = rf;
      nch[n] = ex ? ch : -1;
      nfi[n] = fi;
    }
    for (int l = tid; l <= s0 && l < L; l += kPlanThreads) tnode[l] = a.leaves[l].frow;
    __syncthreads();
    for (int l = tid; l <= s0 && l < L; l += kPlanThreads) {
      tg[l] = ng[tnode[l]];
      trf[l] = nrf[tnode[l]];
    }
  }
  __syncthreads();
  stamp(17);
  // replay of the sequential order by wave 0: the argmax leaf is split while its node is
  // expanded; its children nodes become leaves w and s + 1
  RegLeaf x;
  int done_w = 0, blocker_w = -1;
  int s_w = s0;
  int draw = rd->bynode_next;  // (per-node sampling: the next draw; wave 0 advances it)
  // (extra_trees: the draws counted so far -- the root scan's row 0 for the first plan, then
  // row 1 -- per feature, in LDS; wave 0 advances and stores them)
  __shared__ int s_xcnt[XT ? kXtLaneFeatures * kWave : 1];
  int* xcnt = s_xcnt;
  if (XT && a.round_xt && tid < kWave) {
    for (int f = lane; f < NF; f += kWave) xcnt[f] = a.xt_cum[(ROOT ? 0 : NF) + f];
  }
  if (tid < kWave && L <= kWave) {
    s_w = ReplayRegs<XT>(a, L, s0, ng, nrf, nch, nfi, tnode, acc, accn, &x, &done_w, &draw, xcnt, &blocker_w);
  } else if (tid < kWave) {
    for (;;) {
      if (s_w >= L - 1) {
        done_w = 1;
        break;
      }
      const int w = WaveArgmaxLeaf(tg, trf, s_w, [](int) { return true; });
      if (!(tg[w] > 0.0)) {
        done_w = 1;
        break;
      }
      const int n = tnode[w], c = nch[n];
      if (c < 0) {
        blocker_w = n;
        break;
      }
      bool refunded = false;
      if (a.round_bynode || a.round_cegb || (XT && a.round_xt)) {
        refunded = DeferAccept<XT>(a, s_w, w, n, c, &draw, ng, nrf, nfi, xcnt, -1, tnode);
      }
      if (lane == 0) {
        const int nl = s_w + 1;
        acc[s_w - s0] = w;
        accn[s_w - s0] = n;
        tnode[w] = c;
        tg[w] = ng[c];
        trf[w] = nrf[c];
        tnode[nl] = c + 1;
        tg[nl] = ng[c + 1];
        trf[nl] = nrf[c + 1];
      }
      WaveLdsSync();
      if (refunded) {  // (refunded leaves' new bests)
        for (int l = lane; l <= s_w + 1; l += kWave) {
          tg[l] = ng[tnode[l]];
          trf[l] = nrf[tnode[l]];
        }
        WaveLdsSync();
      }
      ++s_w;
    }
  }
  if (tid == 0) {
    s_s1 = s_w;
    s_draw = draw;
    if (a.round_bynode) rd->bynode_next = draw;
  }
  if (XT && a.round_xt && tid < kWave) {
    for (int f = lane; f < NF; f += kWave) a.xt_cum[NF + f] = xcnt[f];
  }
  __syncthreads();  // the accepted splits and the leaves' final nodes are in LDS
  const int s1 = s_s1, nacc = s1 - s0;
  stamp(18);
  // wave 0 predicts the next round while the other waves write the records of the accepted
  // splits and of the leaves the replay changed (from their final nodes; a leaf changed twice is
  // written twice with the same record) -- those do not depend on the prediction
  auto accepted_record = [&](int i) {
    if (i < nacc) {
      // an accepted split: its record (the node's best split, its partition counts)
      const int k = i;
      const int n = accn[k];
      const FeatureBest& cb = a.cbest[n];
      const int tl = a.rnode[n].total_left, cnt = a.rnode[n].count;
      SplitRecord& rec = a.rec[s0 + k];
      rec.leaf = acc[k];
      rec.left_count = dp ? cb.lc : tl;
      rec.right_count = dp ? cb.rc : cnt - tl;
      ToDeviceSplit(cb, a.cbest_cat + static_cast<size_t>(n) * kMaxCatWords, &rec.split);
    } else {
      const int i2 = i - nacc;
      const int k = i2 >> 1;
      const int l = (i2 & 1) == 0 ? acc[k] : s0 + k + 1;
      const int n = tnode[l];
      const RNode R = a.rnode[n];
      Leaf lf;
      lf.begin = R.begin;
      lf.count = R.count;
      lf.global_count = dp ? R.st.global_count : R.count;
      lf.depth = R.st.depth;
      lf.slot = R.st.slot;
      lf.buf = R.buf;
      lf.frow = n;
      lf.pad = 0;
      lf.icmask = R.st.icmask;
      lf.sum_g = R.st.sum_g;
      lf.sum_h = R.st.sum_h;
      lf.output = R.st.output;
      lf.lsum_g = a.round_vote ? a.rnode_lsum[2 * n] : 0.0;
      lf.lsum_h = a.round_vote ? a.rnode_lsum[2 * n + 1] : 0.0;
      lf.cmin = R.st.cmin;
      lf.cmax = R.st.cmax;
      a.leaves[l] = lf;
      DeviceSplit* d = &a.best[l];
      if (ng[n] != -INFINITY) ToDeviceSplit(a.cbest[n], a.cbest_cat + static_cast<size_t>(n) * kMaxCatWords, d);
      else NoSplit(d);
    }
  };
  if (tid < kWave) {
    int n = 0;
    if (a.round_predict) {
      n = PredictBottleneck(a, L, s1, (nn - 1) / 2, kround, ng, nch, tnode, blocker_w, T.qkey, T.qn, s_pick, &done_w);
      if (ktr != nullptr) ktr[24] = wall_clock64() - tprev;  // (the prediction alone)
    } else if (L <= kWave) {
      n = PredictRegs(a, L, s1, (nn - 1) / 2, kround, ng, nrf, nch, s_pick, &x, &done_w);
    } else if (!done_w) {
      // the sequential order predicted past the blocker from the splits known so far (copies of
      // the leaf tables): an expanded argmax joins its children, an unexpanded one is needed
      // next -- picked (within round_vmax levels below its leaf) with its children unknown.  The
      // blocker is the first pick.
      // budget: after this round, one expansion per split the tree may still need stays
      // available (each round then accepts at least its first pick, the blocker)
      const int need = L - 1 - s1, used = (nn - 1) / 2;
      int kmax = min(kround, a.round_need_div > 0 ? max(1, need / a.round_need_div) : need);
      kmax = min(kmax, a.round_emax - used - (need - 1));
      kmax = max(kmax, min(1, a.round_emax - used));
      if (kmax <= 0) done_w = 1;  // (unreachable: the budget keeps room for the blocker)
      for (int l = lane; l <= s1; l += kWave) {
        sg[l] = tg[l];
        srf[l] = trf[l];
        snode[l] = tnode[l];
        svd[l] = 0;
      }
      WaveLdsSync();
      const int vmax = (a.round_bynode || a.round_xt || a.round_cegb) ? 0 : a.round_vmax;  // (deferred folds: the current leaves only)
      for (int ss = s1; !done_w && n < kmax && ss < L - 1; ++ss) {
        const int w = WaveArgmaxLeaf(sg, srf, ss, [](int) { return true; });
        if (!(sg[w] > 0.0)) break;
        const int nd = snode[w], c = nch[nd], v = svd[w];
        if (lane == 0) {
          const int nl = ss + 1;
          if (c >= 0) {
            snode[w] = c;
            sg[w] = ng[c];
            srf[w] = nrf[c];
            svd[w] = v + 1;
            snode[nl] = c + 1;
            sg[nl] = ng[c + 1];
            srf[nl] = nrf[c + 1];
            svd[nl] = v + 1;
          } else {
            if (v <= vmax) s_pick[n] = nd;
            sg[w] = -INFINITY;
            srf[w] = -1;
            sg[nl] = -INFINITY;
            srf[nl] = -1;
            snode[nl] = -1;
          }
        }
        if (c < 0 && v <= vmax) ++n;
        WaveLdsSync();
      }
      if (n == 0) done_w = 1;  // (unreachable: the blocker is the first argmax)
    }
    if (lane == 0) {
      s_done = done_w;
      s_nexp = done_w ? 0 : n;
    }
    if constexpr (NT == kWave) {  // (one wave: the records after the prediction)
      for (int i = lane; i < 3 * nacc; i += kWave) accepted_record(i);
    }
  } else {
    for (int i = tid - kWave; i < 3 * nacc; i += NT - kWave) accepted_record(i);
  }
  __syncthreads();
  if (a.round_cegb && a.cegb_coupled != nullptr && !s_done && s_nexp > 1) {
    // CEGB coupled penalties: a pick past the blocker is expanded only if no refund can change
    // its best split, i.e. no feature of the tree the model has not used yet has a remembered
    // candidate that would beat it with its coupled penalty back (the blocker is accepted first
    // in the next replay, before any refund)
    __shared__ int s_unsafe[kMaxRoundExp];
    const int ne = s_nexp;
    if (tid < ne) s_unsafe[tid] = 0;
    __syncthreads();
    for (int i = tid; i < (ne - 1) * NF; i += kPlanThreads) {
      const int j = 1 + i / NF, f = i - (j - 1) * NF;
      if (!a.tree_mask[f] || a.cegb_used[f]) continue;
      const int node = s_pick[j];
      int leaf = -1;
      for (int l = 0; l <= s1 && l < L; ++l) {
        if (tnode[l] == node) leaf = l;
      }
      if (leaf < 0) continue;
      const FeatureBest& m = a.cegb_mem[static_cast<size_t>(leaf) * NF + f];
      const double g = m.gain + a.cegb_coupled[f];
      const int rf = m.feature < 0 ? 0x7fffffff : m.real_feature;
      const int crf = nrf[node] < 0 ? 0x7fffffff : nrf[node];
      if (g > ng[node] || (g == ng[node] && rf < crf)) s_unsafe[j] = 1;
    }
    __syncthreads();
    if (tid == 0) {
      int m = 1;
      for (int j = 1; j < ne; ++j) {
        if (!s_unsafe[j]) s_pick[m++] = s_pick[j];
      }
      s_nexp = m;
    }
    __syncthreads();
  }
  const int nexp = s_nexp;
  if (ktr != nullptr) {
    ktr[22] = nacc;
    ktr[23] = nexp;
  }
  // the next round's expansions, one thread each: independent loads (one round trip) of the
  // node, its best split, the split feature's record and interaction mask
  const int next_frow = nn;
  const int nbuf = a.round_vmax + 2;
  const int nent = s_done ? 0 : nexp;
  for (int it = tid; it < nent; it += kPlanThreads) {
    {
      const int j = it, node = s_pick[j];
      const int fi = nfi[node];
      const RNode P = a.rnode[node];
      const FeatureBest& cb = a.cbest[node];
      const double lsg = cb.lg, lsh = cb.lh, lo = cb.lo;
      const double rsg = cb.rg, rsh = cb.rh, ro = cb.ro;
      const int lcnt = cb.lc, rcnt = cb.rc, mono = cb.mono, iscat = cb.ncat > 0 ? 1 : 0;
      const IcMask fmask = a.feat_icmask != nullptr ? a.feat_icmask[fi] : kIcAll;
      ExpPlan& e = s_e[j];
      e.feat = a.feat[fi];
      ToDeviceSplit(cb, a.cbest_cat + static_cast<size_t>(node) * kMaxCatWords, &e.split);
      s_pc[j] = P.count;
      const int hl = lcnt <= rcnt ? 1 : 0;
      e.node = node;
      e.part_begin = P.begin;
      e.part_count = P.count;
      e.src_buf = P.buf;
      e.dst_buf = P.buf + 1 == nbuf ? 0 : P.buf + 1;
      e.hist_left = hl;
      e.slot_parent = P.st.slot;
      e.slot_new = next_slot + j;
      // (per-node sampling: the picked leaf's id -- its row of the reference's flags)
      int fp = node;
      if (a.leaf_rows != nullptr) {
        for (int l = 0; l <= s1 && l < L; ++l) {
          if (tnode[l] == node) fp = l;
        }
      }
      e.frow_parent = fp;
      e.frow_child[0] = next_frow + 2 * j;
      e.frow_child[1] = next_frow + 2 * j + 1;
      // children's statistics from the split (basic monotone constraints: the mid-point bound)
      const int depth = P.st.depth + 1;
      double pmin = P.st.cmin, pmax = P.st.cmax, rmin = P.st.cmin, rmax = P.st.cmax;
      if (!iscat) {
        const double mid = (lo + ro) / 2.0f;
        if (mono < 0) {
          pmin = fmax(pmin, mid);
          rmax = fmin(rmax, mid);
        } else if (mono > 0) {
          pmax = fmin(pmax, mid);
          rmin = fmax(rmin, mid);
        }
      }
      const IcMask icm = P.st.icmask & fmask;
      ChildStats lc, rc;
      lc.sum_g = lsg;
      lc.sum_h = lsh;
      lc.output = lo;
      lc.cmin = pmin;
      lc.cmax = pmax;
      lc.global_count = lcnt;
      lc.depth = depth;
      lc.slot = hl ? e.slot_new : P.st.slot;
      lc.leaf = -1;
      lc.frow = e.frow_child[0];
      lc.icmask = icm;
      rc.sum_g = rsg;
      rc.sum_h = rsh;
      rc.output = ro;
      rc.cmin = rmin;
      rc.cmax = rmax;
      rc.global_count = rcnt;
      rc.depth = depth;
      rc.slot = hl ? P.st.slot : e.slot_new;
      rc.leaf = -1;
      rc.frow = e.frow_child[1];
      rc.icmask = icm;
      e.lr[0] = lc;
      e.lr[1] = rc;
      a.rnode[node].expanded = 1;
      a.rnode[node].child = e.frow_child[0];
      RNode C;
      C.begin = C.count = 0;  // (set by the next plan, from the partition counts)
      C.buf = e.dst_buf;
      C.expanded = 0;
      C.child = -1;
      C.total_left = 0;
      C.st = lc;
      s_c[2 * j] = C;
      C.st = rc;
      s_c[2 * j + 1] = C;
    }
  }
  stamp(19);
  if (s_done) {
    if (tid == 0) {
      rd->done = 1;
      rd->nsplit = s1;
      rd->nexp = 0;
      rd->accepted_max = max(accmax0, nacc);
    }
    if (a.host_out != nullptr) {
      __syncthreads();  // (this plan's records are written)
      HostTreeOut(a, s1, rounds0, nn, s_draw);
    }
    return;
  }
  __syncthreads();
  stamp(20);
  if (tid < kWave) {
    // row blocks: one size for the round (at least blk_min_rows, at most the packed headroom),
    // one lane per expansion
    const int pcj = lane < nexp ? s_pc[lane] : 0;
    const unsigned urows = static_cast<unsigned>(WaveSum(pcj));
    // balanced over the grid: the smallest m with blocks of ceil(rows / (m * grid - nexp))
    // rows under the packed headroom; every workgroup then takes m blocks at most (one
    // partial block per expansion rounds up)
    // (the smallest m with ceil(rows / (m g - nexp)) <= cap, i.e. m g - nexp >= ceil(rows / cap);
    // rows and cap are below 2^31, so every dividend fits 32 unsigned bits: no 64-bit divisions)
    const unsigned g = static_cast<unsigned>(max(1, a.round_grid)), cap = static_cast<unsigned>(a.hist_rows_cap);
    const unsigned unexp = static_cast<unsigned>(nexp);
    const unsigned need = (urows + cap - 1u) / cap + unexp;
    const unsigned m = g <= unexp ? 1u : max(1u, (need + g - 1u) / g);
    long long rpb = m * g > unexp ? (urows + m * g - unexp - 1u) / (m * g - unexp) : cap;
    rpb = max(rpb, static_cast<long long>(a.blk_min_rows));
    rpb = min(rpb, static_cast<long long>(cap));
    rpb = max(rpb, 1ll);
    const unsigned rpb32 = static_cast<unsigned>(rpb);  // (32-bit divisions: a 64-bit one is a long call)
    const int nb = lane < nexp ? static_cast<int>((static_cast<unsigned>(pcj) + rpb32 - 1u) / rpb32) : 0;
    const int incl = WavePrefixIncl(nb);
    if (lane < nexp) {
      s_e[lane].blk_off = incl - nb;
      s_e[lane].nblk = nb;
    }
    if (lane == kWave - 1) {
      rd->rpb = static_cast<int>(rpb);
      rd->nblk = incl;
      rd->nexp = nexp;
      rd->nsplit = s1;
      rd->next_slot = next_slot + nexp;
      rd->next_frow = next_frow + 2 * nexp;
      rd->round = ROOT ? 1 : round0 + 1;  // (parity 0 of the first round holds the root histogram)
      rd->rounds = rounds0 + 1;
      rd->accepted_max = max(accmax0, nacc);
    }
  }
  if (tid < kMaxRoundExp) {
    rd->cur[tid][0] = rd->cur[tid][1] = 0;
    rd->loc_acc[tid][0] = rd->loc_acc[tid][1] = 0ull;
  }
  __syncthreads();
  // the plans and the children's nodes (contiguous from next_frow) in 8-byte words; a plan's
  // category set only when its split is categorical (the split kernel reads it only then)
  {
    constexpr int kEW = sizeof(ExpPlan) / 8, kCW = sizeof(RNode) / 8;
    static_assert(sizeof(ExpPlan) % 8 == 0 && sizeof(RNode) % 8 == 0, "8-byte words");
    // (the words lying wholly inside the category set: its offset need not be 8-aligned)
    constexpr int kCatOff = __builtin_offsetof(ExpPlan, split) + __builtin_offsetof(DeviceSplit, cat_bits);
    constexpr int kCat0 = (kCatOff + 7) / 8;
    constexpr int kCat1 = (kCatOff + 4 * kMaxCatWords) / 8;
    for (int i = tid; i < nexp * kEW; i += kPlanThreads) {
      const int j = i / kEW, w = i - j * kEW;
      if (w >= kCat0 && w < kCat1 && !s_e[j].split.is_categorical) continue;
      reinterpret_cast<unsigned long long*>(&rd->e[j])[w] = reinterpret_cast<const unsigned long long*>(&s_e[j])[w];
    }
    unsigned long long* cdst = reinterpret_cast<unsigned long long*>(a.rnode + next_frow);
    for (int i = tid; i < 2 * nexp * kCW; i += kPlanThreads) cdst[i] = reinterpret_cast<const unsigned long long*>(s_c)[i];
  }
  stamp(21);
}

// (XT: the extra_trees replay's instantiation, launched only with KArgs::round_xt -- its
// registers and stack would slow every other plan)
template <bool ROOT, bool XT>
__global__ __launch_bounds__(kPlanThreads) void k_round_plan(KArgs a) {
  extern __shared__ unsigned char plan_lds[];
  if (a.rd->done) return;
  RoundPlanBody<ROOT, kPlanThreads, XT>(a, plan_lds);
}

namespace {
template <bool ROOT>
void LaunchRoundPlan(const KArgs& a, hipStream_t s) {
  const size_t lds = RoundPlanLds(a.p.num_leaves, a.round_nodes);
  if (a.round_xt) hipLaunchKernelGGL((k_round_plan<ROOT, true>), dim3(1), dim3(kPlanThreads), lds, s, a);
  else hipLaunchKernelGGL((k_round_plan<ROOT, false>), dim3(1), dim3(kPlanThreads), lds, s, a);
}
}  // namespace

size_t RoundPlanLds(int num_leaves, int nodes) {
  const size_t L = static_cast<size_t>(num_leaves), N = static_cast<size_t>(nodes);
  return (2 * N + 2 * L) * sizeof(double) + N * sizeof(int) * 4 + L * sizeof(int) * 7;
}

namespace {

template <int GR, bool VOTE = false>
void LaunchRoundSplit(const KArgs& a, hipStream_t s) {
  const dim3 grid(a.round_grid, a.hist_tiles);
  const size_t lds = sizeof(unsigned long long) * a.hist_units * static_cast<size_t>(a.tile_bins) + sizeof(int) * kSplitSub;
  if (a.sp_ptr != nullptr) {
    if (a.hist_units == 1) hipLaunchKernelGGL((k_round_split<kSparseGPW, 1, GR, VOTE>), grid, dim3(kPartThreads), lds, s, a);
    else hipLaunchKernelGGL((k_round_split<kSparseGPW, 2, GR, VOTE>), grid, dim3(kPartThreads), lds, s, a);
  } else if (a.hist_units == 1) {
    if (a.nibbles) hipLaunchKernelGGL((k_round_split<8, 1, GR, VOTE>), grid, dim3(kPartThreads), lds, s, a);
    else if (a.bin_bytes == 1) hipLaunchKernelGGL((k_round_split<4, 1, GR, VOTE>), grid, dim3(kPartThreads), lds, s, a);
    else if (a.bin_bytes == 2) hipLaunchKernelGGL((k_round_split<2, 1, GR, VOTE>), grid, dim3(kPartThreads), lds, s, a);
    else hipLaunchKernelGGL((k_round_split<0, 1, GR, VOTE>), grid, dim3(kPartThreads), lds, s, a);
  } else {
    if (a.nibbles) hipLaunchKernelGGL((k_round_split<8, 2, GR, VOTE>), grid, dim3(kPartThreads), lds, s, a);
    else if (a.bin_bytes == 1) hipLaunchKernelGGL((k_round_split<4, 2, GR, VOTE>), grid, dim3(kPartThreads), lds, s, a);
    else if (a.bin_bytes == 2) hipLaunchKernelGGL((k_round_split<2, 2, GR, VOTE>), grid, dim3(kPartThreads), lds, s, a);
    else hipLaunchKernelGGL((k_round_split<0, 2, GR, VOTE>), grid, dim3(kPartThreads), lds, s, a);
  }
}

template <int GR, bool VOTE = false>
void AllowRoundSplitLds(int mx) {
  auto allow = [mx](const void* k) {
    if (mx > 65536 && hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, mx) != hipSuccess) {
      (void)hipGetLastError();
    }
  };
  allow(reinterpret_cast<const void*>(k_round_split<8, 1, GR, VOTE>));
  allow(reinterpret_cast<const void*>(k_round_split<8, 2, GR, VOTE>));
  allow(reinterpret_cast<const void*>(k_round_split<4, 1, GR, VOTE>));
  allow(reinterpret_cast<const void*>(k_round_split<2, 1, GR, VOTE>));
  allow(reinterpret_cast<const void*>(k_round_split<0, 1, GR, VOTE>));
  allow(reinterpret_cast<const void*>(k_round_split<4, 2, GR, VOTE>));
  allow(reinterpret_cast<const void*>(k_round_split<2, 2, GR, VOTE>));
  allow(reinterpret_cast<const void*>(k_round_split<0, 2, GR, VOTE>));
  allow(reinterpret_cast<const void*>(k_round_split<kSparseGPW, 1, GR, VOTE>));
  allow(reinterpret_cast<const void*>(k_round_split<kSparseGPW, 2, GR, VOTE>));
}

bool RoundSimpleGains(const KArgs& a) {
  const SplitParams& p = a.p.sp;
  return !p.use_l1 && !p.use_max_output && !p.use_smoothing && !p.use_mc;
}

template <bool VG, bool PIF>
void LaunchRoundFindT(const KArgs& a, hipStream_t s) {
  const int ny = 2 * a.round_k;
  size_t lds = a.p.max_feature_bins <= kFindLdsBins ? 2 * sizeof(double) * static_cast<size_t>(a.p.max_feature_bins) : 0;
  if (a.plan_in_find) lds = std::max(lds, RoundPlanLds(a.p.num_leaves, a.round_nodes));
  const bool simple = RoundSimpleGains(a);
  const bool narrow = a.p.max_feature_bins <= kWave;
  const dim3 b(narrow ? kWave : kFindThreads), bc(kFindThreads);
  // (voting global scan: every elected slot, numerical or categorical, in both kernels)
  const int ncat = (a.round_vote && a.p.vote_phase == 2) ? a.num_scan : a.p.has_cat;
  const dim3 gn(a.num_scan, ny);
  if (a.p.has_cat) {
    if (narrow) {
      if (simple) hipLaunchKernelGGL((k_round_find<1, true, kWave, VG, PIF>), gn, b, lds, s, a);
      else hipLaunchKernelGGL((k_round_find<1, false, kWave, VG, PIF>), gn, b, lds, s, a);
    } else {
      if (simple) hipLaunchKernelGGL((k_round_find<1, true, kFindThreads, VG, PIF>), gn, b, lds, s, a);
      else hipLaunchKernelGGL((k_round_find<1, false, kFindThreads, VG, PIF>), gn, b, lds, s, a);
    }
    if (a.p.wide_cat) hipLaunchKernelGGL((k_round_find<3, false, kFindThreads, VG, PIF>), dim3(ncat, ny), bc, lds, s, a);
    else hipLaunchKernelGGL((k_round_find<2, false, kFindThreads, VG, PIF>), dim3(ncat, ny), bc, lds, s, a);
  } else if (narrow) {
    if (simple) hipLaunchKernelGGL((k_round_find<0, true, kWave, VG, PIF>), gn, b, lds, s, a);
    else hipLaunchKernelGGL((k_round_find<0, false, kWave, VG, PIF>), gn, b, lds, s, a);
  } else {
    if (simple) hipLaunchKernelGGL((k_round_find<0, true, kFindThreads, VG, PIF>), gn, b, lds, s, a);
    else hipLaunchKernelGGL((k_round_find<0, false, kFindThreads, VG, PIF>), gn, b, lds, s, a);
  }
}

void LaunchRoundFind(const KArgs& a, hipStream_t s) {
  if (a.round_vote && a.p.vote_phase == 2) LaunchRoundFindT<true, false>(a, s);
  else if (a.plan_in_find) LaunchRoundFindT<false, true>(a, s);
  else LaunchRoundFindT<false, false>(a, s);
}

}  // namespace

// distributed rounds: each child's best split from the gathered per-feature results; the last
// child to finish plans the next round (as k_round_find's last workgroup does on one process),
// so the gather is followed by one launch instead of a fold and a plan kernel
__global__ __launch_bounds__(kFindThreads) void k_round_childbest(KArgs a) {
  __shared__ RoundFindShared<0, kFindThreads> sh;
  __shared__ int s_last;
  extern __shared__ unsigned char plan_lds[];
  // every workgroup counts, an idle one too: the plan rewrites Round::nexp / done, so it may run
  // only once no workgroup of this launch can still read them (a workgroup dispatched late --
  // the GPU shared with other ranks' kernels -- would otherwise take the next round's nexp)
  Round* rd = a.rd;
  const int done = rd->done, nexp = rd->nexp;
  const int y = blockIdx.x;
  if (!done && y < 2 * nexp) {
    const int node = rd->e[y >> 1].frow_child[y & 1];
    ChildBest<0, kFindThreads>(a, y, node, sh);
    // deferred folds (per-node sampling, CEGB): every rank's copy of the child's per-feature
    // results and flags, from the gathered records (each rank scanned only its own features)
    if (a.round_dist && !a.round_vote && (a.node_fb != nullptr || a.leaf_rows != nullptr)) {
      const int NF = a.p.num_features;
      typedef __attribute__((address_space(1))) int8_t GlobalI8;
      for (int f = threadIdx.x; f < NF; f += blockDim.x) {
        if (!a.tree_mask[f]) continue;  // (no owner this tree)
        const size_t wi = RoundFbIndex(a, y, f);
        const FeatureBest r = a.feat_best[wi];
        if (a.node_fb != nullptr) PublishRecord(&a.node_fb[static_cast<size_t>(node) * NF + f], r);
        if (r.flag >= 0) {
          __hip_atomic_store((GlobalI8*)(a.splittable + static_cast<size_t>(node) * NF + f), static_cast<int8_t>(r.flag),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (a.node_fb_cat != nullptr && a.node_cat_slot[f] >= 0 && r.ncat > 0) {
          PublishCatCopy(a.node_fb_cat + (static_cast<size_t>(node) * a.node_cat_slots + a.node_cat_slot[f]) * kMaxCatWords,
                         a.feat_cat + wi * kMaxCatWords);
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  ArrivalRelease();
  __syncthreads();
  if (threadIdx.x == 0) {
    int last = 0;
    if (atomicAdd(&rd->child_done, 1u) == gridDim.x - 1u) {
      last = 1;
      rd->child_done = 0u;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last || done) return;
  RoundPlanBody<false, kFindThreads>(a, plan_lds);
}

void PrepareRoundKernels(int max_lds) {
  auto allow = [max_lds](const void* k) {
    if (max_lds > 65536 && hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds) != hipSuccess) {
      (void)hipGetLastError();
    }
  };
  allow(reinterpret_cast<const void*>(k_round_hist<8, 1>));
  allow(reinterpret_cast<const void*>(k_round_hist<8, 2>));
  allow(reinterpret_cast<const void*>(k_round_hist<4, 1>));
  allow(reinterpret_cast<const void*>(k_round_hist<2, 1>));
  allow(reinterpret_cast<const void*>(k_round_hist<0, 1>));
  allow(reinterpret_cast<const void*>(k_round_hist<4, 2>));
  allow(reinterpret_cast<const void*>(k_round_hist<2, 2>));
  allow(reinterpret_cast<const void*>(k_round_hist<0, 2>));
  allow(reinterpret_cast<const void*>(k_round_hist<kSparseGPW, 1>));
  allow(reinterpret_cast<const void*>(k_round_hist<kSparseGPW, 2>));
  AllowRoundSplitLds<2>(max_lds);
  AllowRoundSplitLds<4>(max_lds);
  AllowRoundSplitLds<8>(max_lds);
  AllowRoundSplitLds<2, true>(max_lds);
  // the plans' node tables (RoundPlanLds) pass 64 KiB from ~400 leaves
  allow(reinterpret_cast<const void*>(k_round_plan<true, false>));
  allow(reinterpret_cast<const void*>(k_round_plan<false, false>));
  allow(reinterpret_cast<const void*>(k_round_plan<true, true>));
  allow(reinterpret_cast<const void*>(k_round_plan<false, true>));
  allow(reinterpret_cast<const void*>(k_round_childbest));
}

void RoundRootPlan(const KArgs& a, hipStream_t s) {
  LaunchRoundPlan<true>(a, s);
}

void RoundStep(const KArgs& a, hipStream_t s) {
  RoundSplitReduce(a, s);
  RoundFind(a, s);
  if (!a.plan_in_find) {
    LaunchRoundPlan<false>(a, s);
  }
}

void RoundFind(const KArgs& a, hipStream_t s) { LaunchRoundFind(a, s); }

void RoundFindElected(const KArgs& a, hipStream_t s) { LaunchRoundFind(a, s); }  // (a: vote_phase 2, num_scan vote_k)

void RoundChildBestAndPlan(const KArgs& a, hipStream_t s) {
  static_assert(kPlanThreads == kFindThreads, "the fold's workgroup runs the plan");
  hipLaunchKernelGGL(k_round_childbest, dim3(2 * a.round_k), dim3(kFindThreads), RoundPlanLds(a.p.num_leaves, a.round_nodes),
                     s, a);
}

void RoundSplitReduce(const KArgs& a, hipStream_t s) {
  if (a.round_fused) {
    const int gr = a.round_gr > 0 ? a.round_gr
                   : ((a.sp_ptr != nullptr || a.tile_words <= kRGatherNarrowMaxWords) ? kRGatherNarrow : kRGatherWide);
    if (a.round_vote) LaunchRoundSplit<2, true>(a, s);  // (voting: the local sums' variant)
    else if (gr >= 8) LaunchRoundSplit<8>(a, s);
    else if (gr >= 4) LaunchRoundSplit<4>(a, s);
    else LaunchRoundSplit<2>(a, s);
  } else {
    hipLaunchKernelGGL(k_round_part, dim3(a.round_grid), dim3(kPartThreads), 0, s, a);
    const dim3 grid(a.root_grid, a.hist_tiles);
    const size_t lds = sizeof(unsigned long long) * a.hist_units * static_cast<size_t>(a.tile_bins);
    if (a.sp_ptr != nullptr) {
      if (a.hist_units == 1) hipLaunchKernelGGL((k_round_hist<kSparseGPW, 1>), grid, dim3(kHistThreads), lds, s, a);
      else hipLaunchKernelGGL((k_round_hist<kSparseGPW, 2>), grid, dim3(kHistThreads), lds, s, a);
    } else if (a.hist_units == 1) {
      if (a.nibbles) hipLaunchKernelGGL((k_round_hist<8, 1>), grid, dim3(kHistThreads), lds, s, a);
      else if (a.bin_bytes == 1) hipLaunchKernelGGL((k_round_hist<4, 1>), grid, dim3(kHistThreads), lds, s, a);
      else if (a.bin_bytes == 2) hipLaunchKernelGGL((k_round_hist<2, 1>), grid, dim3(kHistThreads), lds, s, a);
      else hipLaunchKernelGGL((k_round_hist<0, 1>), grid, dim3(kHistThreads), lds, s, a);
    } else {
      if (a.nibbles) hipLaunchKernelGGL((k_round_hist<8, 2>), grid, dim3(kHistThreads), lds, s, a);
      else if (a.bin_bytes == 1) hipLaunchKernelGGL((k_round_hist<4, 2>), grid, dim3(kHistThreads), lds, s, a);
      else if (a.bin_bytes == 2) hipLaunchKernelGGL((k_round_hist<2, 2>), grid, dim3(kHistThreads), lds, s, a);
      else hipLaunchKernelGGL((k_round_hist<0, 2>), grid, dim3(kHistThreads), lds, s, a);
    }
  }
  const dim3 rgrid((a.p.total_bins + 255) / 256,
                   std::min(4, (a.hist_max_blocks + kReduceChunk - 1) / kReduceChunk), a.round_k);
  if (a.hist_units == 1) hipLaunchKernelGGL((k_round_reduce<1>), rgrid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((k_round_reduce<2>), rgrid, dim3(256), 0, s, a);
}

}  // namespace dev
}  // namespace lgbm_amd
