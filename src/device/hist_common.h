// LDS histogram accumulation shared by the root / range histogram kernels (hist_kernels.hip)
// and the fused split kernel (partition_kernels.hip).
#pragma once

#include "device_common.h"

namespace lgbm_amd {
namespace dev {

// per-thread constants of a column tile (one 32-bit word of a row per thread)
struct TileCtx {
  int w0, w1, lo_bin, nbins;
  int tpr, rpp, q, rs;  // threads per row, rows per pass, my word, my row slot
  int goff[8];          // histogram offset of each group of my word inside the tile (-1: none)
  int bits;             // bits per group of my word (4, 8 or 16)
  float sg, sh;         // fixed-point scales
};

// row-sparse storage (KArgs::sp_ptr) takes the GPW slot of the kernels' templates
constexpr int kSparseGPW = 1;
constexpr int kSparsePer = kSparsePerThread;  // (KArgs::sp_team threads per row)

// GPW: groups per word (8: 4-bit layout, 4: 8-bit layout, 2: 16-bit layout, 0: mixed layout,
// one more round trip for the word table) or kSparseGPW; otherwise every load is independent
// of the others
template <int GPW>
__device__ __forceinline__ void InitTile(const KArgs& a, TileCtx* t) {
  if (GPW == kSparseGPW) {  // tile = bin range; KArgs::sp_team threads per row
    t->lo_bin = (a.tile_w0 + blockIdx.y) * a.tile_bins;
    t->nbins = min(a.p.total_bins, t->lo_bin + a.tile_bins) - t->lo_bin;
    t->w0 = t->w1 = 0;
    t->tpr = a.sp_team;
    t->rpp = kHistThreads / a.sp_team;
    t->q = threadIdx.x % a.sp_team;
    t->rs = threadIdx.x / a.sp_team;
    t->bits = 0;
    t->sg = static_cast<float>(a.scales[0]);
    t->sh = static_cast<float>(a.scales[1]);
#pragma unroll
    for (int j = 0; j < 8; ++j) t->goff[j] = -1;
    return;
  }
  t->w0 = a.tile_w0 + blockIdx.y * a.tile_words;
  t->w1 = min(a.tile_w1, t->w0 + a.tile_words);
  t->tpr = t->w1 - t->w0;
  t->rpp = kHistThreads / t->tpr;
  t->q = threadIdx.x % t->tpr;
  t->rs = threadIdx.x / t->tpr;
  const int w = t->w0 + t->q;
  int g0, g_end, gfirst, gcount;
  if (GPW == 0) {
    g0 = a.word_g0[t->w0];
    g_end = a.word_g0[t->w1];
    gfirst = a.word_g0[w];
    gcount = a.word_g0[w + 1] - gfirst;
    t->bits = a.word_wide[w] ? 16 : 8;
  } else {
    g0 = t->w0 * GPW;
    g_end = min(a.p.num_groups, t->w1 * GPW);
    gfirst = w * GPW;
    gcount = GPW;
    t->bits = 32 / GPW;
  }
  constexpr int kG = GPW == 8 ? 8 : 4;  // groups a word can hold
  int graw[kG];
#pragma unroll
  for (int j = 0; j < kG; ++j) {
    const int g = gfirst + j;
    graw[j] = (j < gcount && g < a.p.num_groups) ? a.group_off[g] : -1;
  }
  t->lo_bin = a.group_off[g0];
  const int hi_bin = g_end < a.p.num_groups ? a.group_off[g_end] : a.p.total_bins;
  t->sg = static_cast<float>(a.scales[0]);
  t->sh = static_cast<float>(a.scales[1]);
  t->nbins = hi_bin - t->lo_bin;
#pragma unroll
  for (int j = 0; j < kG; ++j) t->goff[j] = graw[j] >= 0 ? graw[j] - t->lo_bin : -1;
}

// Group bin 0 holds every row whose features all sit in their most frequent bin: it is
// outside every feature's histogram range (bin_offsets start at 1) and is restored by
// FixHistogram, so it is never accumulated (this also skips most rows of sparse columns).
// UNITS 1: one packed u64 per bin (g * sg in the signed high half, h * sh in the low half);
// UNITS 2: int64 g and int64 h per bin.  The products are exact (power-of-two scales), the
// rounding to integers is the only quantisation.
// bits: bits per group of the word (GPW 0, mixed layouts)
template <int GPW, int UNITS>
__device__ __forceinline__ void AddRow(unsigned long long* lds, const int* goff, int bits, uint32_t w, float2 v,
                                       float sg, float sh) {
  const long long gq = __float2ll_rn(v.x * sg);
  const long long hq = __float2ll_rn(v.y * sh);
  const unsigned long long pk = (static_cast<unsigned long long>(gq) << 32) + static_cast<unsigned long long>(hq);
#pragma unroll
  for (int j = 0; j < (GPW == 0 ? 4 : GPW); ++j) {
    uint32_t b;
    if (GPW == 0) b = (w >> ((bits * j) & 31)) & (bits == 8 ? 0xffu : 0xffffu);
    else if (GPW == 8) b = (w >> (4 * j)) & 0xfu;
    else b = GPW == 4 ? ((w >> (8 * j)) & 0xffu) : ((w >> (16 * j)) & 0xffffu);
    if (goff[j] >= 0 && b != 0u) {
      if (UNITS == 1) {
        atomicAdd(&lds[goff[j] + b], pk);
      } else {
        atomicAdd(&lds[2 * (goff[j] + b)], static_cast<unsigned long long>(gq));
        atomicAdd(&lds[2 * (goff[j] + b) + 1], static_cast<unsigned long long>(hq));
      }
    }
  }
}

// row-sparse gather of K rows (rr[k] < 0: none) with values v[k]: the t.tpr threads of a row
// take its entries round robin.  The first kSparsePer entries of each thread and row are loaded
// together (one round trip after the rows' bounds; the team size is chosen so that a mean row
// fits); longer rows continue with the K rows' next entries loaded together per round trip.
// Entries outside the tile's bin range are skipped.
template <int K, int UNITS>
__device__ __forceinline__ void AddSparseRows(const KArgs& a, unsigned long long* lds, const TileCtx& t,
                                              const int* rr, const float2* v) {
  const int T = t.tpr;
  int64_t beg[K];
  int cnt[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int x = rr[k] >= 0 ? rr[k] : 0;
    beg[k] = a.sp_ptr[x];
    const int64_t end = a.sp_ptr[x + 1];
    cnt[k] = rr[k] >= 0 ? static_cast<int>(end - beg[k]) : 0;
  }
  uint32_t e[K][kSparsePer];
#pragma unroll
  for (int k = 0; k < K; ++k) {
#pragma unroll
    for (int m = 0; m < kSparsePer; ++m) {
      const int j = t.q + m * T;
      e[k][m] = j < cnt[k] ? static_cast<uint32_t>(a.sp_bin[beg[k] + j]) : 0xffffffffu;
    }
  }
  const uint32_t lo = static_cast<uint32_t>(t.lo_bin), nb = static_cast<uint32_t>(t.nbins);
  long long gq[K], hq[K];
  int longest = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    gq[k] = __float2ll_rn(v[k].x * t.sg);
    hq[k] = __float2ll_rn(v[k].y * t.sh);
    longest = max(longest, cnt[k]);
  }
  auto add = [&](int k, uint32_t bin) {
    const uint32_t b = bin - lo;
    if (b < nb) {
      if (UNITS == 1) {
        atomicAdd(&lds[b], (static_cast<unsigned long long>(gq[k]) << 32) + static_cast<unsigned long long>(hq[k]));
      } else {
        atomicAdd(&lds[2 * b], static_cast<unsigned long long>(gq[k]));
        atomicAdd(&lds[2 * b + 1], static_cast<unsigned long long>(hq[k]));
      }
    }
  };
#pragma unroll
  for (int k = 0; k < K; ++k) {
#pragma unroll
    for (int m = 0; m < kSparsePer; ++m) add(k, e[k][m]);
  }
  for (int j = t.q + kSparsePer * T; j < longest; j += T) {
    uint32_t x[K];
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = j < cnt[k] ? static_cast<uint32_t>(a.sp_bin[beg[k] + j]) : 0xffffffffu;
#pragma unroll
    for (int k = 0; k < K; ++k) add(k, x[k]);
  }
}

// ---- row-block histogram of an explicit row range (root pass, host-assisted ranges, round
// growth's histogrammed children): see hist_kernels.hip
#ifndef LGBM_ROOT_ROWS
#define LGBM_ROOT_ROWS 8
#endif
constexpr int kRowsInFlight = LGBM_ROOT_ROWS;  // independent row gathers per thread

__device__ __forceinline__ void LoadRowIdx(const int32_t* src, int i, int r1, int rpp, int* r) {
#pragma unroll
  for (int k = 0; k < kRowsInFlight; ++k) {
    const int ii = i + k * rpp;
    r[k] = ii < r1 ? (src ? src[ii] : ii) : -1;
  }
}

// one row block [r0, r1) of one column tile -> its partial histogram `out`.  The index
// loads of each batch are issued one batch ahead (the first ones while the LDS is cleared).
// ROOT: the root pass writes the identity row indices of column tile 0 while it reads them
template <bool ROOT, int GPW, int UNITS>
__device__ __forceinline__ void HistBlock(const KArgs& a, unsigned long long* lds, const int32_t* src, int r0, int r1,
                                          const TileCtx& t, unsigned long long* out) {
  const bool active = t.rs < t.rpp;
  int i = r0 + t.rs;
  int r[kRowsInFlight];
  if (active) LoadRowIdx(src, i, r1, t.rpp, r);
  __syncthreads();  // LDS reuse across row blocks
  for (int j = threadIdx.x; j < UNITS * t.nbins; j += kHistThreads) lds[j] = 0ull;
  __syncthreads();
  if (active) {
    const int w = t.w0 + t.q;
    const uint32_t* bins32 = static_cast<const uint32_t*>(a.bins);
    const int64_t wpr = a.row_words;
    const bool write_iota = ROOT && src == nullptr && t.q == 0 && blockIdx.y == 0;
    const int stride = kRowsInFlight * t.rpp;
    for (; i < r1; i += stride) {
      if (write_iota) {
#pragma unroll
        for (int k = 0; k < kRowsInFlight; ++k) {
          if (r[k] >= 0) a.idx[i + k * t.rpp] = r[k];
        }
      }
      float2 v[kRowsInFlight];
      int rn[kRowsInFlight];
      if constexpr (GPW == kSparseGPW) {
#pragma unroll
        for (int k = 0; k < kRowsInFlight; ++k) v[k] = GhAt(a, r[k] >= 0 ? r[k] : 0);
        LoadRowIdx(src, i + stride, r1, t.rpp, rn);
        AddSparseRows<kRowsInFlight, UNITS>(a, lds, t, r, v);
      } else {
        uint32_t wd[kRowsInFlight];
#pragma unroll
        for (int k = 0; k < kRowsInFlight; ++k) {
          const int rr = r[k] >= 0 ? r[k] : 0;
          v[k] = GhAt(a, rr);
          wd[k] = r[k] >= 0 ? bins32[rr * wpr + w] : 0u;  // word 0: every bin skipped
        }
        LoadRowIdx(src, i + stride, r1, t.rpp, rn);  // next batch, in flight during the atomics
#pragma unroll
        for (int k = 0; k < kRowsInFlight; ++k) AddRow<GPW, UNITS>(lds, t.goff, t.bits, wd[k], v[k], t.sg, t.sh);
      }
#pragma unroll
      for (int k = 0; k < kRowsInFlight; ++k) r[k] = rn[k];
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < UNITS * t.nbins; j += kHistThreads) out[j] = lds[j];
}

template <int MODE>
void LaunchReduce(const KArgs& a, hipStream_t s);

}  // namespace dev
}  // namespace lgbm_amd
