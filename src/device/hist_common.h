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
  int goff[4];          // histogram offset of each group of my word inside the tile (-1: none)
  int bits;             // bits per group of my word (8 or 16)
  float sg, sh;         // fixed-point scales
};

// GPW: groups per word (4: 8-bit layout, 2: 16-bit layout, 0: mixed layout, one more round
// trip for the word table); otherwise every load is independent of the others
template <int GPW>
__device__ __forceinline__ void InitTile(const KArgs& a, TileCtx* t) {
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
  int graw[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int g = gfirst + j;
    graw[j] = (j < gcount && g < a.p.num_groups) ? a.group_off[g] : -1;
  }
  t->lo_bin = a.group_off[g0];
  const int hi_bin = g_end < a.p.num_groups ? a.group_off[g_end] : a.p.total_bins;
  t->sg = static_cast<float>(a.scales[0]);
  t->sh = static_cast<float>(a.scales[1]);
  t->nbins = hi_bin - t->lo_bin;
#pragma unroll
  for (int j = 0; j < 4; ++j) t->goff[j] = graw[j] >= 0 ? graw[j] - t->lo_bin : -1;
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

template <int MODE>
void LaunchReduce(const KArgs& a, hipStream_t s);

}  // namespace dev
}  // namespace lgbm_amd
