// Listwise ranking gradients on device: LambdaRank-NDCG and XE-NDCG, one workgroup per
// query (reference src/objective/rank_objective.hpp:98-285 lambdarank, :288-366 xendcg).
//
// A query's documents are staged in LDS (score, label, rank position), or -- queries of more
// than kRankMaxDocs documents -- in a global scratch of the query's own rows, scanned by a
// 1024-thread workgroup (the same code over other storage).  The stable descending sort of the
// reference (std::stable_sort by score) is computed as a rank:
// pos(d) = #{j : s_j > s_d} + #{j < d : s_j == s_d}, O(cnt^2 / threads) broadcasts
// (queries are short: MS-LTR averages ~120 documents).  Every document then accumulates its
// lambda / hessian over the pairs it takes part in in the reference's order (below), so no
// atomics are needed and the result does not depend on scheduling.
#include "device_common.h"

namespace lgbm_amd {
namespace dev {

constexpr int kRankThreads = 128;      // two waves per query
constexpr int kRankBigThreads = 1024;  // queries of more than kRankMaxDocs documents

template <int NT>
__device__ __forceinline__ double RankBlockSum(double v, double* red) {
  for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  const int w = threadIdx.x / kWave;
  __syncthreads();  // red may still be read by a previous reduction
  if ((threadIdx.x & (kWave - 1)) == 0) red[w] = v;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < NT / kWave; ++i) t += red[i];
  return t;
}

// the host objective's sigmoid table (reference rank_objective.hpp:230-245: 1M entries of
// 1 / (1 + exp(x * sigmoid)) over [min, max]), uploaded: the device's exp may differ from the
// host's in the last bit, the table's entries do not
__device__ __forceinline__ double RankSigmoid(const RankArgs& ra, double x) {
  if (x <= ra.sig_min) return ra.sig_table[0];
  if (x >= ra.sig_max) return ra.sig_table[kRankSigmoidBins - 1];
  return ra.sig_table[static_cast<size_t>((x - ra.sig_min) * ra.sig_factor)];
}

// One workgroup per query.  The gradients equal the host's bit for bit (so that device GOSS
// keeps the host's rows): the reference accumulates a document's lambda in float as the
// lower-labelled side of each pair, in the sorted order of the pair's higher side
// (`lambdas[low] -= (float)p`), and adds its own pairs' double sum as the higher side when the
// outer loop reaches its sorted position (`lambdas[high] += (float)sum`,
// rank_objective.hpp:164-221).  Each thread replays that sequence for its documents over the
// sorted order (s_doc), with the host's operation order and no contraction into FMAs.  (The
// normalisation's sum of |lambdas| is a workgroup reduction in double: it differs from the host's
// sequential sum in its last bits only, which reach a float gradient through the log2 factor with
// probability ~2^-29.)
template <int NT>
__device__ void LambdarankQuery(const RankArgs& ra, int q, double* s_score, int* s_label, int* s_pos, int* s_doc,
                                double* s_red, double* s_edge, double* s_disc, float2* pairs, double* hs_lam,
                                double* hs_hes) {
#pragma clang fp contract(off)
  const int b = ra.qb[q];
  const int cnt = ra.qb[q + 1] - b;
  for (int i = threadIdx.x; i < cnt; i += NT) {
    s_score[i] = ra.score[b + i];
    s_label[i] = static_cast<int>(ra.label[b + i]);
    if (s_disc != nullptr) s_disc[i] = ra.discount[i];
  }
  const double* disc = s_disc != nullptr ? s_disc : ra.discount;
  __syncthreads();
  for (int i = threadIdx.x; i < cnt; i += NT) {
    const double si = s_score[i];
    int p = 0;
    for (int j = 0; j < cnt; ++j) {
      const double sj = s_score[j];
      p += (sj > si) | ((sj == si) & (j < i));
    }
    s_pos[i] = p;
    s_doc[p] = i;
    if (p == 0) s_edge[0] = si;
    if (p == cnt - 1) s_edge[1] = si;
    if (p == cnt - 2) s_edge[2] = si;
  }
  __syncthreads();
  const double best = s_edge[0];
  const double worst = (cnt - 1 > 0 && s_edge[1] == kMinScore) ? s_edge[2] : s_edge[1];
  const double inv_max = ra.inv_max_dcg[q];
  const double sig = ra.sigmoid;
  const bool norm = ra.norm != 0 && best != worst;
  // the pair (high, low): its lambda and hessian as rank_objective.hpp:186-209 computes them
  auto pair = [&](double hs, int hl, double hd, double ls, int ll, double ld, double* pl_out, double* ph_out) {
    const double ds = hs - ls;
    const double dcg_gap = ra.label_gain[hl] - ra.label_gain[ll];
    const double paired = fabs(hd - ld);
    double dn = dcg_gap * paired * inv_max;
    if (norm) dn /= (0.01f + fabs(ds));
    double pl = RankSigmoid(ra, ds);
    double ph = pl * (1.0f - pl);
    pl *= -sig * dn;
    ph *= sig * sig * dn;
    *pl_out = pl;
    *ph_out = ph;
  };
  double sum_lambdas = 0.0;
  for (int d = threadIdx.x; d < cnt; d += NT) {
    const double sd = s_score[d];
    const int ld = s_label[d], kd = s_pos[d];
    const double disc_d = disc[kd];
    // d as the higher side: its pairs in the sorted order of the lower side, summed in double
    // (a loop of its own, run by every lane together: nested inside the sorted-order loop below
    // at k == kd it ran once per lane, serialised over the wave -- 30x slower)
    double hsl = 0.0, hsh = 0.0;
    if (sd != kMinScore) {
      for (int k2 = 0; k2 < cnt; ++k2) {
        if (k2 == kd) continue;
        const int j = s_doc[k2];
        const int lj = s_label[j];
        const double sj = s_score[j];
        if (ld <= lj || sj == kMinScore) continue;
        double pl, ph;
        pair(sd, ld, disc_d, sj, lj, disc[k2], &pl, &ph);
        hsl += pl;
        hsh += ph;
        sum_lambdas -= 2 * pl;
        // (the lower side's float terms, read back below in its own order)
        if (pairs != nullptr) pairs[static_cast<size_t>(kd) * cnt + j] = make_float2(static_cast<float>(pl), static_cast<float>(ph));
      }
    }
    hs_lam[d] = hsl;  // (d's double sums: the second loop runs after the block's pair writes)
    hs_hes[d] = hsh;
  }
  if (pairs != nullptr) __syncthreads();  // (block scope: the pair scratch is complete)
  for (int d = threadIdx.x; d < cnt; d += NT) {
    const double sd = s_score[d];
    const int ld = s_label[d], kd = s_pos[d];
    const double disc_d = disc[kd];
    const double hsl = hs_lam[d], hsh = hs_hes[d];
    float lam = 0.0f, hes = 0.0f;
    for (int k = 0; k < cnt; ++k) {
      if (k == kd) {
        if (sd == kMinScore) continue;
        lam = __fadd_rn(lam, static_cast<float>(hsl));
        hes = __fadd_rn(hes, static_cast<float>(hsh));
      } else {
        // d as the lower side of the pair with the document at sorted position k
        const int j = s_doc[k];
        const int lj = s_label[j];
        const double sj = s_score[j];
        if (sj == kMinScore || lj <= ld || sd == kMinScore) continue;
        if (pairs != nullptr) {
          const float2 v = pairs[static_cast<size_t>(k) * cnt + d];
          lam = __fsub_rn(lam, v.x);
          hes = __fadd_rn(hes, v.y);
        } else {
          double pl, ph;
          pair(sj, lj, disc[k], sd, ld, disc_d, &pl, &ph);
          lam = __fsub_rn(lam, static_cast<float>(pl));
          hes = __fadd_rn(hes, static_cast<float>(ph));
        }
      }
    }
    ra.grad[b + d] = lam;
    ra.hess[b + d] = hes;
  }
  const double total = RankBlockSum<NT>(sum_lambdas, s_red);
  const bool renorm = ra.norm != 0 && total > 0;
  const double nf = renorm ? log2(1 + total) / total : 1.0;
  if (!renorm && ra.weights == nullptr) return;
  for (int d = threadIdx.x; d < cnt; d += NT) {
    float g = ra.grad[b + d], h = ra.hess[b + d];
    if (renorm) {
      g = static_cast<float>(g * nf);
      h = static_cast<float>(h * nf);
    }
    if (ra.weights != nullptr) {  // (reference RankingObjective::GetGradients: float products)
      g = __fmul_rn(g, ra.weights[b + d]);
      h = __fmul_rn(h, ra.weights[b + d]);
    }
    ra.grad[b + d] = g;
    ra.hess[b + d] = h;
  }
}

// LDS per query document: score, discount, the two double sums (8 B each); label, sorted
// position, document at position (4 B each)
constexpr int kRankLdsPerDoc = 4 * 8 + 3 * 4;
size_t RankLds(int max_docs) { return static_cast<size_t>(std::max(1, max_docs)) * kRankLdsPerDoc; }

__global__ __launch_bounds__(kRankThreads) void k_lambdarank(RankArgs ra) {
  extern __shared__ double rank_lds[];  // RankLds(ra.max_docs) bytes
  const int M = ra.max_docs;
  double* s_score = rank_lds;
  double* s_disc = s_score + M;
  double* s_hl = s_disc + M;
  double* s_hh = s_hl + M;
  int* s_label = reinterpret_cast<int*>(s_hh + M);
  int* s_pos = s_label + M;  // document -> sorted position
  int* s_doc = s_pos + M;    // sorted position -> document
  __shared__ double s_red[kRankThreads / kWave];
  __shared__ double s_edge[3];  // score at sorted positions 0, cnt-1, cnt-2
  const int q = blockIdx.x;
  if (ra.qb[q + 1] - ra.qb[q] > kRankMaxDocs) return;  // (k_lambdarank_big)
  float2* pairs = ra.pair_buf != nullptr ? ra.pair_buf + ra.pair_off[q] : nullptr;
  LambdarankQuery<kRankThreads>(ra, q, s_score, s_label, s_pos, s_doc, s_red, s_edge, s_disc, pairs, s_hl, s_hh);
}

// queries of more than kRankMaxDocs documents: the same body over the query's rows of a global
// scratch (RankArgs::big_*)
__global__ __launch_bounds__(kRankBigThreads) void k_lambdarank_big(RankArgs ra) {
  __shared__ double s_red[kRankBigThreads / kWave];
  __shared__ double s_edge[3];
  const int q = ra.big_q[blockIdx.x];
  const int b = ra.qb[q];
  LambdarankQuery<kRankBigThreads>(ra, q, ra.big_d0 + b, ra.big_i0 + b, ra.big_i1 + b, ra.big_i2 + b, s_red, s_edge,
                                   nullptr, nullptr, ra.big_d1 + b, ra.big_dh + b);
}

// XE-NDCG (reference rank_objective.hpp:304-366): softmax over the query, per-document
// gamma draws from the query's own LCG (state advanced in place across iterations).
template <int NT>
__device__ void XendcgQuery(const RankArgs& ra, int q, double* s_rho, double* s_par, float* s_lam, double* s_red) {
  const int b = ra.qb[q];
  const int cnt = ra.qb[q + 1] - b;
  if (cnt <= 1) {
    for (int i = threadIdx.x; i < cnt; i += NT) ra.grad[b + i] = ra.hess[b + i] = 0.0f;
    return;
  }
  // softmax (common::Softmax: max shift, exp, normalise)
  double mx = -INFINITY;
  for (int i = threadIdx.x; i < cnt; i += NT) mx = fmax(mx, ra.score[b + i]);
  for (int o = kWave / 2; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, kWave));
  __syncthreads();
  if ((threadIdx.x & (kWave - 1)) == 0) s_red[threadIdx.x / kWave] = mx;
  __syncthreads();
  mx = s_red[0];
  for (int i = 1; i < NT / kWave; ++i) mx = fmax(mx, s_red[i]);
  double den = 0.0;
  for (int i = threadIdx.x; i < cnt; i += NT) {
    const double e = exp(ra.score[b + i] - mx);
    s_rho[i] = e;
    den += e;
  }
  den = RankBlockSum<NT>(den, s_red);
  // gamma draws: the query's LCG is sequential over its documents
  if (threadIdx.x == 0) {
    unsigned st = ra.rng[q];
    for (int i = 0; i < cnt; ++i) {
      st = 214013u * st + 2531011u;
      const float u = static_cast<float>(static_cast<int>((st >> 16) & 0x7FFF)) / 32768.0f;
      s_par[i] = exp2(static_cast<double>(static_cast<int>(ra.label[b + i]))) - u;
    }
    ra.rng[q] = st;
  }
  __syncthreads();
  double sp = 0.0;
  for (int i = threadIdx.x; i < cnt; i += NT) {
    s_rho[i] /= den;
    sp += s_par[i];
  }
  sp = RankBlockSum<NT>(sp, s_red);
  const double inv_den = 1.0 / fmax(kEpsilon, sp);
  double s1 = 0.0;
  for (int i = threadIdx.x; i < cnt; i += NT) {
    const double term = -s_par[i] * inv_den + s_rho[i];
    s_lam[i] = static_cast<float>(term);
    s_par[i] = term / (1. - s_rho[i]);
    s1 += s_par[i];
  }
  s1 = RankBlockSum<NT>(s1, s_red);
  double s2 = 0.0;
  for (int i = threadIdx.x; i < cnt; i += NT) {
    const double term = s_rho[i] * (s1 - s_par[i]);
    s_lam[i] += static_cast<float>(term);
    s_par[i] = term / (1. - s_rho[i]);
    s2 += s_par[i];
  }
  s2 = RankBlockSum<NT>(s2, s_red);
  for (int i = threadIdx.x; i < cnt; i += NT) {
    float lam = s_lam[i] + static_cast<float>(s_rho[i] * (s2 - s_par[i]));
    float hes = static_cast<float>(s_rho[i] * (1.0 - s_rho[i]));
    if (ra.weights != nullptr) {
      lam = static_cast<float>(lam * ra.weights[b + i]);
      hes = static_cast<float>(hes * ra.weights[b + i]);
    }
    ra.grad[b + i] = lam;
    ra.hess[b + i] = hes;
  }
}

__global__ __launch_bounds__(kRankThreads) void k_xendcg(RankArgs ra) {
  __shared__ double s_rho[kRankMaxDocs];
  __shared__ double s_par[kRankMaxDocs];
  __shared__ float s_lam[kRankMaxDocs];
  __shared__ double s_red[kRankThreads / kWave];
  const int q = blockIdx.x;
  if (ra.qb[q + 1] - ra.qb[q] > kRankMaxDocs) return;  // (k_xendcg_big)
  XendcgQuery<kRankThreads>(ra, q, s_rho, s_par, s_lam, s_red);
}

__global__ __launch_bounds__(kRankBigThreads) void k_xendcg_big(RankArgs ra) {
  __shared__ double s_red[kRankBigThreads / kWave];
  const int q = ra.big_q[blockIdx.x];
  const int b = ra.qb[q];
  XendcgQuery<kRankBigThreads>(ra, q, ra.big_d0 + b, ra.big_d1 + b, ra.big_f + b, s_red);
}

// k_lambdarank stages up to kRankMaxDocs documents in dynamic LDS (RankLds(kRankMaxDocs) is 88 KiB):
// above 64 KiB the kernel must be enabled once per process, outside any graph capture
void PrepareRankKernels(int max_lds) {
  if (max_lds > 65536 && hipFuncSetAttribute(reinterpret_cast<const void*>(k_lambdarank),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, max_lds) != hipSuccess) {
    (void)hipGetLastError();  // a launch above 64 KiB then fails, and RankGradients reports it
  }
}

size_t RankLdsBytes(int max_docs) { return RankLds(max_docs); }

void RankGradients(const RankArgs& ra, hipStream_t s) {
  if (ra.num_queries <= 0) return;
  if (ra.kind == kRankKindLambdarank) {
    hipLaunchKernelGGL(k_lambdarank, dim3(ra.num_queries), dim3(kRankThreads), RankLds(ra.max_docs), s, ra);
    if (ra.num_big > 0) hipLaunchKernelGGL(k_lambdarank_big, dim3(ra.num_big), dim3(kRankBigThreads), 0, s, ra);
  } else {
    hipLaunchKernelGGL(k_xendcg, dim3(ra.num_queries), dim3(kRankThreads), 0, s, ra);
    if (ra.num_big > 0) hipLaunchKernelGGL(k_xendcg_big, dim3(ra.num_big), dim3(kRankBigThreads), 0, s, ra);
  }
}

}  // namespace dev
}  // namespace lgbm_amd
