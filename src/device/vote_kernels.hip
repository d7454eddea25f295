// Voting-parallel election on the device (reference voting_parallel_tree_learner.cpp:
// FindBestSplits local top-k :300-318, GlobalVoting :151-182, CopyLocalHistogram :184-240).
// Per step, after the local split scan (Params::vote_phase 1) wrote every feature's local best
// into feat_best:
//   k_vote_local   one workgroup: this rank's top-k features per leaf by local gain (ties:
//                  smaller real feature index) -> its block of vote_buf;
//   (allgather of vote_buf over the device communicator)
//   k_vote_elect   one workgroup per leaf side: the election -- each proposal's gain weighted
//                  by its local rows over the mean rows per rank, a feature's best weighted
//                  gain, the top-k features -> vote_list; feat_best of the side is cleared for
//                  the global scan;
//   k_vote_gather  one workgroup per elected feature: its local histogram slice into
//                  vote_hist;
//   (all-reduce of vote_hist, then the global scan, Params::vote_phase 2, picks the split)
// Every rank runs the same election on the same gathered proposals, so the elected lists,
// the global histograms and the picked split are identical on every rank.
#include "pick.h"

namespace lgbm_amd {
namespace dev {

namespace {

constexpr int kVoteThreads = 256;
constexpr int kVoteWaves = kVoteThreads / kWave;

// (gain, real feature) order of LightSplitInfo: larger gain first, then smaller feature
__device__ __forceinline__ bool Better(double ga, int ra, double gb, int rb) {
  if (ga != gb) return ga > gb;
  return ra < rb;
}

struct Cand {
  double gain;
  int real;
  int idx;
};

// block-wide best candidate (every thread gets it)
__device__ __forceinline__ Cand BlockBest(Cand c, Cand* sh) {
  for (int o = 32; o > 0; o >>= 1) {
    Cand d;
    d.gain = __shfl_xor(c.gain, o, kWave);
    d.real = __shfl_xor(c.real, o, kWave);
    d.idx = __shfl_xor(c.idx, o, kWave);
    if (d.idx >= 0 && (c.idx < 0 || Better(d.gain, d.real, c.gain, c.real))) c = d;
  }
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = c;
  __syncthreads();
  Cand b = sh[0];
  for (int i = 1; i < kVoteWaves; ++i) {
    const Cand d = sh[i];
    if (d.idx >= 0 && (b.idx < 0 || Better(d.gain, d.real, b.gain, b.real))) b = d;
  }
  return b;
}

__device__ __forceinline__ bool StepSkipped(const KArgs& a, bool root, ChildInfo* c) {
  if (root) return false;
  *c = StepChildren(a, a.st);
  return c->skip;
}

}  // namespace

// grid (1): this rank's proposals for the root (side 0) or the step's two children
__global__ __launch_bounds__(kVoteThreads) void k_vote_local(KArgs a, int root) {
  __shared__ Cand sh[kVoteWaves];
  __shared__ int taken[64];
  const Step* st = a.st;
  if (!root && st->done) return;
  ChildInfo c;
  const bool skip = StepSkipped(a, root != 0, &c);
  const int k = a.p.vote_k, nf = a.p.num_features;
  VoteEntry* out = a.vote_buf + static_cast<size_t>(a.vote_rank) * 2 * k;
  for (int side = 0; side < 2; ++side) {
    const bool active = !skip && (side == 0 || !root);
    for (int r = 0; r < k; ++r) {
      Cand best;
      best.idx = -1;
      best.gain = -INFINITY;
      best.real = 0x7fffffff;
      if (active) {
        for (int f = threadIdx.x; f < nf; f += kVoteThreads) {
          const FeatureBest& fb = a.feat_best[FeatBestIndex(a, side, f)];
          if (fb.feature < 0 || !(fb.gain > -INFINITY)) continue;
          bool dup = false;
          for (int j = 0; j < r; ++j) dup |= taken[j] == f;
          if (dup) continue;
          if (best.idx < 0 || Better(fb.gain, fb.real_feature, best.gain, best.real)) {
            best.gain = fb.gain;
            best.real = fb.real_feature;
            best.idx = f;
          }
        }
      }
      const Cand b = BlockBest(best, sh);
      if (threadIdx.x == 0) {
        VoteEntry e;
        e.gain = b.idx >= 0 ? b.gain : -INFINITY;
        e.feature = b.idx;
        e.count = 0;
        if (b.idx >= 0) {
          const FeatureBest& fb = a.feat_best[FeatBestIndex(a, side, b.idx)];
          e.count = fb.lc + fb.rc;
        }
        out[side * k + r] = e;
        taken[r] = b.idx;
      }
      __syncthreads();
    }
  }
}

// grid (sides): the election for one side, then that side's feat_best cleared
__global__ __launch_bounds__(kVoteThreads) void k_vote_elect(KArgs a, int root) {
  __shared__ double wg[1024];
  __shared__ int fe[1024];
  __shared__ int rep[1024];
  const Step* st = a.st;
  if (!root && st->done) return;
  const int side = blockIdx.x;
  const int k = a.p.vote_k, W = a.p.world, nf = a.p.num_features;
  int32_t* list = a.vote_list + side * k;
  for (int r = threadIdx.x; r < k; r += kVoteThreads) list[r] = -1;
  ChildInfo c;
  const bool skip = StepSkipped(a, root != 0, &c);
  const int n = W * k;  // proposals of this side (<= 1024: checked on the host)
  if (!skip) {
    // the side's leaf rows over all ranks (the root: the all-reduced root count)
    int global_rows;
    if (root) {
      global_rows = static_cast<int>(a.root[2]);
    } else {
      const SideInfo sd = StepSide(a, st, c, side);
      global_rows = sd.global_count;
    }
    const double mean = static_cast<double>(global_rows) / W;
    for (int i = threadIdx.x; i < n; i += kVoteThreads) {
      const VoteEntry e = a.vote_buf[static_cast<size_t>(i / k) * 2 * k + side * k + (i % k)];
      const bool ok = e.feature >= 0 && e.gain > -INFINITY && mean > 0.0;
      fe[i] = ok ? e.feature : -1;
      wg[i] = ok ? e.gain * e.count / mean : -INFINITY;
    }
    __syncthreads();
    // a feature's representative: its best weighted gain (first such proposal on ties)
    for (int i = threadIdx.x; i < n; i += kVoteThreads) {
      int is_rep = fe[i] >= 0;
      for (int j = 0; j < n && is_rep; ++j) {
        if (j != i && fe[j] == fe[i] && (wg[j] > wg[i] || (wg[j] == wg[i] && j < i))) is_rep = 0;
      }
      rep[i] = is_rep;
    }
    __syncthreads();
    // the top k representatives by (weighted gain, real feature index)
    for (int i = threadIdx.x; i < n; i += kVoteThreads) {
      if (!rep[i]) continue;
      const int ri = a.feat[fe[i]].real_index;
      int rank = 0;
      for (int j = 0; j < n; ++j) {
        if (j != i && rep[j] && Better(wg[j], a.feat[fe[j]].real_index, wg[i], ri)) ++rank;
      }
      if (rank < k) list[rank] = fe[i];
    }
  }
  // the global scan writes the elected features' results; every other entry is no split
  for (int f = threadIdx.x; f < nf; f += kVoteThreads) {
    FeatureBest& fb = a.feat_best[FeatBestIndex(a, side, f)];
    fb.gain = -INFINITY;
    fb.feature = -1;
  }
}

// grid (vote_k, sides): one elected feature's local histogram into vote_hist
__global__ __launch_bounds__(kVoteThreads) void k_vote_gather(KArgs a, int root) {
  const Step* st = a.st;
  if (!root && st->done) return;
  const int side = blockIdx.y, k = a.p.vote_k;
  const int f = a.vote_list[side * k + blockIdx.x];
  long long* dst = a.vote_hist + static_cast<size_t>(side * k + blockIdx.x) * 2 * a.p.max_feature_bins;
  if (f < 0) {
    for (int i = threadIdx.x; i < 2 * a.p.max_feature_bins; i += kVoteThreads) dst[i] = 0;
    return;
  }
  int slot = 0;
  if (!root) {
    const ChildInfo c = StepChildren(a, st);
    slot = StepSide(a, st, c, side).slot;
  }
  const Feature F = a.feat[f];
  const long long* src = a.hist + static_cast<size_t>(slot) * 2 * a.p.total_bins + 2 * F.hist_offset;
  const int nb2 = 2 * (F.num_bin - F.offset);
  for (int i = threadIdx.x; i < 2 * a.p.max_feature_bins; i += kVoteThreads) dst[i] = i < nb2 ? src[i] : 0;
}

// ---- round growth (KArgs::round_vote): the same election per child of the round's expansions
// (y = 2 j + lr), after the local scan of every child (k_round_find, Params::vote_phase 1).
// vote_buf holds [rank][2 round_k][vote_k] proposals, vote_list [2 round_k][vote_k] elected
// features, vote_hist their [2 round_k][vote_k][2 max_feature_bins] histograms: one allgather
// and one all-reduce per round for all of the round's leaves.
namespace {

// child y of the round: is it scanned (by the global parameters: a child the global scan skips
// proposes nothing, as k_vote_local's skipped step)
struct RoundChild {
  bool active;
  int global_rows, slot;
};

__device__ __forceinline__ RoundChild RoundVoteChild(const KArgs& a, const Round* rd, int y) {
  RoundChild c;
  c.active = false;
  c.global_rows = 0;
  c.slot = 0;
  const int j = y >> 1, lr = y & 1;
  if (rd->done || j >= rd->nexp) return c;
  const ExpPlan& E = rd->e[j];
  const int lc = E.lr[0].global_count, rc = E.lr[1].global_count, depth = E.lr[lr].depth;
  const int md = SkipMinData(a);
  c.active = !((a.p.max_depth > 0 && depth >= a.p.max_depth) || (lc < 2 * md && rc < 2 * md));
  c.global_rows = lr == 0 ? lc : rc;
  const bool is_hist = (lr == 0) == (E.hist_left != 0);
  c.slot = is_hist ? E.slot_new : E.slot_parent;
  return c;
}

}  // namespace

// grid (2 round_k): this rank's top-k features of child y by local gain -> vote_buf[rank][y]
__global__ __launch_bounds__(kVoteThreads) void k_round_vote_local(KArgs a) {
  __shared__ Cand sh[kVoteWaves];
  __shared__ int taken[64];
  const int y = blockIdx.x, k = a.p.vote_k, nf = a.p.num_features;
  const RoundChild c = RoundVoteChild(a, a.rd, y);
  if (a.rd->done) return;
  VoteEntry* out = a.vote_buf + (static_cast<size_t>(a.vote_rank) * 2 * a.round_k + y) * k;
  const FeatureBest* fb0 = a.feat_best + static_cast<size_t>(y) * nf;
  for (int r = 0; r < k; ++r) {
    Cand best;
    best.idx = -1;
    best.gain = -INFINITY;
    best.real = 0x7fffffff;
    if (c.active) {
      for (int f = threadIdx.x; f < nf; f += kVoteThreads) {
        const FeatureBest& fb = fb0[f];
        if (fb.feature < 0 || !(fb.gain > -INFINITY)) continue;
        bool dup = false;
        for (int q = 0; q < r; ++q) dup |= taken[q] == f;
        if (dup) continue;
        if (best.idx < 0 || Better(fb.gain, fb.real_feature, best.gain, best.real)) {
          best.gain = fb.gain;
          best.real = fb.real_feature;
          best.idx = f;
        }
      }
    }
    const Cand b = BlockBest(best, sh);
    if (threadIdx.x == 0) {
      VoteEntry e;
      e.gain = b.idx >= 0 ? b.gain : -INFINITY;
      e.feature = b.idx;
      e.count = 0;
      if (b.idx >= 0) e.count = fb0[b.idx].lc + fb0[b.idx].rc;
      out[r] = e;
      taken[r] = b.idx;
    }
    __syncthreads();
  }
}

// grid (2 round_k): the election of child y, then its per-feature results cleared for the
// global scan of the elected features
__global__ __launch_bounds__(kVoteThreads) void k_round_vote_elect(KArgs a) {
  __shared__ double wg[1024];
  __shared__ int fe[1024];
  __shared__ int rep[1024];
  const Round* rd = a.rd;
  if (rd->done) return;
  const int y = blockIdx.x;
  const int k = a.p.vote_k, W = a.p.world, nf = a.p.num_features;
  int32_t* list = a.vote_list + static_cast<size_t>(y) * k;
  for (int r = threadIdx.x; r < k; r += kVoteThreads) list[r] = -1;
  const RoundChild c = RoundVoteChild(a, rd, y);
  if (y >= 2 * rd->nexp) return;
  const int n = W * k;  // proposals of this child (<= 1024: checked on the host)
  if (c.active) {
    const double mean = static_cast<double>(c.global_rows) / W;
    for (int i = threadIdx.x; i < n; i += kVoteThreads) {
      const VoteEntry e = a.vote_buf[(static_cast<size_t>(i / k) * 2 * a.round_k + y) * k + (i % k)];
      const bool ok = e.feature >= 0 && e.gain > -INFINITY && mean > 0.0;
      fe[i] = ok ? e.feature : -1;
      wg[i] = ok ? e.gain * e.count / mean : -INFINITY;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += kVoteThreads) {
      int is_rep = fe[i] >= 0;
      for (int q = 0; q < n && is_rep; ++q) {
        if (q != i && fe[q] == fe[i] && (wg[q] > wg[i] || (wg[q] == wg[i] && q < i))) is_rep = 0;
      }
      rep[i] = is_rep;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += kVoteThreads) {
      if (!rep[i]) continue;
      const int ri = a.feat[fe[i]].real_index;
      int rank = 0;
      for (int q = 0; q < n; ++q) {
        if (q != i && rep[q] && Better(wg[q], a.feat[fe[q]].real_index, wg[i], ri)) ++rank;
      }
      if (rank < k) list[rank] = fe[i];
    }
  }
  FeatureBest* fb0 = a.feat_best + static_cast<size_t>(y) * nf;
  for (int f = threadIdx.x; f < nf; f += kVoteThreads) {
    fb0[f].gain = -INFINITY;
    fb0[f].feature = -1;
  }
}

// grid (vote_k, 2 round_k): one elected feature's local histogram of child y into vote_hist
// (every slot written: the all-reduce sums the whole buffer)
__global__ __launch_bounds__(kVoteThreads) void k_round_vote_gather(KArgs a) {
  const Round* rd = a.rd;
  if (rd->done) return;
  const int y = blockIdx.y, k = a.p.vote_k;
  const int f = a.vote_list[static_cast<size_t>(y) * k + blockIdx.x];
  long long* dst = a.vote_hist + static_cast<size_t>(y * k + blockIdx.x) * 2 * a.p.max_feature_bins;
  if (f < 0) {
    for (int i = threadIdx.x; i < 2 * a.p.max_feature_bins; i += kVoteThreads) dst[i] = 0;
    return;
  }
  const RoundChild c = RoundVoteChild(a, rd, y);
  const Feature F = a.feat[f];
  const long long* src = a.hist + static_cast<size_t>(c.slot) * 2 * a.p.total_bins + 2 * F.hist_offset;
  const int nb2 = 2 * (F.num_bin - F.offset);
  for (int i = threadIdx.x; i < 2 * a.p.max_feature_bins; i += kVoteThreads) dst[i] = i < nb2 ? src[i] : 0;
}

void RoundVoteLocal(const KArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_round_vote_local, dim3(2 * a.round_k), dim3(kVoteThreads), 0, s, a);
}

void RoundVoteElect(const KArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_round_vote_elect, dim3(2 * a.round_k), dim3(kVoteThreads), 0, s, a);
  hipLaunchKernelGGL(k_round_vote_gather, dim3(a.p.vote_k, 2 * a.round_k), dim3(kVoteThreads), 0, s, a);
}

void VoteLocal(const KArgs& a, hipStream_t s, bool root) {
  hipLaunchKernelGGL(k_vote_local, dim3(1), dim3(kVoteThreads), 0, s, a, root ? 1 : 0);
}

void VoteElect(const KArgs& a, hipStream_t s, bool root) {
  const int sides = root ? 1 : 2;
  hipLaunchKernelGGL(k_vote_elect, dim3(sides), dim3(kVoteThreads), 0, s, a, root ? 1 : 0);
  hipLaunchKernelGGL(k_vote_gather, dim3(a.p.vote_k, sides), dim3(kVoteThreads), 0, s, a, root ? 1 : 0);
}

}  // namespace dev
}  // namespace lgbm_amd
