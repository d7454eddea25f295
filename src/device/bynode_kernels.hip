// Per-node column sampling under interaction constraints, on the device (reference
// src/treelearner/col_sampler.hpp:91-162 GetByNode; host src/treelearner/col_sampler.h).
//
// Without interaction constraints every GetByNode call samples from the same pool, so the host
// draws a tree's worth of node masks up front.  With them the pool is the tree's used features
// that the node's branch allows -- known only once the node exists -- and Random::Sample's
// consumption of the generator depends on the pool size.  So after each step's partition
// k_bynode_step draws the two children's masks in the host learner's order (smaller child,
// then larger) from a device-resident generator state: the filtered pool in the tree-level
// order, K = min(GetCnt(pool, fraction_bynode), filtered size), and Sample(N, K) -- the
// Bernoulli pass when K > N / log2(K), else the Floyd set walk -- exactly as the host.  The
// root's mask and the state after it come from the host; the host generator takes the final
// state after the tree.
#include "device_common.h"
#include "lgbm_amd/random.h"

namespace lgbm_amd {
namespace dev {

namespace {

constexpr int kByNodeThreads = 256;

// one child's mask row (thread 0 samples; the workgroup clears the row first)
__device__ void ByNodeRow(const KArgs& a, IcMask icm, int8_t* row, Random* rng) {
  const int NF = a.p.num_features;
  for (int f = threadIdx.x; f < NF; f += kByNodeThreads) row[f] = 0;
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t* pool = a.bynode_scratch;
    int n = 0;
    for (int i = 0; i < a.bynode_pool_n; ++i) {
      const int f = a.bynode_pool[i];
      if (IcAny(a.feat_icmask[f] & icm)) pool[n++] = f;
    }
    const int k = min(a.bynode_cnt, n);
    if (k > 0 && k <= n) {
      if (k == n) {
        for (int i = 0; i < n; ++i) row[pool[i]] = 1;
      } else if (k > 1 && static_cast<double>(k) > static_cast<double>(n) / log2(static_cast<double>(k))) {
        int taken = 0;
        for (int i = 0; i < n; ++i) {
          const double prob = (k - static_cast<double>(taken)) / static_cast<double>(n - i);
          if (rng->NextFloat() < prob) {
            row[pool[i]] = 1;
            ++taken;
          }
        }
      } else {
        // Floyd: v in [0, r), or r itself when v is taken (r is never taken before its turn);
        // "taken" is the mask row of the pool position's feature (pool features are distinct)
        for (int r = n - k; r < n; ++r) {
          const int v = rng->NextInt(0, r);
          if (row[pool[v]]) row[pool[r]] = 1;
          else row[pool[v]] = 1;
        }
      }
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(kByNodeThreads) void k_bynode_step(KArgs a) {
  const Step* st = a.st;
  if (st->done) return;
  const ChildInfo c = StepChildren(a, st);
  if (c.skip) return;  // no scan of the children: the host learner samples nothing either
  const int mi = st->bynode_next;  // the rows this step's split scans read (advanced by the pick)
  const IcMask icm = st->lr[0].icmask;  // (both children keep the same constraints)
  Random rng(static_cast<int>(*a.bynode_rng));
  for (int side = 0; side < 2; ++side) {
    ByNodeRow(a, icm, const_cast<int8_t*>(a.node_mask) + static_cast<size_t>(mi + side) * a.p.num_features, &rng);
  }
  if (threadIdx.x == 0) *a.bynode_rng = rng.state();
}

}  // namespace

void ByNodeStep(const KArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_bynode_step, dim3(1), dim3(kByNodeThreads), 0, s, a);
}

}  // namespace dev
}  // namespace lgbm_amd
