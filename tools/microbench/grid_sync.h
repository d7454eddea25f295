// Grid-wide barrier experiment for a persistent per-tree kernel (measured, NOT used by the
// learner -- see profiles/r02_grid_barrier.txt).  Every workgroup must be resident at once.
//
// MI355X has one L2 per XCD; cross-XCD visibility of plain stores needs agent-scope
// writeback / invalidate.  Measured on 256 x 1024-thread workgroups (one per CU):
//   * counters only, no fences: 1.9 us per barrier (two-level) / 3.7 us (flat);
//   * MODE 0 below -- the last arrival of each XCD group writes the XCD's L2 back and
//     invalidates it after the release, the others drop their L1: ~2.9 us, but 72% of the
//     reads of another workgroup's plain stores were STALE: incorrect;
//   * MODE 1 -- agent-scope fences in every thread: correct (0 stale reads) but 64 us.
// With 2-3 barriers per split a persistent tree kernel would not beat the kernel-boundary
// synchronisation of the graph-launched step kernels (~1.6 us per launch), so the learner
// keeps those.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace lgbm_amd {
namespace dev {

constexpr int kMaxXcc = 16;
constexpr unsigned kBarSpinLimit = 1u << 22;  // ~1 s of polling

// one 128-byte line per counter
struct alignas(128) BarLine {
  unsigned v;
  unsigned pad[31];
};
struct GridBar {
  BarLine reg[kMaxXcc];        // workgroups per XCC (registration)
  BarLine group[kMaxXcc];      // arrivals per XCC group
  BarLine group_gen[kMaxXcc];  // per-group release generation
  BarLine init_count, init_gen;
  BarLine top;                 // groups arrived
  BarLine gen;                 // global release generation
  BarLine err;
};

// per-workgroup barrier state (thread 0's registers / LDS)
struct BarCtx {
  unsigned gen;
  int xcc, gsize, ngroups;
};

__device__ __forceinline__ unsigned BarLoad(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int HwXccId() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return static_cast<int>(x & (kMaxXcc - 1));
}

__device__ __forceinline__ bool BarWait(GridBar* b, const unsigned* p, unsigned target) {
  unsigned spins = 0;
  while (BarLoad(p) != target) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > kBarSpinLimit) {
      atomicExch(&b->err.v, 1u);
      return false;
    }
  }
  return true;
}

// registration (every thread calls it once, first thing in the kernel); false on timeout
__device__ __forceinline__ bool GridSyncInit(GridBar* b, BarCtx* ctx) {
  __shared__ int s_ok;
  __syncthreads();
  if (threadIdx.x == 0) {
    ctx->gen = 0;
    ctx->xcc = HwXccId();
    atomicAdd(&b->reg[ctx->xcc].v, 1u);
    __threadfence();
    if (atomicAdd(&b->init_count.v, 1u) == gridDim.x - 1) atomicExch(&b->init_gen.v, 1u);
    int ok = BarWait(b, &b->init_gen.v, 1u) ? 1 : 0;
    __threadfence();
    ctx->gsize = static_cast<int>(BarLoad(&b->reg[ctx->xcc].v));
    int ng = 0;
    for (int x = 0; x < kMaxXcc; ++x) ng += BarLoad(&b->reg[x].v) != 0u ? 1 : 0;
    ctx->ngroups = ng;
    s_ok = ok;
  }
  __syncthreads();
  return s_ok != 0;
}

// every thread of every workgroup calls it; false if this or an earlier barrier timed out
// (then every workgroup should leave the kernel)
template <int MODE = 0>
__device__ __forceinline__ bool GridSync(GridBar* b, BarCtx* ctx) {
  __shared__ int s_ok;
  // every wave's stores have reached its XCD's L2 before the group counts this workgroup
  // (a workgroup-scope barrier alone does not wait for them: the CU's L1 is write-through)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (MODE == 1) __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned target = ++ctx->gen;
    const int x = ctx->xcc;
    int ok = BarLoad(&b->err.v) == 0u ? 1 : 0;
    if (atomicAdd(&b->group[x].v, 1u) == static_cast<unsigned>(ctx->gsize - 1)) {
      atomicExch(&b->group[x].v, 0u);  // nobody arrives here again before the release
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // the XCD's writes to memory (buffer_wbl2)
      if (atomicAdd(&b->top.v, 1u) == static_cast<unsigned>(ctx->ngroups - 1)) {
        atomicExch(&b->top.v, 0u);
        atomicExch(&b->gen.v, target);
      }
      if (!BarWait(b, &b->gen.v, target)) ok = 0;
      asm volatile("buffer_inv sc1" ::: "memory");  // drop the XCD's stale L2 (and this CU's L1) lines
      atomicExch(&b->group_gen[x].v, target);
    } else {
      if (!BarWait(b, &b->group_gen[x].v, target)) ok = 0;
      asm volatile("buffer_inv sc0" ::: "memory");  // drop this CU's stale L1 lines
    }
    if (MODE == 1) __threadfence();
    s_ok = ok;
  }
  __syncthreads();
  return s_ok != 0;
}

}  // namespace dev
}  // namespace lgbm_amd
