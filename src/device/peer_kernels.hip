// One-shot peer collectives over symmetric windows (kernels.h PeerArgs; host side
// src/network/peer_comm.cpp).
//
// The reference moves histograms between machines with host-side reduce-scatter / allgather
// over sockets (src/network/network.cpp:232-318, linkers_socket.cpp).  On one MI355X node the
// peers' HBM is directly addressable over xGMI, so a collective here is a single kernel per
// rank that reads the peers' inputs where they lie: no host rendezvous, no proxy thread, no
// ring of steps -- every rank pulls its share from all peers at once (one-shot), which is what
// the per-round histogram reduce-scatter and split-record allgather (kilobytes to a few MB)
// want on point-to-point links.  Being plain kernels, they are captured in the learner's graphs.
//
// Synchronisation (per collective, epoch e = previous + 1, identical on every rank):
//   1. wait until every peer published departure e - 1 (it finished reading this stage);
//   2. copy the input into the own stage; each workgroup releases its writes at system scope
//      and counts itself; the last one publishes arrival e into every peer's flags;
//   3. wait for arrival e of every rank (own included: the whole stage is written), acquire;
//   4. read the peers' stages (reduce in rank order: bit-identical results on every rank);
//   5. the last workgroup to finish publishes departure e into every peer's flags.
// Windows are uncached device memory (hipDeviceMallocUncached), so neither the flags nor the
// staged data can be served from a stale L2 line on either side of the link.  Every wait is
// bounded by a 100 MHz wall-clock deadline and polls the host's abort word: a rank that stops
// leaves its peers with a status code, never a hung queue.
#include "device_common.h"

namespace lgbm_amd {
namespace dev {

namespace {

typedef __attribute__((address_space(1))) unsigned long long PGU64;
typedef __attribute__((address_space(1))) unsigned int PGU32;

__device__ __forceinline__ unsigned long long LoadSys(const unsigned long long* p) {
  return __hip_atomic_load((PGU64*)(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void StoreSys(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store((PGU64*)(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned long long* PeerFlag(char* win, int which, int p) {
  return reinterpret_cast<unsigned long long*>(win) + which * kMaxPeerBufs + p;
}

// a wait failed: the comm is dead on this rank (later collectives exit at once); the first
// error's code and epoch go to the host-mapped status words
__device__ bool PeerFail(const PeerArgs& a, unsigned code, unsigned long long epoch) {
  __hip_atomic_store((PGU64*)(a.ctl + 3), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned expect = 0;
  if (__hip_atomic_compare_exchange_strong((PGU32*)(a.status), &expect, code, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM)) {
    __hip_atomic_store((PGU32*)(a.status + 2), static_cast<unsigned>(epoch), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  return false;
}

// (one thread) every rank's flags[which][p] >= v, p != skip_p; false on timeout / abort /
// another workgroup's failure
__device__ bool PeerWaitAll(const PeerArgs& a, int which, unsigned long long v, int skip_p, long long t0) {
  char* mine = a.win[a.rank];
  for (int p = 0; p < a.n; ++p) {
    if (p == skip_p) continue;
    const unsigned long long* f = PeerFlag(mine, which, p);
    int it = 0;
    while (LoadSys(f) < v) {
      if ((++it & 31) == 0) {
        if (__hip_atomic_load((PGU32*)(a.status + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) {
          return PeerFail(a, kPeerAborted, v);
        }
        if (__hip_atomic_load((PGU64*)(a.ctl + 3), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0ull) return false;
        if (static_cast<long long>(wall_clock64()) - t0 > a.timeout_ticks) return PeerFail(a, kPeerTimeout, v);
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  return true;
}

template <typename T, int OP>
__device__ __forceinline__ T PeerOpApply(T a, T b) {
  if constexpr (OP == 3) {
    return b > a ? b : a;
  } else {
    return a + b;
  }
}

// grid-strided copy with four independent loads in flight per thread (uncached windows: each
// access is a full memory round trip)
template <typename T>
__device__ __forceinline__ void PeerCopy(T* dst, const T* src, size_t cnt, size_t tid, size_t nth) {
  size_t i = tid;
  for (; i + 3 * nth < cnt; i += 4 * nth) {
    const T v0 = src[i], v1 = src[i + nth], v2 = src[i + 2 * nth], v3 = src[i + 3 * nth];
    dst[i] = v0;
    dst[i + nth] = v1;
    dst[i + 2 * nth] = v2;
    dst[i + 3 * nth] = v3;
  }
  for (; i < cnt; i += nth) dst[i] = src[i];
}

// OP: 0 sum, 3 max (reductions: allreduce / reduce-scatter); -1 copy (allgather / broadcast)
template <typename T, int OP>
__global__ __launch_bounds__(256) void k_peer_collective(PeerArgs a) {
  __shared__ int s_go;
  __shared__ unsigned long long s_epoch;
  __shared__ long long s_t0;
  const int kind = a.kind;
  const bool writes_stage = kind != kPeerBroadcast || a.rank == a.root;
  if (threadIdx.x == 0) {
    int go = 1;
    unsigned long long ep = 0;
    const long long t0 = static_cast<long long>(wall_clock64());
    if (a.guard != nullptr && *a.guard != 0) go = 0;  // replicated state: skipped on every rank
    if (go && __hip_atomic_load((PGU64*)(a.ctl + 3), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0ull) go = 0;
    if (go) {
      ep = a.ctl[0] + 1;
      if (a.fail_epoch > 0 && ep == static_cast<unsigned long long>(a.fail_epoch)) {
        if (blockIdx.x == 0) PeerFail(a, kPeerInjected, ep);
        go = 0;
      }
    }
    if (go && writes_stage && ep > 1) go = PeerWaitAll(a, 1, ep - 1, a.rank, t0) ? 1 : 0;
    s_go = go;
    s_epoch = ep;
    s_t0 = t0;
  }
  __syncthreads();
  if (!s_go) return;
  const unsigned long long ep = s_epoch;
  const size_t tid = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const size_t nth = static_cast<size_t>(gridDim.x) * blockDim.x;
  const T* send = reinterpret_cast<const T*>(a.send);
  T* recv = reinterpret_cast<T*>(a.recv);
  const size_t cnt = a.count;
  // 2. the own input -> the own stage (reduce-scatter: the blocks the peers read)
  if (writes_stage) {
    T* stage = reinterpret_cast<T*>(a.win[a.rank] + kPeerFlagBytes);
    if (kind == kPeerReduceScatter) {
      for (int p = 0; p < a.n; ++p) {
        if (p == a.rank) continue;
        PeerCopy(stage + static_cast<size_t>(p) * cnt, send + static_cast<size_t>(p) * a.stride + a.off, cnt, tid, nth);
      }
    } else {
      PeerCopy(stage, send + a.off, cnt, tid, nth);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // (stage stores complete and visible to the peers)
    const unsigned long long old = __hip_atomic_fetch_add((PGU64*)(a.ctl + 1), 1ull, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1) {
      __hip_atomic_store((PGU64*)(a.ctl + 1), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      for (int p = 0; p < a.n; ++p) StoreSys(PeerFlag(a.win[p], 0, a.rank), ep);
    }
    // 3. every rank's stage is complete
    s_go = PeerWaitAll(a, 0, ep, -1, s_t0) ? 1 : 0;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  if (!s_go) return;
  // 4. read the peers' stages where they lie
  if constexpr (OP >= 0) {
    const size_t own_off = kind == kPeerReduceScatter ? static_cast<size_t>(a.rank) * a.stride + a.off : a.off;
    const size_t peer_off = kind == kPeerReduceScatter ? static_cast<size_t>(a.rank) * cnt : 0;
    // two elements per pass: 2 x n independent loads in flight
    for (size_t i = tid; i < cnt; i += 2 * nth) {
      const bool two = i + nth < cnt;
      T v0{}, v1{};
      for (int p = 0; p < a.n; ++p) {
        const T* src = p == a.rank ? send + own_off : reinterpret_cast<const T*>(a.win[p] + kPeerFlagBytes) + peer_off;
        const T x0 = src[i];
        const T x1 = two ? src[i + nth] : T{};
        v0 = p == 0 ? x0 : PeerOpApply<T, OP>(v0, x0);
        v1 = p == 0 ? x1 : PeerOpApply<T, OP>(v1, x1);
      }
      recv[a.off + i] = v0;
      if (two) recv[a.off + i + nth] = v1;
    }
  } else if (kind == kPeerAllgather) {
    for (int p = 0; p < a.n; ++p) {
      const T* src = p == a.rank ? send + a.off : reinterpret_cast<const T*>(a.win[p] + kPeerFlagBytes);
      T* dst = recv + static_cast<size_t>(p) * a.stride + a.off;
      if (p == a.rank && src == dst) continue;  // (in place)
      PeerCopy(dst, src, cnt, tid, nth);
    }
  } else if (a.rank != a.root) {
    PeerCopy(recv + a.off, reinterpret_cast<const T*>(a.win[a.root] + kPeerFlagBytes), cnt, tid, nth);
  }
  // 5. departure: the peers may overwrite their stages once every rank has read them
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // (the reads above have completed)
    const unsigned long long old = __hip_atomic_fetch_add((PGU64*)(a.ctl + 2), 1ull, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1) {
      __hip_atomic_store((PGU64*)(a.ctl + 2), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store((PGU64*)(a.ctl + 0), ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      for (int p = 0; p < a.n; ++p) StoreSys(PeerFlag(a.win[p], 1, a.rank), ep);
    }
  }
}

template <typename T, int OP>
void LaunchPeer(const PeerArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((k_peer_collective<T, OP>), dim3(grid), dim3(256), 0, s, a);
}

}  // namespace

void PeerCollective(const PeerArgs& a, hipStream_t s) {
  // bytes this rank reads: ~16 KB per workgroup (uncached accesses are latency-bound: many
  // workgroups in flight), at most 128 (more only lengthens the arrival / departure counts)
  const size_t blocks = a.kind == kPeerAllgather ? static_cast<size_t>(a.n) : 1;
  const size_t bytes = a.count * static_cast<size_t>(a.elem) *
                       (a.kind == kPeerAllgather ? blocks : static_cast<size_t>(a.kind == kPeerBroadcast ? 1 : a.n));
  // Every workgroup's first thread waits for the peers' arrival, which this rank publishes only
  // once ALL its workgroups have staged their share: the grid must be co-resident.  It is
  // capped at half of what the device holds at once, shared by up to a.n ranks on one device
  // (thread ranks), so other kernels in flight cannot starve the last workgroups.
  static const int resident = [] {
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_peer_collective<double, 0>, 256, 0) != hipSuccess) {
      (void)hipGetLastError();
      b = 4;
    }
    return std::max(1, b) * NumCUs();
  }();
  const size_t cap = std::max<size_t>(1, static_cast<size_t>(resident) / (2 * static_cast<size_t>(std::max(1, a.n))));
  const int grid = static_cast<int>(std::max<size_t>(1, std::min<size_t>(std::min<size_t>(128, cap), (bytes + 16383) / 16384)));
  if (a.kind == kPeerAllreduce || a.kind == kPeerReduceScatter) {
    switch (a.op) {
      case kPeerSumF64: LaunchPeer<double, 0>(a, grid, s); break;
      case kPeerSumF32: LaunchPeer<float, 0>(a, grid, s); break;
      case kPeerSumI64: LaunchPeer<long long, 0>(a, grid, s); break;
      default: LaunchPeer<uint32_t, 3>(a, grid, s); break;
    }
    return;
  }
  switch (a.elem) {
    case 16: LaunchPeer<uint4, -1>(a, grid, s); break;
    case 4: LaunchPeer<uint32_t, -1>(a, grid, s); break;
    default: LaunchPeer<uint8_t, -1>(a, grid, s); break;
  }
}

}  // namespace dev
}  // namespace lgbm_amd
