// Latency of the dependent global accesses a tree step is made of, on one MI355X:
//  * loads of words the PREVIOUS kernel wrote (from many workgroups, so from every XCD),
//    chained so each address depends on the previous value, across
//      - one allocation, 64-byte stride (same pages),
//      - one allocation, 64 KiB stride, and 2 MiB stride,
//      - 16 separate small allocations (separate pages / TLB entries);
//  * device-scope atomicAdd with return, chained;
//  * __threadfence() back to back, and a fence followed by a dependent load.
// One thread times its chain with wall_clock64 (100 MHz); result in ns per access.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/microbench/mem_latency tools/microbench/mem_latency.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

constexpr int kChain = 16;

struct Ptrs {
  int* p[kChain];
};

// chain links: word at element offset off[i] of buffer i holds off[i + 1]; written by a grid of
// 512 workgroups (link i by workgroup 32 * i) so the lines are dirty in different XCDs' L2
__global__ void k_write(Ptrs b, Ptrs dummy, int stride_elems, int salt) {
  const int i = blockIdx.x / 32;
  if (i >= kChain || blockIdx.x % 32 != 0 || threadIdx.x != 0) return;
  const int off = i * stride_elems;
  const int next = (i + 1) * stride_elems;
  b.p[i][off] = next + salt * 0;
  (void)dummy;
}

__global__ void k_chase(Ptrs b, long long* out, int salt) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int x = 0;
  const long long t0 = wall_clock64();
#pragma unroll 1
  for (int i = 0; i < kChain; ++i) x = b.p[i][x] + salt;  // address depends on the previous load
  const long long t1 = wall_clock64();
  out[0] = t1 - t0;
  out[1] = x;
}

__global__ void k_atomic_chain(int* p, long long* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int x = 0;
  const long long t0 = wall_clock64();
#pragma unroll 1
  for (int i = 0; i < kChain; ++i) x = atomicAdd(p + (x & 1) * 16, 1) & 0;
  const long long t1 = wall_clock64();
  out[0] = t1 - t0;
  out[1] = x;
}

__global__ void k_fence_chain(int* p, long long* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const long long t0 = wall_clock64();
#pragma unroll 1
  for (int i = 0; i < kChain; ++i) __threadfence();
  const long long t1 = wall_clock64();
  int x = 0;
#pragma unroll 1
  for (int i = 0; i < kChain; ++i) {
    __threadfence();
    x = p[64 + x * 16];  // a load right after an acquire fence
  }
  const long long t2 = wall_clock64();
  out[0] = t1 - t0;
  out[1] = t2 - t1;
  out[2] = x;
}

// store completion: a plain store then s_waitcnt vmcnt(0), 16 times (the wait a barrier or
// fence after stores pays); variants: the line was just read (L2 hit), fresh line each time
__global__ void k_store_chain(int* p, long long* out, int stride) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const long long t0 = wall_clock64();
#pragma unroll 1
  for (int i = 0; i < kChain; ++i) {
    p[i * stride] = i;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  const long long t1 = wall_clock64();
  out[0] = t1 - t0;
}
// 64 lanes store, then one barrier (s_waitcnt + s_barrier), 16 times
__global__ void k_store_barrier(int* p, long long* out) {
  const long long t0 = wall_clock64();
#pragma unroll 1
  for (int i = 0; i < kChain; ++i) {
    p[i * 4096 + threadIdx.x] = i;
    __syncthreads();
  }
  const long long t1 = wall_clock64();
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = t1 - t0;
}

int main() {
  long long* d_out = nullptr;
  CK(hipMalloc(&d_out, 64));
  // variants of the chained buffers
  const size_t big_bytes = size_t(kChain + 1) * (2u << 20);
  int* big = nullptr;
  CK(hipMalloc(&big, big_bytes));
  CK(hipMemset(big, 0, big_bytes));
  std::vector<int*> small(kChain);
  for (int i = 0; i < kChain; ++i) {
    CK(hipMalloc(&small[i], 4096));
    CK(hipMemset(small[i], 0, 4096));
    // interleave other allocations so the small buffers do not sit on one page
    int* pad = nullptr;
    CK(hipMalloc(&pad, 3 << 20));
  }
  struct V {
    const char* name;
    Ptrs p;
    int stride;  // elements between links (offsets are taken relative to each buffer base)
  };
  std::vector<V> vs;
  for (int s : {16, 16384, 524288}) {  // 64 B, 64 KiB, 2 MiB
    V v;
    v.name = s == 16 ? "one alloc, 64 B stride" : (s == 16384 ? "one alloc, 64 KiB stride" : "one alloc, 2 MiB stride");
    for (int i = 0; i < kChain; ++i) v.p.p[i] = big;  // same base: offsets i * stride
    v.stride = s;
    vs.push_back(v);
  }
  {
    V v;
    v.name = "16 separate allocations";
    for (int i = 0; i < kChain; ++i) v.p.p[i] = small[i] - i * 16;  // link i at element 16 * i of small[i]
    v.stride = 16;
    vs.push_back(v);
  }
  long long h[4];
  for (const V& v : vs) {
    double best = 1e30, sum = 0;
    const int reps = 20;
    for (int r = 0; r < reps; ++r) {
      hipLaunchKernelGGL(k_write, dim3(512), dim3(64), 0, 0, v.p, v.p, v.stride, r);
      hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, 0, v.p, d_out, 0);
      CK(hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost));
      const double ns = h[0] * 10.0 / kChain;
      best = std::min(best, ns);
      sum += ns;
    }
    std::printf("%-34s fresh-written dependent load: %7.0f ns (best %6.0f)\n", v.name, sum / reps, best);
    // warm: chase twice in the same kernel sequence (second run hits caches / TLB)
    hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, 0, v.p, d_out, 0);
    hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, 0, v.p, d_out, 0);
    CK(hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost));
    std::printf("%-34s re-read (previous kernel read it):  %7.0f ns\n", v.name, h[0] * 10.0 / kChain);
  }
  for (int stride : {0, 16, 16384}) {
    hipLaunchKernelGGL(k_store_chain, dim3(1), dim3(64), 0, 0, big, d_out, stride);
    hipLaunchKernelGGL(k_store_chain, dim3(1), dim3(64), 0, 0, big, d_out, stride);
    CK(hipMemcpy(h, d_out, 8, hipMemcpyDeviceToHost));
    std::printf("store + s_waitcnt vmcnt(0), stride %6d elems: %7.0f ns each\n", stride, h[0] * 10.0 / kChain);
  }
  hipLaunchKernelGGL(k_store_barrier, dim3(1), dim3(256), 0, 0, big, d_out);
  hipLaunchKernelGGL(k_store_barrier, dim3(1), dim3(256), 0, 0, big, d_out);
  CK(hipMemcpy(h, d_out, 8, hipMemcpyDeviceToHost));
  std::printf("256 threads store, __syncthreads: %7.0f ns each\n", h[0] * 10.0 / kChain);
  for (int r = 0; r < 3; ++r) {
    hipLaunchKernelGGL(k_atomic_chain, dim3(1), dim3(64), 0, 0, big, d_out);
    CK(hipMemcpy(h, d_out, 16, hipMemcpyDeviceToHost));
    std::printf("device-scope atomicAdd with return, chained: %7.0f ns\n", h[0] * 10.0 / kChain);
  }
  for (int r = 0; r < 3; ++r) {
    hipLaunchKernelGGL(k_write, dim3(512), dim3(64), 0, 0, vs[0].p, vs[0].p, 16, r);
    hipLaunchKernelGGL(k_fence_chain, dim3(1), dim3(64), 0, 0, big, d_out);
    CK(hipMemcpy(h, d_out, 24, hipMemcpyDeviceToHost));
    std::printf("__threadfence(): %6.0f ns each; fence + dependent load: %6.0f ns\n", h[0] * 10.0 / kChain,
                h[1] * 10.0 / kChain);
  }
  return 0;
}
