// Does the instruction cache stay warm across kernel launches?  One workgroup runs a long
// straight-line body (~kOps independent v_fma, ~8 bytes each) once per launch; the body's
// in-kernel duration is timed over repeated launches (same kernel back to back), with a
// second large kernel interleaved, and cold (first launch).
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/microbench/icache tools/microbench/icache.hip
#include <hip/hip_runtime.h>

#include <cstdio>

template <int N>
__device__ __forceinline__ void Body(float& a, float& b, float& c, float& d) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a) : "v"(b), "v"(c));
    asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(d) : "v"(c), "v"(b));
  }
}

template <int N, int TAG>
__global__ void k_body(float* out, long long* t, int slot) {
  float a = out[threadIdx.x], b = 1.0001f, c = 0.9999f, d = a;
  const long long t0 = wall_clock64();
  Body<N>(a, b, c, d);
  __builtin_amdgcn_s_waitcnt(0);
  const long long t1 = wall_clock64();
  out[threadIdx.x] = a + d;
  if (threadIdx.x == 0) t[slot] = t1 - t0;
}

int main() {
  float* out = nullptr;
  long long* t = nullptr;
  hipMalloc(&out, 4096);
  hipMemset(out, 0, 4096);
  hipMalloc(&t, 64 * 8);
  constexpr int N = 512;  // 1024 v_fma ~ 8 KiB of code
  long long h[64];
  // back to back, same kernel
  for (int i = 0; i < 8; ++i) hipLaunchKernelGGL((k_body<N, 0>), dim3(1), dim3(64), 0, 0, out, t, i);
  // alternating with another 8 KiB kernel
  for (int i = 8; i < 16; i += 2) {
    hipLaunchKernelGGL((k_body<N, 0>), dim3(1), dim3(64), 0, 0, out, t, i);
    hipLaunchKernelGGL((k_body<N, 1>), dim3(1), dim3(64), 0, 0, out, t, i + 1);
  }
  // a wide grid of the same kernel (every CU runs it), then 1 workgroup
  hipLaunchKernelGGL((k_body<N, 2>), dim3(1024), dim3(64), 0, 0, out, t, 16);
  hipLaunchKernelGGL((k_body<N, 2>), dim3(1), dim3(64), 0, 0, out, t, 17);
  hipDeviceSynchronize();
  hipMemcpy(h, t, 18 * 8, hipMemcpyDeviceToHost);
  std::printf("body of %d v_fma (~%d KiB code); in-kernel us per launch:\n", 2 * N, 2 * N * 8 / 1024);
  std::printf("same kernel back to back:");
  for (int i = 0; i < 8; ++i) std::printf(" %.2f", h[i] * 0.01);
  std::printf("\nalternating A/B:        ");
  for (int i = 8; i < 16; ++i) std::printf(" %.2f", h[i] * 0.01);
  std::printf("\nafter a 1024-WG launch of the same kernel, 1 WG: %.2f\n", h[17] * 0.01);
  std::printf("(warm reference: 1024 v_fma at 1 wave ~ %.2f us at 2.4 GHz)\n", 2 * N * 4.0 / 2400.0);
  return 0;
}
