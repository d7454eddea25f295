// LDS atomic throughput on MI355X: f32 / f64 / u32 / u64 adds to pseudo-random addresses in a
// 56 KiB region (the histogram working set), 2 blocks of 256 threads per CU.
//   hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics lds_atomics.hip -o lds_atomics
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kWords = 14336;  // 56 KiB of 4-byte words
constexpr int kIters = 4096;

template <typename T, int MODE>  // MODE 0 random, 1 same-feature-region random (256 words), 2 conflict-free
__global__ __launch_bounds__(256) void k_atomics(void* outp, int seed) {
  T* out = static_cast<T*>(outp);
  __shared__ T lds[kWords * 4 / sizeof(T)];
  constexpr int n = kWords * 4 / sizeof(T);
  for (int i = threadIdx.x; i < n; i += 256) lds[i] = T(0);
  __syncthreads();
  uint32_t s = seed ^ (threadIdx.x * 2654435761u) ^ (blockIdx.x * 40503u);
  T v = T(1);
  for (int it = 0; it < kIters; ++it) {
    s = s * 1664525u + 1013904223u;
    int a;
    if (MODE == 0) a = (s >> 8) % n;
    else if (MODE == 1) a = ((it % 28) * 256 + ((s >> 8) & 255)) % n;
    else a = (threadIdx.x + it * 256) % n;
    atomicAdd(&lds[a], v);
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = lds[seed % n];
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int grid = 2 * cus;
  void* out;
  hipMalloc(&out, grid * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* name, auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, out, 7);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, out, 7 + r);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double ops = 5.0 * grid * 256.0 * kIters;
    printf("%-34s %8.3f ms  %8.1f G lane-atomics/s  %.3f per CU-cycle@2.4GHz\n", name, ms, ops / ms / 1e6,
           ops / (ms * 1e-3) / cus / 2.4e9);
  };
  run("f32 random", k_atomics<float, 0>);
  run("f32 feature-region", k_atomics<float, 1>);
  run("f32 conflict-free", k_atomics<float, 2>);
  run("f64 random", k_atomics<double, 0>);
  run("f64 conflict-free", k_atomics<double, 2>);
  run("u32 random", k_atomics<unsigned int, 0>);
  run("u32 conflict-free", k_atomics<unsigned int, 2>);
  run("u64 random", k_atomics<unsigned long long, 0>);
  run("u64 conflict-free", k_atomics<unsigned long long, 2>);
  run("i32 random", k_atomics<int, 0>);
  return 0;
}
