// Workgroup throughput of short, latency-bound kernels on MI355X: each workgroup runs a
// chain of `depth` dependent loads (pointer chasing in a small L2-resident table) and one
// store, like a split-scan workgroup's dependent header loads.  Kernel time vs grid size
// and workgroup size separates dispatch cost from the chain's latency.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench/wg_throughput tools/microbench/wg_throughput.hip
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

__global__ void k_chain(const int* next, int depth, int* out, int with_sync) {
  int p = (blockIdx.x * 7) & 1023;
  for (int i = 0; i < depth; ++i) p = next[p + threadIdx.x % 4];  // dependent loads
  if (with_sync) __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = p;
}

__global__ void k_chain_fence(const int* next, int depth, int* out, unsigned* counter) {
  int p = (blockIdx.x * 7) & 1023;
  for (int i = 0; i < depth; ++i) p = next[p + threadIdx.x % 4];
  if (threadIdx.x == 0) {
    out[blockIdx.x] = p;
    __threadfence();
    atomicAdd(counter, 1u);
  }
}

// mode 0: fence only, 1: atomic only, 2: fence + atomic on one of 32 counters
__global__ void k_chain_part(const int* next, int depth, int* out, unsigned* counter, int mode) {
  int p = (blockIdx.x * 7) & 1023;
  for (int i = 0; i < depth; ++i) p = next[p + threadIdx.x % 4];
  if (threadIdx.x == 0) {
    out[blockIdx.x] = p;
    if (mode != 1) __threadfence();
    if (mode == 1) atomicAdd(counter, 1u);
    if (mode == 2) atomicAdd(counter + 16 * (blockIdx.x % 32), 1u);
  }
}

int main() {
  std::vector<int> h(2048);
  for (int i = 0; i < 2048; ++i) h[i] = (i * 37 + 11) & 1023;
  int *d_next = nullptr, *d_out = nullptr;
  unsigned* d_cnt = nullptr;
  CK(hipMalloc(&d_next, sizeof(int) * 2048));
  CK(hipMalloc(&d_out, sizeof(int) * 65536));
  CK(hipMalloc(&d_cnt, sizeof(unsigned) * 1024));
  CK(hipMemcpy(d_next, h.data(), sizeof(int) * 2048, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::printf("kernel        block  depth   grid   us/launch  ns/workgroup\n");
  for (int variant = 0; variant < 6; ++variant) {
    for (int block : {64}) {
      for (int depth : {1}) {
        for (int grid : {56, 256, 1024, 4000, 16000}) {
          auto launch = [&] {
            if (variant >= 3) hipLaunchKernelGGL(k_chain_part, dim3(grid), dim3(block), 0, 0, d_next, depth, d_out, d_cnt, variant - 3);
            else if (variant == 2) hipLaunchKernelGGL(k_chain_fence, dim3(grid), dim3(block), 0, 0, d_next, depth, d_out, d_cnt);
            else hipLaunchKernelGGL(k_chain, dim3(grid), dim3(block), 0, 0, d_next, depth, d_out, variant);
          };
          launch();
          CK(hipDeviceSynchronize());
          const int reps = 50;
          CK(hipEventRecord(e0));
          for (int r = 0; r < reps; ++r) launch();
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          const double us = 1000.0 * ms / reps;
          const char* names[] = {"chain", "chain+sync", "chain+fence+atomic", "chain+fence", "chain+atomic", "fence+32 counters"};
          const char* name = names[variant];
          std::printf("%-19s %4d %6d %6d %10.2f %10.1f\n", name, block, depth, grid, us, 1000.0 * us / grid);
        }
      }
    }
  }
  return 0;
}
