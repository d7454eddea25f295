// Cost and correctness of a persistent-kernel grid barrier (grid_sync.h, an experiment):
// one 1024-thread workgroup per CU, barriers back to back.  Correctness: before each barrier
// every workgroup writes an iteration-dependent pattern with plain stores; after it, every
// workgroup reads another workgroup's pattern (usually another XCD's) and counts stale
// values -- this exercises the per-XCD L2 writeback / invalidate scheme.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/microbench/grid_barrier tools/microbench/grid_barrier.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#include "grid_sync.h"

using namespace lgbm_amd::dev;

template <int MODE>
__global__ __launch_bounds__(1024) void k_bar(GridBar* b, unsigned* data, unsigned* bad, int iters, long long* out,
                                              int check, int* xcc_out) {
  extern __shared__ int lds[];
  __shared__ BarCtx ctx;
  if (!GridSyncInit(b, &ctx)) return;
  if (threadIdx.x == 0) xcc_out[blockIdx.x] = ctx.xcc;
  const int nb = gridDim.x;
  const int peer = (blockIdx.x + 37) % nb;
  const long long t0 = wall_clock64();
  for (int i = 0; i < iters; ++i) {
    if (check) data[blockIdx.x * 1024 + threadIdx.x] = i * 4096u + blockIdx.x;
    if (!GridSync<MODE>(b, &ctx)) return;
    if (check) {
      const unsigned v = data[peer * 1024 + threadIdx.x];
      if (v != i * 4096u + peer) atomicAdd(bad, 1u);
      if (!GridSync<MODE>(b, &ctx)) return;  // the next writes must not overtake this read
    }
  }
  lds[threadIdx.x] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) out[0] = wall_clock64() - t0;
}

int main() {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const size_t lds = 80 * 1024;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_bar<0>), hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_bar<1>), hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  int occ = 0;
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_bar<0>, 1024, lds);
  std::printf("CUs %d, resident 1024-thread workgroups per CU at 80 KiB LDS: %d\n", cus, occ);
  if (occ < 1) return 1;
  GridBar* b = nullptr;
  unsigned *data = nullptr, *bad = nullptr;
  long long* out = nullptr;
  int* xcc = nullptr;
  (void)hipMalloc(&b, sizeof(GridBar));
  (void)hipMalloc(&data, sizeof(unsigned) * 1024 * cus);
  (void)hipMalloc(&bad, 8);
  (void)hipMalloc(&out, 8);
  (void)hipMalloc(&xcc, sizeof(int) * cus);
  for (int mode : {0, 1})
  for (int grid : {cus, 64}) {
    for (int check : {1, 0}) {
      const int iters = 2000;
      (void)hipMemset(b, 0, sizeof(GridBar));
      (void)hipMemset(bad, 0, 8);
      (void)hipMemset(data, 0xff, sizeof(unsigned) * 1024 * cus);
      if (mode == 0) hipLaunchKernelGGL(k_bar<0>, dim3(grid), dim3(1024), lds, 0, b, data, bad, iters, out, check, xcc);
      else hipLaunchKernelGGL(k_bar<1>, dim3(grid), dim3(1024), lds, 0, b, data, bad, iters, out, check, xcc);
      if (hipDeviceSynchronize() != hipSuccess) {
        std::printf("kernel failed\n");
        return 1;
      }
      long long t = 0;
      unsigned nbad = 0, err = 0;
      (void)hipMemcpy(&t, out, 8, hipMemcpyDeviceToHost);
      (void)hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost);
      (void)hipMemcpy(&err, &b->err.v, 4, hipMemcpyDeviceToHost);
      std::printf("%s grid %3d x 1024: %d iterations%s: %.2f us per barrier; stale reads %u; timeout %u\n",
                  mode ? "full fences " : "per-XCD     ", grid, iters,
                  check ? " (write, barrier, read peer, barrier)" : " (barriers only)",
                  t * 0.01 / (iters * (check ? 2 : 1)), nbad, err);
    }
  }
  int h[512];
  (void)hipMemcpy(h, xcc, sizeof(int) * 16, hipMemcpyDeviceToHost);
  std::printf("XCC of workgroups 0..15 (last run):");
  for (int i = 0; i < 16; ++i) std::printf(" %d", h[i]);
  std::printf("\n");
  return 0;
}
