// Back-to-back dependent kernel cost on one stream: empty kernels of several grid shapes
// and kernel-argument sizes, eager vs hipGraph replay.  Build:
//   hipcc --offload-arch=gfx950 -O2 -o tools/microbench/launch_overhead tools/microbench/launch_overhead.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);     \
      return 1;                                                                \
    }                                                                          \
  } while (0)

struct Big {
  int v[96];  // 384-byte kernel argument block, like the learner's KArgs
};

__global__ void k_small(int* flag) {
  if (flag[0] == 12345 && threadIdx.x == 0) flag[1] = blockIdx.x;
}
__global__ void k_big(Big b, int* flag) {
  if (flag[0] == b.v[3] && threadIdx.x == 0) flag[1] = blockIdx.x;
}
// reads a word written by the previous kernel (dependent chain through memory)
__global__ void k_chain(int* flag) {
  if (threadIdx.x == 0 && blockIdx.x == 0) flag[2] = flag[2] + 1;
}
// `depth` dependent loads of words the previous kernel wrote (pointer chase through memory)
__global__ void k_dep(int* buf, int depth) {
  int idx = 0;
  for (int d = 0; d < depth; ++d) idx = buf[16 + idx * 32 + d];
  if (threadIdx.x == 0) buf[16 + (blockIdx.x & 7) * 32 + 40] = idx;  // dirty a line
}
// every wave of a 1024-thread workgroup reads the same 16 words the previous kernel wrote
__global__ __launch_bounds__(1024) void k_hot_all(int* buf) {
  extern __shared__ int lds[];
  int acc = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) acc += buf[8192 + k];
  lds[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 0) buf[8192 + (lds[5] & 15)] = acc + 1;
}
// only wave 0 reads them; the others get them through LDS
__global__ __launch_bounds__(1024) void k_hot_one(int* buf) {
  extern __shared__ int lds[];
  if (threadIdx.x < 64) {
    int acc = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) acc += buf[8192 + k];
    lds[threadIdx.x] = acc;
  }
  __syncthreads();
  const int acc = lds[threadIdx.x & 63];
  if (threadIdx.x == 0 && blockIdx.x == 0) buf[8192 + (acc & 15)] = acc + 1;
}
__global__ void k_init(int* buf) {
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) buf[16 + i] = 0;
}
__global__ __launch_bounds__(1024) void k_lds(int* flag) {
  extern __shared__ int lds[];
  if (flag[0] == 12345) {
    lds[threadIdx.x] = 1;
    __syncthreads();
    flag[1] = lds[0];
  }
}

int main() {
  int* flag;
  CK(hipMalloc(&flag, 1 << 20));
  CK(hipMemset(flag, 0, 1 << 20));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  Big b{};
  const int N = 2000;
  struct Case {
    const char* name;
    int kind, grid, block, lds;
  };
  std::vector<Case> cases = {
      {"small 1x64", 0, 1, 64, 0},          {"small 256x256", 0, 256, 256, 0},
      {"small 1024x256", 0, 1024, 256, 0},  {"big 1x64", 1, 1, 64, 0},
      {"big 256x256", 1, 256, 256, 0},      {"chain 1x64", 2, 1, 64, 0},
      {"lds 256x1024 56K", 3, 256, 1024, 57344}, {"lds 512x1024 56K", 3, 512, 1024, 57344},
      {"dep1 1x64", 11, 1, 64, 0}, {"dep2 1x64", 12, 1, 64, 0}, {"dep4 1x64", 14, 1, 64, 0},
      {"dep8 1x64", 18, 1, 64, 0}, {"dep2 896x256", 12, 896, 256, 0}, {"dep4 256x256", 14, 256, 256, 0},
      {"hot-all 256x1024", 30, 256, 1024, 8192}, {"hot-one 256x1024", 31, 256, 1024, 8192},
      {"hot-all 64x1024", 30, 64, 1024, 8192}, {"hot-one 64x1024", 31, 64, 1024, 8192},
  };
  auto launch = [&](const Case& c) {
    if (c.kind == 0) hipLaunchKernelGGL(k_small, dim3(c.grid), dim3(c.block), 0, s, flag);
    if (c.kind == 1) hipLaunchKernelGGL(k_big, dim3(c.grid), dim3(c.block), 0, s, b, flag);
    if (c.kind == 2) hipLaunchKernelGGL(k_chain, dim3(c.grid), dim3(c.block), 0, s, flag);
    if (c.kind == 3) hipLaunchKernelGGL(k_lds, dim3(c.grid), dim3(c.block), c.lds, s, flag);
    if (c.kind > 10 && c.kind < 30) hipLaunchKernelGGL(k_dep, dim3(c.grid), dim3(c.block), 0, s, flag, c.kind - 10);
    if (c.kind == 30) hipLaunchKernelGGL(k_hot_all, dim3(c.grid), dim3(c.block), c.lds, s, flag);
    if (c.kind == 31) hipLaunchKernelGGL(k_hot_one, dim3(c.grid), dim3(c.block), c.lds, s, flag);
  };
  hipLaunchKernelGGL(k_init, dim3(1), dim3(256), 0, s, flag);
  for (const Case& c : cases) {
    for (int i = 0; i < 50; ++i) launch(c);
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < N; ++i) launch(c);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    // graph of the same N launches
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < N; ++i) launch(c);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float gms = 0;
    CK(hipEventElapsedTime(&gms, e0, e1));
    std::printf("%-20s eager %6.2f us/kernel   graph %6.2f us/kernel\n", c.name, 1000.f * ms / N, 1000.f * gms / N);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
