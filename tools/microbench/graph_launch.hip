// Host cost of hipGraphLaunch and the GPU's idle time inside a graph, by kernel-argument size
// and node count: a chain of N tiny kernels (each spins ~`us` microseconds) captured once and
// launched repeatedly.  Prints per launch: host time in hipGraphLaunch, wall time to
// completion, and the GPU-busy share.
//   hipcc --offload-arch=gfx950 -O2 tools/microbench/graph_launch.hip -o /tmp/graph_launch
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

template <int BYTES>
struct Args {
  long long spin;  // wall-clock ticks (100 MHz) to spin
  int* out;
  char pad[BYTES > 16 ? BYTES - 16 : 1];
};

template <int BYTES>
__global__ void k_spin(Args<BYTES> a) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < a.spin) {
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) a.out[0] += 1;
}

template <int BYTES>
void Run(int nodes, int us, int reps) {
  hipStream_t s;
  CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int* out;
  CHK(hipMalloc(&out, sizeof(int)));
  Args<BYTES> a{};
  a.spin = us * 100;
  a.out = out;
  hipGraph_t g;
  hipGraphExec_t ge;
  CHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < nodes; ++i) hipLaunchKernelGGL(k_spin<BYTES>, dim3(256), dim3(256), 0, s, a);
  CHK(hipStreamEndCapture(s, &g));
  CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 3; ++i) CHK(hipGraphLaunch(ge, s));
  CHK(hipStreamSynchronize(s));
  double host = 0, wall = 0;
  for (int r = 0; r < reps; ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    CHK(hipGraphLaunch(ge, s));
    const auto t1 = std::chrono::steady_clock::now();
    CHK(hipStreamSynchronize(s));
    const auto t2 = std::chrono::steady_clock::now();
    host += std::chrono::duration<double, std::micro>(t1 - t0).count();
    wall += std::chrono::duration<double, std::micro>(t2 - t0).count();
  }
  host /= reps;
  wall /= reps;
  std::printf("args %5d B  nodes %3d  spin %3d us: hipGraphLaunch %8.1f us (%5.2f / node)  wall %8.1f us  "
              "overhead %6.2f us / node\n",
              BYTES, nodes, us, host, host / nodes, wall, (wall - double(nodes) * us) / nodes);
  CHK(hipGraphExecDestroy(ge));
  CHK(hipGraphDestroy(g));
  CHK(hipFree(out));
  CHK(hipStreamDestroy(s));
}

int main() {
  for (int us : {2, 10}) {
    for (int nodes : {12, 42}) {
      Run<16>(nodes, us, 20);
      Run<256>(nodes, us, 20);
      Run<1024>(nodes, us, 20);
      Run<2048>(nodes, us, 20);
    }
  }
  return 0;
}
