// Micro-benchmark of histogram-construction layouts on MI355X (standalone; not part of the
// library).  10M rows x 28 uint8 features, (g, h) fp32 per row; reports us per full pass.
//   hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics hist_variants.hip -o hist_variants
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      printf("HIP error %s line %d: %s\n", #x, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int F = 28;      // features (one byte each)
constexpr int W = 7;       // words per row
constexpr int NB = 256;    // bins per feature slot
constexpr int TB = F * NB;  // total bins

// V1: 7 threads per row, interleaved (g,h) LDS layout, global atomic flush
template <bool PLANAR, bool FLUSH>
__global__ __launch_bounds__(256) void k_v1(const uint32_t* __restrict__ bins, const float2* __restrict__ gh,
                                            const int* __restrict__ idx, int n, float* __restrict__ out) {
  extern __shared__ float lds[];
  for (int i = threadIdx.x; i < 2 * TB; i += 256) lds[i] = 0.f;
  __syncthreads();
  const int chunk = (n + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * chunk, r1 = min(n, r0 + chunk);
  const int q = threadIdx.x % W, rs = threadIdx.x / W, rpp = 256 / W;
  if (rs < rpp) {
    for (int i = r0 + rs; i < r1; i += rpp) {
      const int r = idx ? idx[i] : i;
      const float2 v = gh[r];
      const uint32_t w = bins[(size_t)r * W + q];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int b = (4 * q + j) * NB + ((w >> (8 * j)) & 0xff);
        if (PLANAR) {
          atomicAdd(&lds[b], v.x);
          atomicAdd(&lds[TB + b], v.y);
        } else {
          atomicAdd(&lds[2 * b], v.x);
          atomicAdd(&lds[2 * b + 1], v.y);
        }
      }
    }
  }
  __syncthreads();
  if (FLUSH) {
    for (int i = threadIdx.x; i < 2 * TB; i += 256) {
      const float v = lds[i];
      if (v != 0.f) atomicAdd(&out[i], v);
    }
  }
}

// V2: one wave handles 64 rows at a time; lane l loads row (base + l) fully (7 words) and
// adds feature f for all lanes in lockstep (feature-major issue order)
template <bool FLUSH>
__global__ __launch_bounds__(256) void k_v2(const uint32_t* __restrict__ bins, const float2* __restrict__ gh,
                                            const int* __restrict__ idx, int n, float* __restrict__ out) {
  extern __shared__ float lds[];
  for (int i = threadIdx.x; i < 2 * TB; i += 256) lds[i] = 0.f;
  __syncthreads();
  const int chunk = (n + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * chunk, r1 = min(n, r0 + chunk);
  for (int i = r0 + threadIdx.x; i < r1; i += 256) {
    const int r = idx ? idx[i] : i;
    const float2 v = gh[r];
    uint32_t w[W];
#pragma unroll
    for (int k = 0; k < W; ++k) w[k] = bins[(size_t)r * W + k];
#pragma unroll
    for (int k = 0; k < W; ++k) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int b = (4 * k + j) * NB + ((w[k] >> (8 * j)) & 0xff);
        atomicAdd(&lds[b], v.x);
        atomicAdd(&lds[TB + b], v.y);
      }
    }
  }
  __syncthreads();
  if (FLUSH) {
    for (int i = threadIdx.x; i < 2 * TB; i += 256) {
      const float v = lds[i];
      if (v != 0.f) atomicAdd(&out[i], v);
    }
  }
}

// V3: like V1 planar, but each block writes its partial histogram (no atomics) and a
// second kernel reduces the partial slabs
__global__ __launch_bounds__(256) void k_v3(const uint32_t* __restrict__ bins, const float2* __restrict__ gh,
                                            const int* __restrict__ idx, int n, float* __restrict__ slabs) {
  extern __shared__ float lds[];
  for (int i = threadIdx.x; i < 2 * TB; i += 256) lds[i] = 0.f;
  __syncthreads();
  const int chunk = (n + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * chunk, r1 = min(n, r0 + chunk);
  const int q = threadIdx.x % W, rs = threadIdx.x / W, rpp = 256 / W;
  if (rs < rpp) {
    for (int i = r0 + rs; i < r1; i += rpp) {
      const int r = idx ? idx[i] : i;
      const float2 v = gh[r];
      const uint32_t w = bins[(size_t)r * W + q];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int b = (4 * q + j) * NB + ((w >> (8 * j)) & 0xff);
        atomicAdd(&lds[b], v.x);
        atomicAdd(&lds[TB + b], v.y);
      }
    }
  }
  __syncthreads();
  float* dst = slabs + (size_t)blockIdx.x * 2 * TB;
  for (int i = threadIdx.x; i < 2 * TB; i += 256) dst[i] = lds[i];
}

__global__ void k_v3_reduce(const float* __restrict__ slabs, int nslab, float* __restrict__ out) {
  // grid: (2*TB/256, S) ; each block sums nslab/S slabs for 256 bins then one atomic
  const int bin = blockIdx.x * 256 + threadIdx.x;
  const int per = (nslab + gridDim.y - 1) / gridDim.y;
  const int s0 = blockIdx.y * per, s1 = min(nslab, s0 + per);
  float acc = 0.f;
  for (int s = s0; s < s1; ++s) acc += slabs[(size_t)s * 2 * TB + bin];
  if (bin < 2 * TB) atomicAdd(&out[bin], acc);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 10000000;
  std::vector<uint32_t> hb((size_t)n * W);
  std::vector<float2> hgh(n);
  unsigned s = 12345;
  for (size_t i = 0; i < hb.size(); ++i) {
    uint32_t w = 0;
    for (int j = 0; j < 4; ++j) {
      s = s * 1664525u + 1013904223u;
      w |= ((s >> 16) % 255u) << (8 * j);
    }
    hb[i] = w;
  }
  for (int i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    hgh[i] = make_float2(((s >> 8) & 0xffff) / 65536.f - 0.5f, 0.25f);
  }
  std::vector<int> hidx(n);
  for (int i = 0; i < n; ++i) hidx[i] = i;
  // a random half for the gather case
  for (int i = n - 1; i > 0; --i) {
    s = s * 1664525u + 1013904223u;
    int j = (s >> 4) % (i + 1);
    std::swap(hidx[i], hidx[j]);
  }
  uint32_t* d_bins;
  float2* d_gh;
  int* d_idx;
  float *d_out, *d_slab;
  CHECK(hipMalloc(&d_bins, hb.size() * 4));
  CHECK(hipMalloc(&d_gh, (size_t)n * 8));
  CHECK(hipMalloc(&d_idx, (size_t)n * 4));
  CHECK(hipMalloc(&d_out, 2 * TB * 4));
  CHECK(hipMalloc(&d_slab, (size_t)2048 * 2 * TB * 4));
  CHECK(hipMemcpy(d_bins, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_gh, hgh.data(), (size_t)n * 8, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_idx, hidx.data(), (size_t)n * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const size_t lds = 2 * TB * 4;
  auto timeit = [&](const char* name, auto launch) {
    for (int w = 0; w < 2; ++w) launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    const int reps = 5;
    for (int r = 0; r < reps; ++r) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-48s %9.1f us\n", name, 1000.f * ms / reps);
  };
  const int half = n / 2;
  for (int grid : {256, 512, 1024}) {
    char buf[128];
    snprintf(buf, sizeof buf, "v1 interleaved flush grid=%d", grid);
    timeit(buf, [&] { hipLaunchKernelGGL((k_v1<false, true>), dim3(grid), dim3(256), lds, 0, d_bins, d_gh, nullptr, n, d_out); });
    snprintf(buf, sizeof buf, "v1 interleaved NOflush grid=%d", grid);
    timeit(buf, [&] { hipLaunchKernelGGL((k_v1<false, false>), dim3(grid), dim3(256), lds, 0, d_bins, d_gh, nullptr, n, d_out); });
    snprintf(buf, sizeof buf, "v1 planar flush grid=%d", grid);
    timeit(buf, [&] { hipLaunchKernelGGL((k_v1<true, true>), dim3(grid), dim3(256), lds, 0, d_bins, d_gh, nullptr, n, d_out); });
    snprintf(buf, sizeof buf, "v1 planar NOflush grid=%d", grid);
    timeit(buf, [&] { hipLaunchKernelGGL((k_v1<true, false>), dim3(grid), dim3(256), lds, 0, d_bins, d_gh, nullptr, n, d_out); });
    snprintf(buf, sizeof buf, "v2 row-per-lane planar flush grid=%d", grid);
    timeit(buf, [&] { hipLaunchKernelGGL((k_v2<true>), dim3(grid), dim3(256), lds, 0, d_bins, d_gh, nullptr, n, d_out); });
    snprintf(buf, sizeof buf, "v2 row-per-lane planar NOflush grid=%d", grid);
    timeit(buf, [&] { hipLaunchKernelGGL((k_v2<false>), dim3(grid), dim3(256), lds, 0, d_bins, d_gh, nullptr, n, d_out); });
    snprintf(buf, sizeof buf, "v3 planar slabs+reduce grid=%d", grid);
    timeit(buf, [&] {
      hipLaunchKernelGGL(k_v3, dim3(grid), dim3(256), lds, 0, d_bins, d_gh, nullptr, n, d_slab);
      hipLaunchKernelGGL(k_v3_reduce, dim3(2 * TB / 256, 16), dim3(256), 0, 0, d_slab, grid, d_out);
    });
    snprintf(buf, sizeof buf, "v1 planar flush GATHER half grid=%d", grid);
    timeit(buf, [&] { hipLaunchKernelGGL((k_v1<true, true>), dim3(grid), dim3(256), lds, 0, d_bins, d_gh, d_idx, half, d_out); });
    snprintf(buf, sizeof buf, "v2 planar flush GATHER half grid=%d", grid);
    timeit(buf, [&] { hipLaunchKernelGGL((k_v2<true>), dim3(grid), dim3(256), lds, 0, d_bins, d_gh, d_idx, half, d_out); });
  }
  // small leaf: 20k random rows
  for (int grid : {8, 16, 64}) {
    char buf[128];
    snprintf(buf, sizeof buf, "v1 planar flush GATHER 20k grid=%d", grid);
    timeit(buf, [&] { hipLaunchKernelGGL((k_v1<true, true>), dim3(grid), dim3(256), lds, 0, d_bins, d_gh, d_idx, 20000, d_out); });
  }
  printf("done\n");
  return 0;
}
