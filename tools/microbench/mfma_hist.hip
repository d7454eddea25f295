// A/B micro-benchmark: the root histogram as an int8 MFMA one-hot product vs LDS integer
// atomics (standalone; not part of the library).  N rows x 28 features of NB bins (16 or 64 --
// the reference's dedicated small-bin kernels, ocl/histogram16.cl / histogram64.cl), fixed-point
// (g, h) per row, every histogram exact (int64) and checked against a host reference.
//
//   A  atomics: the production layout -- row-major bin words (4 features per u32) + interleaved
//      (g, h); 1024-thread workgroups; per word 4 LDS ds_add_u64 of a packed (g << 32 | h)
//   B  MFMA:    H[bin][plane] = sum_rows onehot[bin][row] * V[row][plane] with
//      __builtin_amdgcn_mfma_i32_16x16x64_i8: A = one-hot of 16 bins x 64 rows (byte -128 where
//      the row's bin is the lane's bin: one v_xad + one v_bfi per 4 rows from a column-major
//      copy of the bins), B = 7-bit planes of g and h (4 of the 16 columns), int32 accumulators
//      per (feature, 16-bin tile), flushed to int64 per workgroup
//
//   hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics mfma_hist.hip -o mfma_hist
//   ./mfma_hist [rows=10000000] [reps=20]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      printf("HIP error %s line %d: %s\n", #x, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int F = 28;  // features
constexpr int W = 7;   // bin words per row (row-major layout)
constexpr int kGBits = 13, kHBits = 14;  // g in [-2^13, 2^13), h in [0, 2^14): two 7-bit planes each

using i32x4 = __attribute__((ext_vector_type(4))) int;
using i32x4v = __attribute__((ext_vector_type(4))) int;

// ---------------------------------------------------------------- A: LDS integer atomics
template <int NB>
__global__ __launch_bounds__(1024) void k_atomic(const uint32_t* __restrict__ bins, const int2* __restrict__ gh, int n,
                                                 int rows_per_wg, long long* __restrict__ out) {
  __shared__ unsigned long long lds[F * NB];
  for (int i = threadIdx.x; i < F * NB; i += 1024) lds[i] = 0ull;
  __syncthreads();
  const int r0 = blockIdx.x * rows_per_wg, r1 = min(n, r0 + rows_per_wg);
  // thread -> (row slot, word): 146 row slots x 7 words
  const int q = threadIdx.x % W, rs = threadIdx.x / W, rpp = 1024 / W;
  if (rs < rpp) {
    for (int r = r0 + rs; r < r1; r += rpp) {
      const int2 v = gh[r];
      const uint32_t w = bins[static_cast<size_t>(r) * W + q];
      const unsigned long long p = (static_cast<unsigned long long>(static_cast<long long>(v.x)) << 32) +
                                   static_cast<unsigned long long>(static_cast<uint32_t>(v.y));
#pragma unroll
      for (int j = 0; j < 4; ++j) atomicAdd(&lds[(4 * q + j) * NB + ((w >> (8 * j)) & 0xffu)], p);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < F * NB; i += 1024) {
    const unsigned long long p = lds[i];
    // the packed sum: h in the low 32 bits (non-negative, < 2^32 here), g (signed) above it
    const long long h = static_cast<long long>(p & 0xffffffffull);
    const long long g = (static_cast<long long>(p) - h) >> 32;
    if (g != 0) atomicAdd(reinterpret_cast<unsigned long long*>(&out[2 * i]), static_cast<unsigned long long>(g));
    if (h != 0) atomicAdd(reinterpret_cast<unsigned long long*>(&out[2 * i + 1]), static_cast<unsigned long long>(h));
  }
}

// ---------------------------------------------------------------- B: int8 MFMA one-hot
// value planes of a row: g = g1 * 128 + g0, h = h1 * 128 + h0 (g0, h0, h1 in [0, 127], g1 signed)
__device__ __forceinline__ uint32_t PlaneByte(int g, int h, int plane) {
  switch (plane) {
    case 0: return static_cast<uint32_t>(g & 127);
    case 1: return static_cast<uint32_t>((g >> 7) & 0xff);  // (arithmetic shift: the signed high plane)
    case 2: return static_cast<uint32_t>(h & 127);
    case 3: return static_cast<uint32_t>((h >> 7) & 127);
    default: return 0u;
  }
}

// 256 threads = 4 waves; wave w scans features w, w + 4, ... (FPW of them) over the
// workgroup's rows, 64 rows per step (n and the workgroup's row count are multiples of 64).
// The B fragment: each lane loads its row's (g, h) (one coalesced load), writes the row's four
// plane bytes into a plane-major LDS image, and lane (q, m) reads plane m of rows 16q .. 16q + 15
// back as one 16-byte LDS read
template <int NB>
__global__ __launch_bounds__(256) void k_mfma(const uint8_t* __restrict__ col, const int2* __restrict__ gh, int n,
                                              int rows_per_wg, long long* __restrict__ out) {
  constexpr int T = NB / 16;       // bin tiles of a feature
  constexpr int FPW = F / 4;       // features per wave
  __shared__ __attribute__((aligned(16))) uint8_t s_planes[4][16][64];  // [wave][plane][row]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int q = lane >> 4, m = lane & 15;  // row group of the fragment, lane's bin / plane column
  const int r0 = blockIdx.x * rows_per_wg, r1 = min(n, r0 + rows_per_wg);
  for (int p = lane; p < 16 * 64; p += 64) s_planes[wv][p / 64][p % 64] = 0;  // (planes 4..15 stay 0)
  i32x4 acc[FPW][T];
#pragma unroll
  for (int a = 0; a < FPW; ++a)
#pragma unroll
    for (int t = 0; t < T; ++t) acc[a][t] = i32x4{0, 0, 0, 0};
  for (int c = r0; c < r1; c += 64) {
    const int2 v = gh[c + lane];
    uint4 bb[FPW];
#pragma unroll
    for (int a = 0; a < FPW; ++a) bb[a] = *reinterpret_cast<const uint4*>(col + static_cast<size_t>(wv + 4 * a) * n + c + 16 * q);
    __builtin_amdgcn_wave_barrier();
    s_planes[wv][0][lane] = static_cast<uint8_t>(PlaneByte(v.x, v.y, 0));
    s_planes[wv][1][lane] = static_cast<uint8_t>(PlaneByte(v.x, v.y, 1));
    s_planes[wv][2][lane] = static_cast<uint8_t>(PlaneByte(v.x, v.y, 2));
    s_planes[wv][3][lane] = static_cast<uint8_t>(PlaneByte(v.x, v.y, 3));
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint4 bw = *reinterpret_cast<const uint4*>(&s_planes[wv][m][16 * q]);
    const i32x4v bfrag = {static_cast<int>(bw.x), static_cast<int>(bw.y), static_cast<int>(bw.z), static_cast<int>(bw.w)};
#pragma unroll
    for (int a = 0; a < FPW; ++a) {
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const uint32_t mrep = static_cast<uint32_t>(16 * t + m) * 0x01010101u;
        // byte -128 (0x80) where the row's bin is 16t + m: (bin ^ m) + 0x7f has bit 7 clear
        // only for a zero byte (bins < 128: no carry between bytes); v_bfi keeps bit 7 of ~x
        const uint32_t x0 = (bb[a].x ^ mrep) + 0x7f7f7f7fu, x1 = (bb[a].y ^ mrep) + 0x7f7f7f7fu;
        const uint32_t x2 = (bb[a].z ^ mrep) + 0x7f7f7f7fu, x3 = (bb[a].w ^ mrep) + 0x7f7f7f7fu;
        const i32x4v afrag = {static_cast<int>(~x0 & 0x80808080u), static_cast<int>(~x1 & 0x80808080u),
                              static_cast<int>(~x2 & 0x80808080u), static_cast<int>(~x3 & 0x80808080u)};
        acc[a][t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afrag, bfrag, acc[a][t], 0, 0, 0);
      }
    }
  }
  // D[bin][plane]: lane holds rows (bins) 4q .. 4q + 3 of column (plane) m; each value is -128 x
  // the plane sum.  Planes combine in int64 through the workgroup's LDS
  __shared__ long long s_p[F][NB][4];
#pragma unroll
  for (int a = 0; a < FPW; ++a)
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (m < 4) s_p[wv + 4 * a][16 * t + 4 * q + i][m] = static_cast<long long>(acc[a][t][i]) / -128;
      }
  __syncthreads();
  for (int i = threadIdx.x; i < F * NB; i += 256) {
    const long long* p = s_p[i / NB][i % NB];
    const long long g = p[0] + 128 * p[1], h = p[2] + 128 * p[3];
    if (g != 0) atomicAdd(reinterpret_cast<unsigned long long*>(&out[2 * i]), static_cast<unsigned long long>(g));
    if (h != 0) atomicAdd(reinterpret_cast<unsigned long long*>(&out[2 * i + 1]), static_cast<unsigned long long>(h));
  }
}

template <int NB>
void Run(int n, int reps) {
  std::vector<uint8_t> colh(static_cast<size_t>(F) * n);
  std::vector<uint32_t> rowh(static_cast<size_t>(W) * n);
  std::vector<int> gv(n), hv(n);
  uint64_t s = 12345;
  auto rnd = [&]() {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return static_cast<uint32_t>(s >> 33);
  };
  for (int r = 0; r < n; ++r) {
    for (int f = 0; f < F; ++f) {
      const uint32_t b = (f % 3 == 0) ? (rnd() % 3 == 0 ? rnd() % NB : 0) : rnd() % NB;  // some skewed features
      colh[static_cast<size_t>(f) * n + r] = static_cast<uint8_t>(b);
      rowh[static_cast<size_t>(r) * W + f / 4] |= b << (8 * (f % 4));
    }
    gv[r] = static_cast<int>(rnd() % (1u << (kGBits + 1))) - (1 << kGBits);
    hv[r] = static_cast<int>(rnd() % (1u << kHBits));
  }
  std::vector<long long> ref(2 * F * NB, 0);
  for (int r = 0; r < n; ++r)
    for (int f = 0; f < F; ++f) {
      const int b = colh[static_cast<size_t>(f) * n + r];
      ref[2 * (f * NB + b)] += gv[r];
      ref[2 * (f * NB + b) + 1] += hv[r];
    }
  std::vector<int2> ghh(n);
  for (int r = 0; r < n; ++r) ghh[r] = int2{gv[r], hv[r]};
  uint8_t* dcol;
  uint32_t* drow;
  int2* dgh;
  long long* dout;
  CHECK(hipMalloc(&dcol, colh.size()));
  CHECK(hipMalloc(&drow, rowh.size() * 4));
  CHECK(hipMalloc(&dgh, ghh.size() * sizeof(int2)));
  CHECK(hipMalloc(&dout, ref.size() * 8));
  CHECK(hipMemcpy(dcol, colh.data(), colh.size(), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(drow, rowh.data(), rowh.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dgh, ghh.data(), ghh.size() * sizeof(int2), hipMemcpyHostToDevice));
  int dev = 0, cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto bench = [&](const char* name, int wgs, auto launch) {
    std::vector<long long> got(ref.size());
    CHECK(hipMemset(dout, 0, ref.size() * 8));
    launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(got.data(), dout, got.size() * 8, hipMemcpyDeviceToHost));
    const bool exact = got == ref;
    launch();
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("bins %3d  %-26s wgs %6d  %8.1f us  %s\n", NB, name, wgs, 1000.0 * ms / reps, exact ? "exact" : "MISMATCH");
  };
  for (int per_cu : {2, 4}) {
    const int wgs = per_cu * cus;
    const int rpw = (n + wgs - 1) / wgs;
    char nm[64];
    snprintf(nm, sizeof(nm), "A lds-atomic (%d wg/CU)", per_cu);
    bench(nm, wgs, [&]() { hipLaunchKernelGGL(k_atomic<NB>, dim3(wgs), dim3(1024), 0, 0, drow, dgh, n, rpw, dout); });
  }
  for (int per_cu : {4, 8}) {
    const int wgs = per_cu * cus;
    const int rpw = ((n + wgs - 1) / wgs + 63) / 64 * 64;  // (n % 64 == 0: whole 64-row steps)
    char nm[64];
    snprintf(nm, sizeof(nm), "B mfma one-hot (%d wg/CU)", per_cu);
    bench(nm, wgs, [&]() { hipLaunchKernelGGL(k_mfma<NB>, dim3((n + rpw - 1) / rpw), dim3(256), 0, 0, dcol, dgh, n, rpw, dout); });
  }
  CHECK(hipFree(dcol));
  CHECK(hipFree(drow));
  CHECK(hipFree(dgh));
  CHECK(hipFree(dout));
}

int main(int argc, char** argv) {
  const int n = (argc > 1 ? atoi(argv[1]) : 10000000) / 64 * 64;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  printf("rows %d, %d features; bins-word reads %.0f MB (A) / column reads %.0f MB (B), (g, h) %.0f MB\n", n, F,
         4.0 * W * n / 1e6, 1.0 * F * n / 1e6, 8.0 * n / 1e6);
  Run<16>(n, reps);
  Run<64>(n, reps);
  return 0;
}
