// A/B of the split scan's prefix sums on MI355X: exact int64 prefix sums of fixed-point
// histograms (g, h) of F features x B bins, one wave per feature, computed
//   (a) with wave shuffles (what k_find does: per-lane runs + a wave-wide scan), and
//   (b) on the matrix cores: P = L . H with L the lower-triangular ones matrix, H the
//       histogram split into 16 byte planes (8 bytes of g, 8 of h) as signed i8
//       (v_mfma_i32_16x16x64_i8, exact i32 accumulation), the planes recombined into int64
//       (byte b' = byte - 128 makes the bytes signed; the offset's prefix is added back),
//   (c) as (b) with the planes staged through LDS and recombined in registers.
// All are checked against a host prefix sum.  Wide shapes: Epsilon (2000 features), Bosch
// (968), Higgs (28); 64 and 256 bins.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench/mfma_scan tools/microbench/mfma_scan.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));
constexpr int kMaxBins = 256;

// (a) one wave per feature; lane l owns bins [l*per, (l+1)*per)
__global__ __launch_bounds__(64) void k_scan_shuffle(const long long* hist, long long* out, int bins) {
  const int f = blockIdx.x, lane = threadIdx.x;
  const int per = (bins + 63) / 64;
  const long long* h = hist + static_cast<size_t>(f) * 2 * bins;
  long long* o = out + static_cast<size_t>(f) * 2 * bins;
  long long g[4], hh[4], sg = 0, sh = 0;
  for (int j = 0; j < per; ++j) {
    const int b = lane * per + j;
    g[j] = b < bins ? h[2 * b] : 0;
    hh[j] = b < bins ? h[2 * b + 1] : 0;
    sg += g[j];
    sh += hh[j];
  }
  // inclusive wave scan of the lane totals
  long long ig = sg, ih = sh;
  for (int d = 1; d < 64; d <<= 1) {
    const long long tg = __shfl_up(ig, d, 64), th = __shfl_up(ih, d, 64);
    if (lane >= d) {
      ig += tg;
      ih += th;
    }
  }
  long long rg = ig - sg, rh = ih - sh;
  for (int j = 0; j < per; ++j) {
    const int b = lane * per + j;
    rg += g[j];
    rh += hh[j];
    if (b < bins) {
      o[2 * b] = rg;
      o[2 * b + 1] = rh;
    }
  }
}

// (b) one wave per feature: 16 row tiles of 16 bins; per tile, K-steps of 64 bins
__global__ __launch_bounds__(64) void k_scan_mfma(const long long* hist, long long* out, int bins) {
  __shared__ int c_lds[kMaxBins][17];  // per bin: the 16 byte-plane prefix sums (padded)
  const int f = blockIdx.x, lane = threadIdx.x;
  const long long* h = hist + static_cast<size_t>(f) * 2 * bins;
  long long* o = out + static_cast<size_t>(f) * 2 * bins;
  const int plane = lane & 15;              // B column: byte (plane & 7) of g (plane < 8) or h
  const int kq = 16 * (lane >> 4);          // this lane's 16 k positions inside a K-step
  const int tiles = (bins + 15) / 16, ksteps = (bins + 63) / 64;
  // B fragments of every K-step: 16 signed bytes per lane
  v4i bf[kMaxBins / 64];
  for (int q = 0; q < ksteps; ++q) {
    unsigned char v[16];
    for (int j = 0; j < 16; ++j) {
      const int b = 64 * q + kq + j;
      const unsigned long long x = b < bins ? static_cast<unsigned long long>(h[2 * b + (plane >> 3)]) : 0ull;
      const unsigned char byte = static_cast<unsigned char>(x >> (8 * (plane & 7)));
      v[j] = b < bins ? static_cast<unsigned char>(byte - 128) : 0;  // two's complement of byte - 128
    }
    for (int w = 0; w < 4; ++w) {
      bf[q][w] = static_cast<int>(v[4 * w] | (v[4 * w + 1] << 8) | (v[4 * w + 2] << 16) |
                                  (static_cast<unsigned>(v[4 * w + 3]) << 24));
    }
  }
  for (int r = 0; r < tiles; ++r) {
    v4i acc = {0, 0, 0, 0};
    const int row = 16 * r + (lane & 15);  // A row of this lane
    for (int q = 0; q < ksteps && 64 * q <= 16 * r + 15; ++q) {
      v4i af;
      for (int w = 0; w < 4; ++w) {
        unsigned word = 0;
        for (int j = 0; j < 4; ++j) {
          const int k = 64 * q + kq + 4 * w + j;
          word |= (k <= row ? 1u : 0u) << (8 * j);
        }
        af[w] = static_cast<int>(word);
      }
      acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(af, bf[q], acc, 0, 0, 0);
    }
    // C/D: col = lane & 15 (plane), row = 4 * (lane >> 4) + reg
    for (int reg = 0; reg < 4; ++reg) c_lds[16 * r + 4 * (lane >> 4) + reg][plane] = acc[reg];
  }
  __syncthreads();
  // recombine: prefix(b) = sum_p C_p(b) 256^p + (b + 1) * 128 * sum_p 256^p   (mod 2^64)
  const unsigned long long off = 0x8080808080808080ull;
  for (int b = lane; b < bins; b += 64) {
    unsigned long long pg = 0, ph = 0;
    for (int p = 0; p < 8; ++p) {
      pg += static_cast<unsigned long long>(static_cast<long long>(c_lds[b][p])) << (8 * p);
      ph += static_cast<unsigned long long>(static_cast<long long>(c_lds[b][8 + p])) << (8 * p);
    }
    pg += static_cast<unsigned long long>(b + 1) * off;
    ph += static_cast<unsigned long long>(b + 1) * off;
    o[2 * b] = static_cast<long long>(pg);
    o[2 * b + 1] = static_cast<long long>(ph);
  }
}

// (c) as (b), but the byte planes are built once through LDS (coalesced loads, transposed
// to plane-major bytes, ds_read_b128 fragments), the triangular A fragments come from a
// ones count, and the planes are recombined in registers (xor butterflies over the 8 lanes
// holding one value's planes) instead of through LDS
__global__ __launch_bounds__(64) void k_scan_mfma2(const long long* hist, long long* out, int bins) {
  __shared__ __attribute__((aligned(16))) unsigned char planes[16][kMaxBins];
  const int f = blockIdx.x, lane = threadIdx.x;
  const long long* h = hist + static_cast<size_t>(f) * 2 * bins;
  long long* o = out + static_cast<size_t>(f) * 2 * bins;
  const int per = bins / 64;  // 1 or 4 bins per lane
  if (per == 4) {
    long long g[4], hh[4];
    for (int j = 0; j < 4; ++j) {
      g[j] = h[2 * (4 * lane + j)];
      hh[j] = h[2 * (4 * lane + j) + 1];
    }
    for (int p = 0; p < 8; ++p) {
      unsigned wg = 0, wh = 0;
      for (int j = 0; j < 4; ++j) {
        wg |= static_cast<unsigned>((static_cast<unsigned long long>(g[j]) >> (8 * p)) & 0xff) << (8 * j);
        wh |= static_cast<unsigned>((static_cast<unsigned long long>(hh[j]) >> (8 * p)) & 0xff) << (8 * j);
      }
      *reinterpret_cast<unsigned*>(&planes[p][4 * lane]) = wg ^ 0x80808080u;
      *reinterpret_cast<unsigned*>(&planes[8 + p][4 * lane]) = wh ^ 0x80808080u;
    }
  } else {
    const unsigned long long g = static_cast<unsigned long long>(h[2 * lane]);
    const unsigned long long hh = static_cast<unsigned long long>(h[2 * lane + 1]);
    for (int p = 0; p < 8; ++p) {
      planes[p][lane] = static_cast<unsigned char>(((g >> (8 * p)) & 0xff) ^ 0x80);
      planes[8 + p][lane] = static_cast<unsigned char>(((hh >> (8 * p)) & 0xff) ^ 0x80);
    }
  }
  __syncthreads();
  const int plane = lane & 15, kq = 16 * (lane >> 4);
  const int tiles = bins / 16, ksteps = bins / 64;
  v4i bf[kMaxBins / 64];
  for (int q = 0; q < ksteps; ++q) bf[q] = *reinterpret_cast<const v4i*>(&planes[plane][64 * q + kq]);
  const unsigned long long off = 0x8080808080808080ull;
  for (int r = 0; r < tiles; ++r) {
    v4i acc = {0, 0, 0, 0};
    const int row = 16 * r + (lane & 15);
    for (int q = 0; q < ksteps && 64 * q <= 16 * r + 15; ++q) {
      const int ones = min(16, max(0, row - (64 * q + kq) + 1));  // k <= row, low bytes first
      v4i af;
      for (int w = 0; w < 4; ++w) {
        const int c = min(4, max(0, ones - 4 * w));
        af[w] = static_cast<int>(c == 4 ? 0x01010101u : (0x01010101u & ((1u << (8 * c)) - 1u)));
      }
      acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(af, bf[q], acc, 0, 0, 0);
    }
    for (int reg = 0; reg < 4; ++reg) {
      unsigned long long v = static_cast<unsigned long long>(static_cast<long long>(acc[reg])) << (8 * (plane & 7));
      for (int d = 1; d < 8; d <<= 1) v += static_cast<unsigned long long>(__shfl_xor(static_cast<long long>(v), d, 64));
      const int b = 16 * r + 4 * (lane >> 4) + reg;
      if ((plane & 7) == 0) o[2 * b + (plane >> 3)] = static_cast<long long>(v + static_cast<unsigned long long>(b + 1) * off);
    }
  }
}

int main() {
  std::mt19937_64 rng(7);
  long long* d_h = nullptr;
  long long* d_o = nullptr;
  const int max_f = 2000;
  CK(hipMalloc(&d_h, sizeof(long long) * 2 * kMaxBins * max_f));
  CK(hipMalloc(&d_o, sizeof(long long) * 2 * kMaxBins * max_f));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::printf("shape                 bins  shuffle us  mfma us  mfma-lds us   exact(shuffle, mfma, mfma-lds)\n");
  for (int F : {2000, 968, 28}) {
    for (int bins : {64, 256}) {
      std::vector<long long> h(static_cast<size_t>(2) * bins * F), ref(h.size()), got(h.size());
      for (size_t i = 0; i < h.size(); i += 2) {
        h[i] = static_cast<long long>(rng() % (1ull << 41)) - (1ll << 40);  // g: signed, |g| < 2^40
        h[i + 1] = static_cast<long long>(rng() % (1ull << 40));             // h: >= 0
      }
      for (int f = 0; f < F; ++f) {
        long long sg = 0, sh = 0;
        for (int b = 0; b < bins; ++b) {
          const size_t i = (static_cast<size_t>(f) * bins + b) * 2;
          sg += h[i];
          sh += h[i + 1];
          ref[i] = sg;
          ref[i + 1] = sh;
        }
      }
      CK(hipMemcpy(d_h, h.data(), sizeof(long long) * h.size(), hipMemcpyHostToDevice));
      bool ok[3];
      float us[3];
      for (int v = 0; v < 3; ++v) {
        auto launch = [&] {
          if (v == 0) hipLaunchKernelGGL(k_scan_shuffle, dim3(F), dim3(64), 0, 0, d_h, d_o, bins);
          else if (v == 1) hipLaunchKernelGGL(k_scan_mfma, dim3(F), dim3(64), 0, 0, d_h, d_o, bins);
          else hipLaunchKernelGGL(k_scan_mfma2, dim3(F), dim3(64), 0, 0, d_h, d_o, bins);
        };
        CK(hipMemset(d_o, 0, sizeof(long long) * h.size()));
        launch();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got.data(), d_o, sizeof(long long) * h.size(), hipMemcpyDeviceToHost));
        ok[v] = got == ref;
        const int reps = 200;
        CK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        us[v] = 1000.0f * ms / reps;
      }
      const char* name = F == 2000 ? "Epsilon (2000 feat)" : F == 968 ? "Bosch (968 feat)" : "Higgs (28 feat)";
      std::printf("%-21s %4d  %10.2f  %8.2f  %11.2f   %s, %s, %s\n", name, bins, us[0], us[1], us[2],
                  ok[0] ? "yes" : "NO", ok[1] ? "yes" : "NO", ok[2] ? "yes" : "NO");
    }
  }
  return 0;
}
