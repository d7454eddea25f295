// Point-wise objective gradients on device (reference src/objective/*.hpp GetGradients):
// regression family, binary / cross-entropy, multiclass softmax.  One thread per row; the
// training score never leaves HBM.
#include "objective_common.h"

namespace lgbm_amd {
namespace dev {

#ifndef LGBM_GRAD_ROWS
#define LGBM_GRAD_ROWS 4
#endif
constexpr int kGradRows = LGBM_GRAD_ROWS;  // rows per thread per iteration (independent loads in flight)

__global__ __launch_bounds__(256) void k_gradients(GradArgs ga) {
  const int64_t n = ga.num_data;
  // fused packing (one model per iteration): (g, h) interleaved for the histogram gathers,
  // per-workgroup max|g| / max h (fixed-point scales) and (sum g, sum h) (root statistics),
  // reduced in a fixed order by k_reduce_parts: deterministic, no contended atomics
  float mg = 0.f, mh = 0.f;
  double sg = 0.0, shh = 0.0;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t base = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; base < n;
       base += kGradRows * stride) {
    double yv[kGradRows], sv[kGradRows], wv[kGradRows];
#pragma unroll
    for (int k = 0; k < kGradRows; ++k) {
      const int64_t i = base + k * stride;
      const bool ok = i < n;
      yv[k] = ok ? static_cast<double>(ga.label[i]) : 0.0;
      sv[k] = ok ? ga.score[i] : 0.0;
      wv[k] = ok && ga.weights ? static_cast<double>(ga.weights[i]) : 1.0;
    }
#pragma unroll
    for (int k = 0; k < kGradRows; ++k) {
      const int64_t i = base + k * stride;
      if (i >= n) break;
      double g, h;
      if (!RowGrad(ga, i, n, yv[k], sv[k], wv[k], g, h)) continue;
      const float gf = static_cast<float>(g), hf = static_cast<float>(h);
      if (ga.write_split || ga.gh == nullptr) {  // (without gh, grad / hess are the only output)
        ga.grad[i] = gf;
        ga.hess[i] = hf;
      }
      if (ga.gh != nullptr) {
        reinterpret_cast<float2*>(ga.gh)[i * ga.gh_stride] = make_float2(gf, hf);
        mg = fmaxf(mg, fabsf(gf));
        mh = HessMax(mh, hf);
        sg += gf;
        shh += hf;
      }
    }
  }
  if (ga.gh == nullptr) return;
  __shared__ float smg[4], smh[4];
  __shared__ double ssg[4], ssh[4];
  for (int o = 32; o > 0; o >>= 1) {
    mg = fmaxf(mg, __shfl_xor(mg, o, kWave));
    mh = HessMax(mh, __shfl_xor(mh, o, kWave));
    sg += __shfl_xor(sg, o, kWave);
    shh += __shfl_xor(shh, o, kWave);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    smg[w] = mg;
    smh[w] = mh;
    ssg[w] = sg;
    ssh[w] = shh;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double tg = 0.0, th = 0.0;
    for (int i = 0; i < static_cast<int>(blockDim.x >> 6); ++i) {
      mg = fmaxf(mg, smg[i]);
      mh = HessMax(mh, smh[i]);
      tg += ssg[i];
      th += ssh[i];
    }
    ga.max_parts[2 * blockIdx.x] = mg;
    ga.max_parts[2 * blockIdx.x + 1] = mh;
    ga.root_parts[2 * blockIdx.x] = tg;
    ga.root_parts[2 * blockIdx.x + 1] = th;
  }
}

// per-workgroup maxima (and root sums) of the gradient / packing kernels, fixed order (one
// workgroup of kReduceParts threads)
constexpr int kReducePartsThreads = 1024;
__global__ __launch_bounds__(kReducePartsThreads) void k_reduce_parts(const float* max_parts, const double* root_parts,
                                                                      int nparts, int64_t n, int rows_cap,
                                                                      uint32_t* absmax, double* root, int units,
                                                                      double* scales) {
  __shared__ double sg[kReducePartsThreads], sh[kReducePartsThreads];
  __shared__ float mg[kReducePartsThreads], mh[kReducePartsThreads];
  double a = 0.0, b = 0.0;
  float x = 0.f, y = 0.f;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
    x = fmaxf(x, max_parts[2 * i]);
    y = HessMax(y, max_parts[2 * i + 1]);
    if (root_parts != nullptr) {
      a += root_parts[2 * i];
      b += root_parts[2 * i + 1];
    }
  }
  sg[threadIdx.x] = a;
  sh[threadIdx.x] = b;
  mg[threadIdx.x] = x;
  mh[threadIdx.x] = y;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if (static_cast<int>(threadIdx.x) < o) {
      sg[threadIdx.x] += sg[threadIdx.x + o];
      sh[threadIdx.x] += sh[threadIdx.x + o];
      mg[threadIdx.x] = fmaxf(mg[threadIdx.x], mg[threadIdx.x + o]);
      mh[threadIdx.x] = HessMax(mh[threadIdx.x], mh[threadIdx.x + o]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const uint32_t am[4] = {__float_as_uint(mg[0]),  // non-negative floats order like their bit patterns
                            __float_as_uint(fabsf(mh[0])),
                            static_cast<uint32_t>(rows_cap),  // (the row cap, max over ranks after the all-reduce)
                            signbit(mh[0]) ? 1u : 0u};        // (a negative hessian: signed packed h)
    for (int k = 0; k < 4; ++k) absmax[k] = am[k];
    // one process: the tree's scales at once (no all-reduce between: k_scales' work, one launch less)
    if (scales != nullptr) ScalesFromAbsmax(am, rows_cap, units, scales);
    if (root != nullptr) {
      root[0] = sg[0];
      root[1] = sh[0];
      root[2] = static_cast<double>(n);
    }
  }
}

int GradientBlocks(int64_t n) { return GridFor(n); }

void ReduceParts(const float* max_parts, const double* root_parts, int nparts, int64_t n, int rows_cap,
                 uint32_t* absmax, double* root, hipStream_t s, int units, double* scales) {
  hipLaunchKernelGGL(k_reduce_parts, dim3(1), dim3(kReducePartsThreads), 0, s, max_parts, root_parts, nparts, n, rows_cap,
                     absmax, root, units, scales);
}

void Gradients(const GradArgs& g, hipStream_t s) {
  hipLaunchKernelGGL(k_gradients, dim3(GradientBlocks(g.num_data)), dim3(256), 0, s, g);
}

__global__ __launch_bounds__(256) void k_unpack_gh(const float2* __restrict__ gh, int64_t stride, int64_t n,
                                                   float* __restrict__ grad, float* __restrict__ hess) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const float2 v = gh[i * stride];
    grad[i] = v.x;
    hess[i] = v.y;
  }
}

void UnpackGH(const GH* gh, int64_t gh_stride, int64_t n, float* grad, float* hess, hipStream_t s) {
  hipLaunchKernelGGL(k_unpack_gh, dim3(GridFor(n)), dim3(256), 0, s, reinterpret_cast<const float2*>(gh), gh_stride, n,
                     grad, hess);
}

}  // namespace dev
}  // namespace lgbm_amd
