// Point-wise objective gradients on device (reference src/objective/*.hpp GetGradients):
// regression family, binary / cross-entropy, multiclass softmax.  One thread per row; the
// training score never leaves HBM.
#include "device_common.h"

namespace lgbm_amd {
namespace dev {

// gradient / hessian of row i (false: multiclass, which writes all its classes itself)
__device__ __forceinline__ bool RowGrad(const GradArgs& ga, int64_t i, int64_t n, double y, double s, double w,
                                        double& g, double& h) {
  g = 0;
  h = 0;
  switch (ga.kind) {
    case 1:  // L2
      g = (s - y) * w;
      h = w;
      break;
    case 2: {  // L1
      const double d = s - y;
      g = ((d > 0) - (d < 0)) * w;
      h = w;
      break;
    }
    case 3: {  // Huber
      const double d = s - y;
      g = (fabs(d) <= ga.p0 ? d : ((d > 0) - (d < 0)) * ga.p0) * w;
      h = w;
      break;
    }
    case 4: {  // Fair
      const double x = s - y, c = ga.p0;
      g = c * x / (fabs(x) + c) * w;
      h = c * c / ((fabs(x) + c) * (fabs(x) + c)) * w;
      break;
    }
    case 5:  // Poisson
      g = (exp(s) - y) * w;
      h = exp(s + ga.p0) * w;
      break;
    case 6: {  // Quantile
      const float d = static_cast<float>(s - y);
      const float alpha = static_cast<float>(ga.p0);
      if (ga.weights) {
        g = (d >= 0 ? (1.0f - alpha) : -alpha) * w;
        h = w;
      } else {
        g = d >= 0 ? (1.0f - alpha) : -alpha;
        h = 1.0f;
      }
      break;
    }
    case 7: {  // MAPE
      const double d = s - y;
      g = ((d > 0) - (d < 0)) * static_cast<double>(ga.label_weight[i]);
      h = ga.weights ? ga.weights[i] : 1.0f;
      break;
    }
    case 8:  // Gamma
      if (ga.weights) {
        g = 1.0 - y / exp(s) * w;
        h = y / exp(s) * w;
      } else {
        g = 1.0 - y / exp(s);
        h = y / exp(s);
      }
      break;
    case 9: {  // Tweedie
      const double rho = ga.p0;
      const double e1 = exp((1 - rho) * s), e2 = exp((2 - rho) * s);
      g = (-y * e1 + e2) * w;
      h = (-y * (1 - rho) * e1 + (2 - rho) * e2) * w;
      break;
    }
    case 10: {  // binary logloss
      const int pos = y > 0;
      const int lab = pos ? 1 : -1;
      const double lw = pos ? ga.lw1 : ga.lw0;
      const double sig = ga.p0;
      const double resp = -lab * sig / (1.0f + exp(lab * sig * s));
      const double ar = fabs(resp);
      g = resp * lw * w;
      h = ar * (sig - ar) * lw * w;
      break;
    }
    case 11: {  // cross entropy
      const double z = 1.0f / (1.0f + exp(-s));
      g = (z - y) * w;
      h = z * (1.0f - z) * w;
      break;
    }
    case 12: {  // cross entropy lambda
      if (!ga.weights) {
        const double z = 1.0f / (1.0f + exp(-s));
        g = z - y;
        h = z * (1.0f - z);
      } else {
        const double epf = exp(s);
        const double hhat = log(1.0f + epf);
        const double z = 1.0f - exp(-w * hhat);
        const double enf = 1.0f / epf;
        g = (1.0f - y / z) * w / (1.0f + enf);
        const double c = 1.0f / (1.0f - z);
        double d = 1.0f + epf;
        const double aa = w * epf / (d * d);
        d = c - 1.0f;
        const double b = (c / (d * d)) * (1.0f + w * epf - c);
        h = aa * (1.0f + y * b);
      }
      break;
    }
    case 13: {  // multiclass softmax (all classes of row i)
      const int K = ga.num_class;
      double mx = -INFINITY;
      for (int k = 0; k < K; ++k) mx = fmax(mx, ga.score[k * n + i]);
      double den = 0.0;
      for (int k = 0; k < K; ++k) den += exp(ga.score[k * n + i] - mx);
      const int lab = static_cast<int>(y);
      for (int k = 0; k < K; ++k) {
        const double pk = exp(ga.score[k * n + i] - mx) / den;
        ga.grad[k * n + i] = static_cast<float>((lab == k ? pk - 1.0f : pk) * w);
        ga.hess[k * n + i] = static_cast<float>(ga.p0 * pk * (1.0f - pk) * w);
      }
      return false;  // (ga.gh is null for multi-model objectives)
    }
    default:
      break;
  }
  return true;
}

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
      if (ga.write_split) {
        ga.grad[i] = gf;
        ga.hess[i] = hf;
      }
      if (ga.gh != nullptr) {
        reinterpret_cast<float2*>(ga.gh)[i * ga.gh_stride] = make_float2(gf, hf);
        mg = fmaxf(mg, fabsf(gf));
        mh = fmaxf(mh, fabsf(hf));
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
    mh = fmaxf(mh, __shfl_xor(mh, o, kWave));
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
      mh = fmaxf(mh, smh[i]);
      tg += ssg[i];
      th += ssh[i];
    }
    ga.max_parts[2 * blockIdx.x] = mg;
    ga.max_parts[2 * blockIdx.x + 1] = mh;
    ga.root_parts[2 * blockIdx.x] = tg;
    ga.root_parts[2 * blockIdx.x + 1] = th;
  }
}

// per-workgroup maxima (and root sums) of the gradient / packing kernels, fixed order
__global__ void k_reduce_parts(const float* max_parts, const double* root_parts, int nparts, int64_t n,
                               int rows_cap, uint32_t* absmax, double* root) {
  __shared__ double sg[256], sh[256];
  __shared__ float mg[256], mh[256];
  double a = 0.0, b = 0.0;
  float x = 0.f, y = 0.f;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
    x = fmaxf(x, max_parts[2 * i]);
    y = fmaxf(y, max_parts[2 * i + 1]);
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
      mh[threadIdx.x] = fmaxf(mh[threadIdx.x], mh[threadIdx.x + o]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    absmax[0] = __float_as_uint(mg[0]);  // non-negative floats order like their bit patterns
    absmax[1] = __float_as_uint(mh[0]);
    absmax[2] = static_cast<uint32_t>(rows_cap);  // (the row cap, max over ranks after the all-reduce)
    absmax[3] = 0u;
    if (root != nullptr) {
      root[0] = sg[0];
      root[1] = sh[0];
      root[2] = static_cast<double>(n);
    }
  }
}

int GradientBlocks(int64_t n) { return GridFor(n); }

void ReduceParts(const float* max_parts, const double* root_parts, int nparts, int64_t n, int rows_cap,
                 uint32_t* absmax, double* root, hipStream_t s) {
  hipLaunchKernelGGL(k_reduce_parts, dim3(1), dim3(256), 0, s, max_parts, root_parts, nparts, n, rows_cap, absmax,
                     root);
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
