// Per-row gradient math shared by the gradient kernel (objective_kernels.hip) and the score
// walk that computes the next iteration's gradients (score_kernels.hip)
#pragma once

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

}  // namespace dev
}  // namespace lgbm_amd
