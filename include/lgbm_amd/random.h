// 32-bit LCG with the reference's constants (x = 214013*x + 2531011) so that every
// sampled set (bin-construction sample, bagging, feature_fraction, GOSS, DART drops,
// extra_trees thresholds, EFB search order) is bit-identical to the reference
// (reference: include/LightGBM/utils/random.h:14-117).  Usable on device.
#pragma once

#include <cmath>
#include <set>
#include <vector>

#include "lgbm_amd/meta.h"

namespace lgbm_amd {

class Random {
 public:
  LGBM_HD Random() : x_(123456789u) {}
  LGBM_HD explicit Random(int seed) : x_(static_cast<unsigned>(seed)) {}

  // [lo, hi) from the 15-bit stream
  LGBM_HD int NextShort(int lo, int hi) { return Step16() % (hi - lo) + lo; }
  // [lo, hi) from the 31-bit stream
  LGBM_HD int NextInt(int lo, int hi) { return Step31() % (hi - lo) + lo; }
  // [0, 1)
  LGBM_HD float NextFloat() { return static_cast<float>(Step16()) / 32768.0f; }

  // K ordered samples from {0..N-1}
  std::vector<int> Sample(int N, int K) {
    std::vector<int> out;
    if (K > N || K <= 0) return out;
    out.reserve(K);
    if (K == N) {
      for (int i = 0; i < N; ++i) out.push_back(i);
    } else if (K > 1 && K > (N / std::log2(K))) {
      for (int i = 0; i < N; ++i) {
        double prob = (K - static_cast<double>(out.size())) / static_cast<double>(N - i);
        if (NextFloat() < prob) out.push_back(i);
      }
    } else {
      std::set<int> chosen;
      for (int r = N - K; r < N; ++r) {
        int v = NextInt(0, r);
        if (!chosen.insert(v).second) chosen.insert(r);
      }
      out.assign(chosen.begin(), chosen.end());
    }
    return out;
  }

  LGBM_HD unsigned state() const { return x_; }

 private:
  LGBM_HD int Step16() { x_ = 214013u * x_ + 2531011u; return static_cast<int>((x_ >> 16) & 0x7FFF); }
  LGBM_HD int Step31() { x_ = 214013u * x_ + 2531011u; return static_cast<int>(x_ & 0x7FFFFFFF); }
  unsigned x_;
};

}  // namespace lgbm_amd
