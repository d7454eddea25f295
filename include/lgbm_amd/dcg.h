// DCG helper tables for lambdarank / NDCG (reference src/metric/dcg_calculator.cpp:1-173):
// default label gains 2^i - 1 (i < 31), discount 1/log2(2+i) for 10000 positions.
#pragma once

#include <vector>

#include "lgbm_amd/meta.h"

namespace lgbm_amd {

class DCG {
 public:
  static void DefaultEvalAt(std::vector<int>* eval_at);
  static void DefaultLabelGain(std::vector<double>* gain);
  static void Init(const std::vector<double>& gain);
  static double Discount(data_size_t i) { return discount()[i]; }
  static const std::vector<double>& label_gain() { return label_gain_(); }
  static double MaxDCGAtK(data_size_t k, const label_t* label, data_size_t n);
  static void MaxDCG(const std::vector<data_size_t>& ks, const label_t* label, data_size_t n, std::vector<double>* out);
  static void DCGAt(const std::vector<data_size_t>& ks, const label_t* label, const double* score, data_size_t n,
                    std::vector<double>* out);
  static void CheckLabel(const label_t* label, data_size_t n);
  static const data_size_t kMaxPosition = 10000;

 private:
  static std::vector<double>& label_gain_() { static std::vector<double> g; return g; }
  static std::vector<double>& discount() { static std::vector<double> d; return d; }
};

}  // namespace lgbm_amd
