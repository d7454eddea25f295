#include "lgbm_amd/dcg.h"

#include <algorithm>
#include <cmath>

#include "lgbm_amd/log.h"

namespace lgbm_amd {

void DCG::DefaultEvalAt(std::vector<int>* eval_at) {
  if (eval_at->empty()) {
    for (int i = 1; i <= 5; ++i) eval_at->push_back(i);
  } else {
    for (int k : *eval_at) LGBM_CHECK_GT(k, 0);
  }
}

void DCG::DefaultLabelGain(std::vector<double>* gain) {
  if (!gain->empty()) return;
  gain->push_back(0.0);
  for (int i = 1; i < 31; ++i) gain->push_back(static_cast<double>((1 << i) - 1));
}

void DCG::Init(const std::vector<double>& gain) {
  label_gain_() = gain;
  auto& d = discount();
  if (d.empty()) {
    d.resize(kMaxPosition);
    for (data_size_t i = 0; i < kMaxPosition; ++i) d[i] = 1.0 / std::log2(2.0 + i);
  }
}

double DCG::MaxDCGAtK(data_size_t k, const label_t* label, data_size_t n) {
  const auto& g = label_gain_();
  std::vector<data_size_t> cnt(g.size(), 0);
  for (data_size_t i = 0; i < n; ++i) ++cnt[static_cast<int>(label[i])];
  int top = static_cast<int>(g.size()) - 1;
  if (k > n) k = n;
  double r = 0;
  for (data_size_t j = 0; j < k; ++j) {
    while (top > 0 && cnt[top] <= 0) --top;
    if (top < 0) break;
    r += discount()[j] * g[top];
    cnt[top] -= 1;
  }
  return r;
}

void DCG::MaxDCG(const std::vector<data_size_t>& ks, const label_t* label, data_size_t n, std::vector<double>* out) {
  const auto& g = label_gain_();
  std::vector<data_size_t> cnt(g.size(), 0);
  for (data_size_t i = 0; i < n; ++i) ++cnt[static_cast<int>(label[i])];
  double cur = 0;
  data_size_t left = 0;
  int top = static_cast<int>(g.size()) - 1;
  for (size_t i = 0; i < ks.size(); ++i) {
    data_size_t k = std::min(ks[i], n);
    for (data_size_t j = left; j < k; ++j) {
      while (top > 0 && cnt[top] <= 0) --top;
      if (top < 0) break;
      cur += discount()[j] * g[top];
      cnt[top] -= 1;
    }
    (*out)[i] = cur;
    left = k;
  }
}

void DCG::DCGAt(const std::vector<data_size_t>& ks, const label_t* label, const double* score, data_size_t n,
                std::vector<double>* out) {
  std::vector<data_size_t> idx(n);
  for (data_size_t i = 0; i < n; ++i) idx[i] = i;
  std::stable_sort(idx.begin(), idx.end(), [score](data_size_t a, data_size_t b) { return score[a] > score[b]; });
  double cur = 0;
  data_size_t left = 0;
  for (size_t i = 0; i < ks.size(); ++i) {
    data_size_t k = std::min(ks[i], n);
    for (data_size_t j = left; j < k; ++j) cur += label_gain_()[static_cast<int>(label[idx[j]])] * discount()[j];
    (*out)[i] = cur;
    left = k;
  }
}

void DCG::CheckLabel(const label_t* label, data_size_t n) {
  for (data_size_t i = 0; i < n; ++i) {
    label_t d = std::fabs(label[i] - static_cast<int>(label[i]));
    if (d > kEpsilon) {
      Log::Fatal("label should be int type (met %f) for ranking task,\nfor the gain of label, please set the label_gain parameter",
                 label[i]);
    }
    if (label[i] < 0) Log::Fatal("Label should be non-negative (met %f) for ranking task", label[i]);
    if (static_cast<size_t>(label[i]) >= label_gain_().size()) {
      Log::Fatal("Label %zu is not less than the number of label mappings (%zu)", static_cast<size_t>(label[i]),
                 label_gain_().size());
    }
  }
}

}  // namespace lgbm_amd
