// All metrics.  Loss formulas, tie handling in AUC (ties share half credit), top-k
// multi_error, AUC-mu, NDCG/MAP query weighting and names follow the reference
// (src/metric/{regression,binary,multiclass,rank,map,xentropy}_metric.hpp).
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <numeric>

#include "lgbm_amd/common.h"
#include "lgbm_amd/dcg.h"
#include "lgbm_amd/log.h"
#include "lgbm_amd/metric.h"

namespace lgbm_amd {

namespace {

// ----------------------------------------------------------------- point-wise metrics
using PointLoss = double (*)(label_t label, double score, const Config& cfg);

class PointwiseMetric : public Metric {
 public:
  PointwiseMetric(const Config& cfg, const char* name, PointLoss loss, bool convert, double factor)
      : cfg_(cfg), loss_(loss), convert_(convert), factor_(factor) {
    name_.push_back(name);
    // device kinds (src/device/kernels.h kMetric*) and the loss parameter they take
    static const struct { const char* name; int kind; } kinds[] = {
        {"l2", 1}, {"rmse", 2}, {"l1", 3}, {"binary_logloss", 4}, {"binary_error", 5}, {"quantile", 7},
        {"huber", 8}, {"fair", 9}, {"poisson", 10}, {"mape", 11}, {"gamma", 12}, {"gamma_deviance", 13},
        {"tweedie", 14}, {"cross_entropy", 15}, {"kullback_leibler", 15}};
    for (const auto& k : kinds) {
      if (std::string(name) == k.name) device_kind_ = k.kind;
    }
    device_param_ = device_kind_ == 9 ? cfg.fair_c : device_kind_ == 14 ? cfg.tweedie_variance_power : cfg.alpha;
  }
  DeviceMetricSpec DeviceSpec(const ObjectiveFunction* obj) const override {
    DeviceMetricSpec d;
    if (device_kind_ == 0) return d;
    double param = 1.0;
    const int conv = (convert_ && obj != nullptr) ? obj->DeviceOutputKind(&param) : 0;
    if (conv < 0 || conv > 3) return d;
    d.kind = device_kind_;
    d.convert = conv;
    d.sigmoid = param;
    d.param = device_param_;
    d.label = label_;
    d.weights = weights_;
    return d;
  }
  std::vector<double> FinishDevice(const std::vector<double>& sums) const override { return {Average(sums[0])}; }
  void Init(const Metadata& md, data_size_t n) override {
    num_data_ = n;
    label_ = md.label();
    weights_ = md.weights();
    sum_w_ = 0;
    if (weights_) {
      for (data_size_t i = 0; i < n; ++i) sum_w_ += weights_[i];
    } else {
      sum_w_ = n;
    }
  }
  const std::vector<std::string>& GetName() const override { return name_; }
  double factor_to_bigger_better() const override { return factor_; }
  std::vector<double> Eval(const double* score, const ObjectiveFunction* obj) const override {
    double s = 0;
#pragma omp parallel for schedule(static) reduction(+ : s)
    for (data_size_t i = 0; i < num_data_; ++i) {
      double v = score[i];
      if (convert_ && obj != nullptr) obj->ConvertOutput(&score[i], &v);
      const double l = loss_(label_[i], v, cfg_);
      s += weights_ ? l * weights_[i] : l;
    }
    return {Average(s)};
  }
  virtual double Average(double s) const { return s / sum_w_; }

 protected:
  Config cfg_;
  PointLoss loss_;
  int device_kind_ = 0;
  double device_param_ = 0.0;
  bool convert_;
  double factor_;
  std::vector<std::string> name_;
  data_size_t num_data_ = 0;
  const label_t* label_ = nullptr;
  const label_t* weights_ = nullptr;
  double sum_w_ = 0;
};

class RMSEMetric : public PointwiseMetric {
 public:
  using PointwiseMetric::PointwiseMetric;
  double Average(double s) const override { return std::sqrt(s / sum_w_); }
};

class GammaDevianceMetric : public PointwiseMetric {
 public:
  using PointwiseMetric::PointwiseMetric;
  double Average(double s) const override { return s * 2; }
};

double L2Loss(label_t y, double s, const Config&) { return (s - y) * (s - y); }
double L1Loss(label_t y, double s, const Config&) { return std::fabs(s - y); }
double QuantileLoss(label_t y, double s, const Config& c) {
  double d = y - s;
  return d < 0 ? (c.alpha - 1.0f) * d : c.alpha * d;
}
double HuberLoss(label_t y, double s, const Config& c) {
  const double d = s - y;
  if (std::fabs(d) <= c.alpha) return 0.5f * d * d;
  return c.alpha * (std::fabs(d) - 0.5f * c.alpha);
}
double FairLoss(label_t y, double s, const Config& c) {
  const double x = std::fabs(s - y);
  return c.fair_c * x - c.fair_c * c.fair_c * std::log(1.0f + x / c.fair_c);
}
double PoissonLoss(label_t y, double s, const Config&) {
  const double eps = 1e-10f;
  if (s < eps) s = eps;
  return s - y * std::log(s);
}
double MapeLoss(label_t y, double s, const Config&) { return std::fabs(y - s) / std::max(1.0f, std::fabs(y)); }
double GammaLoss(label_t y, double s, const Config&) {
  const double psi = 1.0, theta = -1.0 / s, a = psi;
  const double b = -common::SafeLog(-theta);
  const double c = 1. / psi * common::SafeLog(y / psi) - common::SafeLog(static_cast<double>(y)) - 0;
  return -((y * theta - b) / a + c);
}
double GammaDevLoss(label_t y, double s, const Config&) {
  const double t = y / (s + 1.0e-9);
  return t - common::SafeLog(t) - 1;
}
double TweedieLoss(label_t y, double s, const Config& c) {
  const double rho = c.tweedie_variance_power;
  const double eps = 1e-10f;
  if (s < eps) s = eps;
  const double a = y * std::exp((1 - rho) * std::log(s)) / (1 - rho);
  const double b = std::exp((2 - rho) * std::log(s)) / (2 - rho);
  return -a + b;
}
double BinLogloss(label_t y, double p, const Config&) {
  if (y <= 0) {
    if (1.0f - p > kEpsilon) return -std::log(1.0f - p);
  } else {
    if (p > kEpsilon) return -std::log(p);
  }
  return -std::log(kEpsilon);
}
double BinError(label_t y, double p, const Config&) {
  if (p <= 0.5f) return y > 0;
  return y <= 0;
}
double XentLoss(label_t y, double p) {
  const double e = 1.0e-12;
  double a = y * (p > e ? std::log(p) : std::log(e));
  double b = (1.0f - y) * (1.0f - p > e ? std::log(1.0f - p) : std::log(e));
  return -(a + b);
}
double XentPoint(label_t y, double p, const Config&) { return XentLoss(y, p); }

// ----------------------------------------------------------------- AUC
class AUCMetric : public Metric {
 public:
  explicit AUCMetric(const Config&) { name_.push_back("auc"); }
  DeviceMetricSpec DeviceSpec(const ObjectiveFunction*) const override {
    DeviceMetricSpec d;
    d.kind = 6;  // AUC ranks raw scores (no output transform)
    d.nout = 2;  // tie-aware accumulator, positive weight
    d.label = label_;
    d.weights = weights_;
    return d;
  }
  std::vector<double> FinishDevice(const std::vector<double>& sums) const override {
    const double pos = sums[1];
    return {(pos > 0.0 && pos != sum_w_) ? sums[0] / (pos * (sum_w_ - pos)) : 1.0};
  }
  void Init(const Metadata& md, data_size_t n) override {
    num_data_ = n;
    label_ = md.label();
    weights_ = md.weights();
    sum_w_ = 0;
    if (weights_) {
      for (data_size_t i = 0; i < n; ++i) sum_w_ += weights_[i];
    } else {
      sum_w_ = n;
    }
  }
  const std::vector<std::string>& GetName() const override { return name_; }
  double factor_to_bigger_better() const override { return 1.0; }
  std::vector<double> Eval(const double* score, const ObjectiveFunction*) const override {
    std::vector<data_size_t> idx(num_data_);
    std::iota(idx.begin(), idx.end(), 0);
    std::sort(idx.begin(), idx.end(), [score](data_size_t a, data_size_t b) { return score[a] > score[b]; });
    double cur_pos = 0, sum_pos = 0, accum = 0, cur_neg = 0;
    double thr = num_data_ > 0 ? score[idx[0]] : 0;
    for (data_size_t k = 0; k < num_data_; ++k) {
      const data_size_t i = idx[k];
      if (score[i] != thr) {
        thr = score[i];
        accum += cur_neg * (cur_pos * 0.5f + sum_pos);
        sum_pos += cur_pos;
        cur_neg = cur_pos = 0;
      }
      const double w = weights_ ? weights_[i] : 1.0;
      cur_neg += (label_[i] <= 0) * w;
      cur_pos += (label_[i] > 0) * w;
    }
    accum += cur_neg * (cur_pos * 0.5f + sum_pos);
    sum_pos += cur_pos;
    double auc = 1.0;
    if (sum_pos > 0.0 && sum_pos != sum_w_) auc = accum / (sum_pos * (sum_w_ - sum_pos));
    return {auc};
  }

 private:
  std::vector<std::string> name_;
  data_size_t num_data_ = 0;
  const label_t* label_ = nullptr;
  const label_t* weights_ = nullptr;
  double sum_w_ = 0;
};

// ----------------------------------------------------------------- multiclass
class MulticlassMetric : public Metric {
 public:
  MulticlassMetric(const Config& cfg, bool is_error) : cfg_(cfg), is_error_(is_error), num_class_(cfg.num_class) {
    if (is_error) {
      name_.push_back(cfg.multi_error_top_k == 1 ? std::string("multi_error")
                                                  : "multi_error@" + std::to_string(cfg.multi_error_top_k));
    } else {
      name_.push_back("multi_logloss");
    }
  }
  void Init(const Metadata& md, data_size_t n) override {
    num_data_ = n;
    label_ = md.label();
    weights_ = md.weights();
    sum_w_ = 0;
    if (weights_) {
      for (data_size_t i = 0; i < n; ++i) sum_w_ += weights_[i];
    } else {
      sum_w_ = n;
    }
  }
  const std::vector<std::string>& GetName() const override { return name_; }
  double factor_to_bigger_better() const override { return -1.0; }
  DeviceMetricSpec DeviceSpec(const ObjectiveFunction* obj) const override {
    DeviceMetricSpec d;
    double param = 1.0;
    const int conv = obj != nullptr ? obj->DeviceOutputKind(&param) : 0;
    if (conv != 0 && conv != 4 && conv != 5) return d;
    d.kind = is_error_ ? 21 : 20;
    d.convert = conv;
    d.sigmoid = param;
    d.num_class = num_class_;
    d.top_k = cfg_.multi_error_top_k;
    d.label = label_;
    d.weights = weights_;
    return d;
  }
  std::vector<double> FinishDevice(const std::vector<double>& sums) const override { return {sums[0] / sum_w_}; }
  std::vector<double> Eval(const double* score, const ObjectiveFunction* obj) const override {
    double s = 0;
    const int nk = num_class_;
#pragma omp parallel for schedule(static) reduction(+ : s)
    for (data_size_t i = 0; i < num_data_; ++i) {
      std::vector<double> raw(nk), rec(nk);
      for (int k = 0; k < nk; ++k) raw[k] = score[static_cast<size_t>(num_data_) * k + i];
      if (obj) obj->ConvertOutput(raw.data(), rec.data());
      else rec = raw;
      const size_t y = static_cast<size_t>(label_[i]);
      double l;
      if (is_error_) {
        int larger = 0;
        l = 0.0;
        for (int k = 0; k < nk; ++k) {
          if (rec[k] >= rec[y]) ++larger;
          if (larger > cfg_.multi_error_top_k) { l = 1.0; break; }
        }
      } else {
        l = rec[y] > kEpsilon ? -std::log(rec[y]) : -std::log(kEpsilon);
      }
      s += weights_ ? l * weights_[i] : l;
    }
    return {s / sum_w_};
  }

 private:
  Config cfg_;
  bool is_error_;
  int num_class_;
  std::vector<std::string> name_;
  data_size_t num_data_ = 0;
  const label_t* label_ = nullptr;
  const label_t* weights_ = nullptr;
  double sum_w_ = 0;
};

class AucMuMetric : public Metric {
 public:
  explicit AucMuMetric(const Config& c) : num_class_(c.num_class), w_(c.auc_mu_weights_matrix) {
    name_.push_back("auc_mu");
  }
  DeviceMetricSpec DeviceSpec(const ObjectiveFunction*) const override {
    DeviceMetricSpec d;
    d.kind = 22;  // dev::kMetricAucMu: per class pair, the tie-aware binary AUC on the device
    d.num_class = num_class_;
    d.nout = num_class_ * (num_class_ - 1);  // (accumulator, class-j count) per pair
    d.label = label_;
    d.key = this;
    for (const auto& row : w_) d.qconst.insert(d.qconst.end(), row.begin(), row.end());
    if (static_cast<int>(d.qconst.size()) != num_class_ * num_class_) d.kind = 0;
    return d;
  }
  std::vector<double> FinishDevice(const std::vector<double>& sums) const override {
    std::vector<data_size_t> cs(num_class_, 0);
    for (data_size_t i = 0; i < num_data_; ++i) ++cs[static_cast<int>(label_[i])];
    double ans = 0;
    int pair = 0;
    for (int i = 0; i < num_class_; ++i) {
      for (int j = i + 1; j < num_class_; ++j, ++pair) ans += (sums[2 * pair] / cs[i]) / cs[j];
    }
    return {(2 * ans / num_class_) / (num_class_ - 1)};
  }
  void Init(const Metadata& md, data_size_t n) override {
    num_data_ = n;
    label_ = md.label();
    sorted_.resize(n);
    std::iota(sorted_.begin(), sorted_.end(), 0);
    std::stable_sort(sorted_.begin(), sorted_.end(), [this](data_size_t a, data_size_t b) { return label_[a] < label_[b]; });
  }
  const std::vector<std::string>& GetName() const override { return name_; }
  double factor_to_bigger_better() const override { return 1.0; }
  std::vector<double> Eval(const double* score, const ObjectiveFunction*) const override {
    std::vector<data_size_t> cs(num_class_, 0);
    for (data_size_t i = 0; i < num_data_; ++i) ++cs[static_cast<int>(label_[i])];
    std::vector<std::vector<double>> S(num_class_, std::vector<double>(num_class_, 0));
    int is = 0;
    for (int i = 0; i < num_class_; ++i) {
      int js = is + cs[i];
      for (int j = i + 1; j < num_class_; ++j) {
        std::vector<double> v(num_class_);
        for (int k = 0; k < num_class_; ++k) v[k] = w_[i][k] - w_[j][k];
        const double t1 = v[i] - v[j];
        std::vector<data_size_t> ij(sorted_.begin() + is, sorted_.begin() + is + cs[i]);
        ij.insert(ij.end(), sorted_.begin() + js, sorted_.begin() + js + cs[j]);
        std::vector<std::pair<data_size_t, double>> dist;
        for (data_size_t a : ij) {
          double va = 0;
          for (int m = 0; m < num_class_; ++m) va += v[m] * score[static_cast<size_t>(num_data_) * m + a];
          dist.emplace_back(a, t1 * va);
        }
        std::stable_sort(dist.begin(), dist.end(), [this](const std::pair<data_size_t, double>& a,
                                                          const std::pair<data_size_t, double>& b) {
          if (std::fabs(a.second - b.second) < kEpsilon) return label_[a.first] > label_[b.first];
          return a.second < b.second;
        });
        double num_j = 0, last = 0, cur_j = 0;
        for (auto& d : dist) {
          if (label_[d.first] == i) {
            S[i][j] += std::fabs(d.second - last) < kEpsilon ? num_j - 0.5 * cur_j : num_j;
          } else {
            ++num_j;
            if (std::fabs(d.second - last) < kEpsilon) {
              ++cur_j;
            } else {
              last = d.second;
              cur_j = 1;
            }
          }
        }
        js += cs[j];
      }
      is += cs[i];
    }
    double ans = 0;
    for (int i = 0; i < num_class_; ++i) {
      for (int j = i + 1; j < num_class_; ++j) ans += (S[i][j] / cs[i]) / cs[j];
    }
    ans = (2 * ans / num_class_) / (num_class_ - 1);
    return {ans};
  }

 private:
  int num_class_;
  std::vector<std::vector<double>> w_;
  std::vector<std::string> name_;
  data_size_t num_data_ = 0;
  const label_t* label_ = nullptr;
  std::vector<data_size_t> sorted_;
};

// ----------------------------------------------------------------- ranking
class QueryMetricBase : public Metric {
 public:
  void InitQueries(const Metadata& md, data_size_t n) {
    num_data_ = n;
    label_ = md.label();
    qb_ = md.query_boundaries();
    nq_ = md.num_queries();
    qw_ = md.query_weights();
    sum_qw_ = 0;
    if (qw_) {
      for (data_size_t q = 0; q < nq_; ++q) sum_qw_ += qw_[q];
    } else {
      sum_qw_ = nq_;
    }
  }
  const std::vector<std::string>& GetName() const override { return name_; }
  double factor_to_bigger_better() const override { return 1.0; }
  std::vector<double> FinishDevice(const std::vector<double>& sums) const override {
    std::vector<double> r(sums);
    for (auto& v : r) v /= sum_qw_;
    return r;
  }

 protected:
  DeviceMetricSpec QuerySpec(int kind) const {
    DeviceMetricSpec d;
    if (qb_ == nullptr || nq_ <= 0) return d;
    for (data_size_t q = 0; q < nq_; ++q) d.max_query_docs = std::max(d.max_query_docs, qb_[q + 1] - qb_[q]);
    d.kind = kind;
    d.nout = static_cast<int>(eval_at_.size());
    d.label = label_;
    d.key = this;
    d.qb = qb_;
    d.nq = nq_;
    d.qw = qw_;
    d.eval_at.assign(eval_at_.begin(), eval_at_.end());
    return d;
  }
  // queries of up to this many documents are staged in LDS by the device kernel (kRankMaxDocs);
  // longer ones take its global-scratch variant
  static constexpr data_size_t kDeviceMaxQueryDocs = 2048;
  std::vector<std::string> name_;
  std::vector<data_size_t> eval_at_;
  data_size_t num_data_ = 0, nq_ = 0;
  const label_t* label_ = nullptr;
  const data_size_t* qb_ = nullptr;
  const label_t* qw_ = nullptr;
  double sum_qw_ = 0;
};

class NDCGMetric : public QueryMetricBase {
 public:
  explicit NDCGMetric(const Config& c) {
    std::vector<int> at = c.eval_at;
    DCG::DefaultEvalAt(&at);
    eval_at_.assign(at.begin(), at.end());
    auto gain = c.label_gain;
    DCG::DefaultLabelGain(&gain);
    DCG::Init(gain);
  }
  void Init(const Metadata& md, data_size_t n) override {
    for (auto k : eval_at_) name_.push_back("ndcg@" + std::to_string(k));
    InitQueries(md, n);
    DCG::CheckLabel(label_, n);
    if (qb_ == nullptr) Log::Fatal("The NDCG metric requires query information");
    inv_max_.assign(nq_, std::vector<double>(eval_at_.size(), 0.0));
#pragma omp parallel for schedule(static)
    for (data_size_t q = 0; q < nq_; ++q) {
      DCG::MaxDCG(eval_at_, label_ + qb_[q], qb_[q + 1] - qb_[q], &inv_max_[q]);
      for (auto& v : inv_max_[q]) v = v > 0.0 ? 1.0 / v : -1.0;
    }
  }
  DeviceMetricSpec DeviceSpec(const ObjectiveFunction*) const override {
    DeviceMetricSpec d = QuerySpec(30);
    if (d.kind == 0) return d;
    const size_t K = eval_at_.size();
    d.qconst.resize(static_cast<size_t>(nq_) * K);
    for (data_size_t q = 0; q < nq_; ++q) {
      for (size_t j = 0; j < K; ++j) d.qconst[q * K + j] = inv_max_[q][j];
    }
    d.label_gain = DCG::label_gain();
    d.discount.resize(std::max(kDeviceMaxQueryDocs, d.max_query_docs));
    for (size_t i = 0; i < d.discount.size(); ++i) d.discount[i] = DCG::Discount(static_cast<data_size_t>(i));
    return d;
  }
  std::vector<double> Eval(const double* score, const ObjectiveFunction*) const override {
    const size_t K = eval_at_.size();
    const int nt = omp_get_max_threads();
    std::vector<std::vector<double>> buf(nt, std::vector<double>(K, 0.0));
#pragma omp parallel
    {
      std::vector<double> tmp(K, 0.0);
      const int tid = omp_get_thread_num();
#pragma omp for schedule(static)
      for (data_size_t q = 0; q < nq_; ++q) {
        const double w = qw_ ? qw_[q] : 1.0;
        if (inv_max_[q][0] <= 0.0) {
          for (size_t j = 0; j < K; ++j) buf[tid][j] += 1.0 * w;
        } else {
          DCG::DCGAt(eval_at_, label_ + qb_[q], score + qb_[q], qb_[q + 1] - qb_[q], &tmp);
          for (size_t j = 0; j < K; ++j) buf[tid][j] += tmp[j] * inv_max_[q][j] * w;
        }
      }
    }
    std::vector<double> r(K, 0.0);
    for (size_t j = 0; j < K; ++j) {
      for (int t = 0; t < nt; ++t) r[j] += buf[t][j];
      r[j] /= sum_qw_;
    }
    return r;
  }

 private:
  std::vector<std::vector<double>> inv_max_;
};

class MapMetric : public QueryMetricBase {
 public:
  explicit MapMetric(const Config& c) {
    std::vector<int> at = c.eval_at;
    DCG::DefaultEvalAt(&at);
    eval_at_.assign(at.begin(), at.end());
  }
  void Init(const Metadata& md, data_size_t n) override {
    for (auto k : eval_at_) name_.push_back("map@" + std::to_string(k));
    InitQueries(md, n);
    if (qb_ == nullptr) Log::Fatal("For MAP metric, there should be query information");
    npos_.assign(nq_, 0);
    for (data_size_t q = 0; q < nq_; ++q) {
      for (data_size_t j = qb_[q]; j < qb_[q + 1]; ++j) {
        if (label_[j] > 0.5f) ++npos_[q];
      }
    }
  }
  void MapAt(data_size_t npos, const label_t* label, const double* score, data_size_t n, std::vector<double>* out) const {
    std::vector<data_size_t> idx(n);
    std::iota(idx.begin(), idx.end(), 0);
    std::stable_sort(idx.begin(), idx.end(), [score](data_size_t a, data_size_t b) { return score[a] > score[b]; });
    int hit = 0;
    double sum_ap = 0;
    data_size_t left = 0;
    for (size_t i = 0; i < eval_at_.size(); ++i) {
      data_size_t k = std::min(eval_at_[i], n);
      for (data_size_t j = left; j < k; ++j) {
        if (label[idx[j]] > 0.5f) {
          ++hit;
          sum_ap += static_cast<double>(hit) / (j + 1.0f);
        }
      }
      (*out)[i] = npos > 0 ? sum_ap / std::min(npos, k) : 1.0;
      left = k;
    }
  }
  DeviceMetricSpec DeviceSpec(const ObjectiveFunction*) const override {
    DeviceMetricSpec d = QuerySpec(31);
    if (d.kind == 0) return d;
    d.qconst.assign(npos_.begin(), npos_.end());
    return d;
  }
  std::vector<double> Eval(const double* score, const ObjectiveFunction*) const override {
    const size_t K = eval_at_.size();
    const int nt = omp_get_max_threads();
    std::vector<std::vector<double>> buf(nt, std::vector<double>(K, 0.0));
#pragma omp parallel
    {
      std::vector<double> tmp(K, 0.0);
      const int tid = omp_get_thread_num();
#pragma omp for schedule(guided)
      for (data_size_t q = 0; q < nq_; ++q) {
        MapAt(npos_[q], label_ + qb_[q], score + qb_[q], qb_[q + 1] - qb_[q], &tmp);
        const double w = qw_ ? qw_[q] : 1.0;
        for (size_t j = 0; j < K; ++j) buf[tid][j] += tmp[j] * w;
      }
    }
    std::vector<double> r(K, 0.0);
    for (size_t j = 0; j < K; ++j) {
      for (int t = 0; t < nt; ++t) r[j] += buf[t][j];
      r[j] /= sum_qw_;
    }
    return r;
  }

 private:
  std::vector<data_size_t> npos_;
};

// ----------------------------------------------------------------- cross-entropy family
class XentLambdaMetric : public Metric {
 public:
  explicit XentLambdaMetric(const Config&) { name_.push_back("cross_entropy_lambda"); }
  void Init(const Metadata& md, data_size_t n) override {
    num_data_ = n;
    label_ = md.label();
    weights_ = md.weights();
  }
  const std::vector<std::string>& GetName() const override { return name_; }
  double factor_to_bigger_better() const override { return -1.0; }
  std::vector<double> Eval(const double* score, const ObjectiveFunction* obj) const override {
    double s = 0;
#pragma omp parallel for schedule(static) reduction(+ : s)
    for (data_size_t i = 0; i < num_data_; ++i) {
      double hhat;
      if (obj == nullptr) hhat = std::log(1.0f + std::exp(score[i]));
      else obj->ConvertOutput(&score[i], &hhat);
      const double w = weights_ ? weights_[i] : 1.0f;
      s += XentLoss(label_[i], 1.0f - std::exp(-w * hhat));
    }
    return {s / static_cast<double>(num_data_)};
  }

 private:
  std::vector<std::string> name_;
  data_size_t num_data_ = 0;
  const label_t* label_ = nullptr;
  const label_t* weights_ = nullptr;
};

class KLMetric : public PointwiseMetric {
 public:
  explicit KLMetric(const Config& c) : PointwiseMetric(c, "kullback_leibler", XentPoint, true, -1.0) {}
  void Init(const Metadata& md, data_size_t n) override {
    PointwiseMetric::Init(md, n);
    pre_ = 0;
    for (data_size_t i = 0; i < n; ++i) {
      double p = label_[i], hp = 0;
      if (p > 0) hp += p * std::log(p);
      double q = 1.0f - p;
      if (q > 0) hp += q * std::log(q);
      pre_ += weights_ ? hp * weights_[i] : hp;
    }
    pre_ /= sum_w_;
  }
  double Average(double s) const override { return pre_ + s / sum_w_; }

 private:
  double pre_ = 0;
};

}  // namespace

Metric* Metric::CreateMetric(const std::string& t, const Config& c) {
  if (t == "l2") return new PointwiseMetric(c, "l2", L2Loss, true, -1.0);
  if (t == "rmse") return new RMSEMetric(c, "rmse", L2Loss, true, -1.0);
  if (t == "l1") return new PointwiseMetric(c, "l1", L1Loss, true, -1.0);
  if (t == "quantile") return new PointwiseMetric(c, "quantile", QuantileLoss, true, -1.0);
  if (t == "huber") return new PointwiseMetric(c, "huber", HuberLoss, true, -1.0);
  if (t == "fair") return new PointwiseMetric(c, "fair", FairLoss, true, -1.0);
  if (t == "poisson") return new PointwiseMetric(c, "poisson", PoissonLoss, true, -1.0);
  if (t == "binary_logloss") return new PointwiseMetric(c, "binary_logloss", BinLogloss, true, -1.0);
  if (t == "binary_error") return new PointwiseMetric(c, "binary_error", BinError, true, -1.0);
  if (t == "auc") return new AUCMetric(c);
  if (t == "auc_mu") return new AucMuMetric(c);
  if (t == "ndcg") return new NDCGMetric(c);
  if (t == "map") return new MapMetric(c);
  if (t == "multi_logloss") return new MulticlassMetric(c, false);
  if (t == "multi_error") return new MulticlassMetric(c, true);
  if (t == "cross_entropy") return new PointwiseMetric(c, "cross_entropy", XentPoint, true, -1.0);
  if (t == "cross_entropy_lambda") return new XentLambdaMetric(c);
  if (t == "kullback_leibler") return new KLMetric(c);
  if (t == "mape") return new PointwiseMetric(c, "mape", MapeLoss, true, -1.0);
  if (t == "gamma") return new PointwiseMetric(c, "gamma", GammaLoss, true, -1.0);
  if (t == "gamma_deviance") return new GammaDevianceMetric(c, "gamma_deviance", GammaDevLoss, true, -1.0);
  if (t == "tweedie") return new PointwiseMetric(c, "tweedie", TweedieLoss, true, -1.0);
  return nullptr;
}

}  // namespace lgbm_amd
