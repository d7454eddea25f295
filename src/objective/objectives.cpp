// All objective functions.  Gradient formulas, init scores (BoostFromScore), leaf
// renewal (weighted percentiles) and model strings follow the reference
// (src/objective/{regression,binary,multiclass,xentropy,rank}_objective.hpp); point-wise
// objectives also describe themselves to the HIP gradient kernel (DeviceSpec).
#include <algorithm>
#include <cmath>
#include <numeric>
#include <sstream>

#include "lgbm_amd/common.h"
#include "lgbm_amd/dcg.h"
#include "lgbm_amd/log.h"
#include "lgbm_amd/network.h"
#include "lgbm_amd/objective.h"
#include "lgbm_amd/random.h"

namespace lgbm_amd {

namespace {

// unweighted percentile with linear interpolation between the (pos)th and (pos+1)th
// largest values, pos = floor((1 - alpha) * n)  (reference PercentileFun)
template <typename Reader>
double Percentile(const Reader& rd, data_size_t n, double alpha) {
  if (n <= 1) return rd(0);
  std::vector<double> v(n);
  for (data_size_t i = 0; i < n; ++i) v[i] = rd(i);
  const double fpos = (1.0f - alpha) * n;
  const data_size_t pos = static_cast<data_size_t>(fpos);
  if (pos < 1) return *std::max_element(v.begin(), v.end());
  if (pos >= n) return *std::min_element(v.begin(), v.end());
  const double bias = fpos - pos;
  std::nth_element(v.begin(), v.begin() + (pos - 1), v.end(), std::greater<double>());
  const double v1 = v[pos - 1];
  const double v2 = *std::max_element(v.begin() + pos, v.end());
  return v1 - (v1 - v2) * bias;
}

template <typename Reader, typename WReader>
double WeightedPercentile(const Reader& rd, const WReader& wr, data_size_t n, double alpha) {
  if (n <= 1) return rd(0);
  std::vector<data_size_t> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](data_size_t a, data_size_t b) { return rd(a) < rd(b); });
  std::vector<double> cdf(n);
  cdf[0] = wr(idx[0]);
  for (data_size_t i = 1; i < n; ++i) cdf[i] = cdf[i - 1] + wr(idx[i]);
  const double thr = cdf[n - 1] * alpha;
  size_t pos = std::upper_bound(cdf.begin(), cdf.end(), thr) - cdf.begin();
  pos = std::min(pos, static_cast<size_t>(n - 1));
  if (pos == 0 || pos == static_cast<size_t>(n - 1)) return rd(idx[pos]);
  const double v1 = rd(idx[pos - 1]);
  const double v2 = rd(idx[pos]);
  if (cdf[pos + 1] - cdf[pos] >= 1.0f) return (thr - cdf[pos]) / (cdf[pos + 1] - cdf[pos]) * (v2 - v1) + v1;
  return v2;
}

std::vector<std::string> Tokens(const std::string& s) { return common::Split(s.c_str(), ' '); }

double ParseKey(const std::vector<std::string>& toks, const char* key, double dflt) {
  for (auto& t : toks) {
    auto kv = common::Split(t.c_str(), ':');
    if (kv.size() == 2 && kv[0] == key) {
      double v = dflt;
      common::Atof(kv[1].c_str(), &v);
      return v;
    }
  }
  return dflt;
}

bool HasToken(const std::vector<std::string>& toks, const char* t) {
  return std::find(toks.begin(), toks.end(), std::string(t)) != toks.end();
}

// ------------------------------------------------------------------ regression family
class RegressionL2 : public ObjectiveFunction {
 public:
  explicit RegressionL2(const Config& c) : sqrt_(c.reg_sqrt) {}
  explicit RegressionL2(const std::vector<std::string>& t) : sqrt_(HasToken(t, "sqrt")) {}
  void Init(const Metadata& md, data_size_t n) override {
    num_data_ = n;
    label_ = md.label();
    if (sqrt_) {
      trans_.resize(n);
      for (data_size_t i = 0; i < n; ++i) trans_[i] = common::Sign(label_[i]) * std::sqrt(std::fabs(label_[i]));
      label_ = trans_.data();
    }
    weights_ = md.weights();
  }
  void GetGradients(const double* s, score_t* g, score_t* h) const override {
#pragma omp parallel for schedule(static)
    for (data_size_t i = 0; i < num_data_; ++i) {
      const double w = weights_ ? weights_[i] : 1.0;
      g[i] = static_cast<score_t>((s[i] - label_[i]) * w);
      h[i] = static_cast<score_t>(w);
    }
  }
  const char* GetName() const override { return "regression"; }
  void ConvertOutput(const double* in, double* out) const override {
    out[0] = sqrt_ ? common::Sign(in[0]) * in[0] * in[0] : in[0];
  }
  int DeviceOutputKind(double*) const override { return sqrt_ ? 2 : 0; }
  std::string ToString() const override { return std::string(GetName()) + (sqrt_ ? " sqrt" : ""); }
  bool IsConstantHessian() const override { return weights_ == nullptr; }
  double BoostFromScore(int) const override {
    double sl = 0, sw = 0;
    if (weights_) {
#pragma omp parallel for schedule(static) reduction(+ : sl, sw)
      for (data_size_t i = 0; i < num_data_; ++i) {
        sl += label_[i] * weights_[i];
        sw += weights_[i];
      }
    } else {
      sw = static_cast<double>(num_data_);
#pragma omp parallel for schedule(static) reduction(+ : sl)
      for (data_size_t i = 0; i < num_data_; ++i) sl += label_[i];
    }
    return sl / sw;
  }
  DeviceGradSpec DeviceSpec() const override { return Spec(DeviceGradKind::L2); }

 protected:
  DeviceGradSpec Spec(DeviceGradKind k) const {
    DeviceGradSpec d;
    d.kind = k;
    d.label = label_;
    d.weights = weights_;
    return d;
  }
  bool sqrt_;
  data_size_t num_data_ = 0;
  const label_t* weights_ = nullptr;
  std::vector<label_t> trans_;
};

class RegressionL1 : public RegressionL2 {
 public:
  using RegressionL2::RegressionL2;
  void GetGradients(const double* s, score_t* g, score_t* h) const override {
#pragma omp parallel for schedule(static)
    for (data_size_t i = 0; i < num_data_; ++i) {
      const double w = weights_ ? weights_[i] : 1.0;
      g[i] = static_cast<score_t>(common::Sign(s[i] - label_[i]) * w);
      h[i] = static_cast<score_t>(w);
    }
  }
  double BoostFromScore(int) const override {
    auto rd = [this](data_size_t i) { return static_cast<double>(label_[i]); };
    if (weights_) {
      auto wr = [this](data_size_t i) { return static_cast<double>(weights_[i]); };
      return static_cast<label_t>(WeightedPercentile(rd, wr, num_data_, 0.5));
    }
    return static_cast<label_t>(Percentile(rd, num_data_, 0.5));
  }
  bool IsConstantHessian() const override { return false; }
  bool IsRenewTreeOutput() const override { return true; }
  double RenewTreeOutput(double, const std::function<double(const label_t*, int)>& res, const data_size_t* im,
                         const data_size_t* bm, data_size_t n) const override {
    auto rd = [&](data_size_t i) { return res(label_, bm ? bm[im[i]] : im[i]); };
    if (weights_) {
      auto wr = [&](data_size_t i) { return static_cast<double>(weights_[bm ? bm[im[i]] : im[i]]); };
      return WeightedPercentile(rd, wr, n, 0.5);
    }
    return Percentile(rd, n, 0.5);
  }
  bool DeviceRenew(DeviceRenewSpec* d) const override {
    d->alpha = 0.5;
    d->label = label_;
    d->weights = weights_;
    return !sqrt_;
  }
  const char* GetName() const override { return "regression_l1"; }
  std::string ToString() const override { return std::string(GetName()) + (sqrt_ ? " sqrt" : ""); }
  DeviceGradSpec DeviceSpec() const override { return Spec(DeviceGradKind::L1); }
};

class Huber : public RegressionL2 {
 public:
  explicit Huber(const Config& c) : RegressionL2(c), alpha_(c.alpha) {
    if (sqrt_) {
      Log::Warning("Cannot use sqrt transform in %s Regression, will auto disable it", GetName());
      sqrt_ = false;
    }
  }
  explicit Huber(const std::vector<std::string>& t) : RegressionL2(t), alpha_(0.9) { sqrt_ = false; }
  void GetGradients(const double* s, score_t* g, score_t* h) const override {
#pragma omp parallel for schedule(static)
    for (data_size_t i = 0; i < num_data_; ++i) {
      const double w = weights_ ? weights_[i] : 1.0;
      const double d = s[i] - label_[i];
      g[i] = static_cast<score_t>((std::fabs(d) <= alpha_ ? d : common::Sign(d) * alpha_) * w);
      h[i] = static_cast<score_t>(w);
    }
  }
  const char* GetName() const override { return "huber"; }
  std::string ToString() const override { return GetName(); }
  bool IsConstantHessian() const override { return false; }
  DeviceGradSpec DeviceSpec() const override {
    auto d = Spec(DeviceGradKind::Huber);
    d.p0 = alpha_;
    return d;
  }

 private:
  double alpha_;
};

class Fair : public RegressionL2 {
 public:
  explicit Fair(const Config& c) : RegressionL2(c), c_(c.fair_c) {}
  explicit Fair(const std::vector<std::string>& t) : RegressionL2(t), c_(1.0) {}
  void GetGradients(const double* s, score_t* g, score_t* h) const override {
#pragma omp parallel for schedule(static)
    for (data_size_t i = 0; i < num_data_; ++i) {
      const double w = weights_ ? weights_[i] : 1.0;
      const double x = s[i] - label_[i];
      g[i] = static_cast<score_t>(c_ * x / (std::fabs(x) + c_) * w);
      h[i] = static_cast<score_t>(c_ * c_ / ((std::fabs(x) + c_) * (std::fabs(x) + c_)) * w);
    }
  }
  const char* GetName() const override { return "fair"; }
  std::string ToString() const override { return GetName(); }
  bool IsConstantHessian() const override { return false; }
  DeviceGradSpec DeviceSpec() const override {
    auto d = Spec(DeviceGradKind::Fair);
    d.p0 = c_;
    return d;
  }

 private:
  double c_;
};

class Poisson : public RegressionL2 {
 public:
  explicit Poisson(const Config& c) : RegressionL2(c), max_delta_step_(c.poisson_max_delta_step) {
    if (sqrt_) {
      Log::Warning("Cannot use sqrt transform in %s Regression, will auto disable it", GetName());
      sqrt_ = false;
    }
  }
  explicit Poisson(const std::vector<std::string>& t) : RegressionL2(t), max_delta_step_(0.7) { sqrt_ = false; }
  void Init(const Metadata& md, data_size_t n) override {
    sqrt_ = false;
    RegressionL2::Init(md, n);
    double sum = 0;
    label_t mn = label_[0];
    for (data_size_t i = 0; i < n; ++i) {
      mn = std::min(mn, label_[i]);
      sum += label_[i];
    }
    if (mn < 0.0f) Log::Fatal("[%s]: at least one target label is negative", GetName());
    if (sum == 0.0) Log::Fatal("[%s]: sum of labels is zero", GetName());
  }
  void GetGradients(const double* s, score_t* g, score_t* h) const override {
#pragma omp parallel for schedule(static)
    for (data_size_t i = 0; i < num_data_; ++i) {
      const double w = weights_ ? weights_[i] : 1.0;
      g[i] = static_cast<score_t>((std::exp(s[i]) - label_[i]) * w);
      h[i] = static_cast<score_t>(std::exp(s[i] + max_delta_step_) * w);
    }
  }
  void ConvertOutput(const double* in, double* out) const override { out[0] = std::exp(in[0]); }
  int DeviceOutputKind(double*) const override { return 3; }
  const char* GetName() const override { return "poisson"; }
  std::string ToString() const override { return GetName(); }
  double BoostFromScore(int) const override { return common::SafeLog(RegressionL2::BoostFromScore(0)); }
  bool IsConstantHessian() const override { return false; }
  DeviceGradSpec DeviceSpec() const override {
    auto d = Spec(DeviceGradKind::Poisson);
    d.p0 = max_delta_step_;
    return d;
  }

 protected:
  double max_delta_step_;
};

class Quantile : public RegressionL2 {
 public:
  explicit Quantile(const Config& c) : RegressionL2(c), alpha_(static_cast<score_t>(c.alpha)) {
    LGBM_CHECK(alpha_ > 0 && alpha_ < 1);
  }
  explicit Quantile(const std::vector<std::string>& t) : RegressionL2(t), alpha_(0.9f) {}
  void GetGradients(const double* s, score_t* g, score_t* h) const override {
#pragma omp parallel for schedule(static)
    for (data_size_t i = 0; i < num_data_; ++i) {
      const score_t d = static_cast<score_t>(s[i] - label_[i]);
      const double w = weights_ ? weights_[i] : 1.0;
      if (weights_) {
        g[i] = static_cast<score_t>((d >= 0 ? (1.0f - alpha_) : -alpha_) * w);
        h[i] = static_cast<score_t>(w);
      } else {
        g[i] = d >= 0 ? (1.0f - alpha_) : -alpha_;
        h[i] = 1.0f;
      }
    }
  }
  const char* GetName() const override { return "quantile"; }
  std::string ToString() const override { return GetName(); }
  bool IsConstantHessian() const override { return weights_ == nullptr; }
  double BoostFromScore(int) const override {
    auto rd = [this](data_size_t i) { return static_cast<double>(label_[i]); };
    if (weights_) {
      auto wr = [this](data_size_t i) { return static_cast<double>(weights_[i]); };
      return static_cast<label_t>(WeightedPercentile(rd, wr, num_data_, alpha_));
    }
    return static_cast<label_t>(Percentile(rd, num_data_, alpha_));
  }
  bool IsRenewTreeOutput() const override { return true; }
  double RenewTreeOutput(double, const std::function<double(const label_t*, int)>& res, const data_size_t* im,
                         const data_size_t* bm, data_size_t n) const override {
    auto rd = [&](data_size_t i) { return res(label_, bm ? bm[im[i]] : im[i]); };
    if (weights_) {
      auto wr = [&](data_size_t i) { return static_cast<double>(weights_[bm ? bm[im[i]] : im[i]]); };
      return WeightedPercentile(rd, wr, n, alpha_);
    }
    return Percentile(rd, n, alpha_);
  }
  bool DeviceRenew(DeviceRenewSpec* d) const override {
    d->alpha = alpha_;
    d->label = label_;
    d->weights = weights_;
    return !sqrt_;
  }
  DeviceGradSpec DeviceSpec() const override {
    auto d = Spec(DeviceGradKind::Quantile);
    d.p0 = alpha_;
    return d;
  }

 private:
  score_t alpha_;
};

class Mape : public RegressionL1 {
 public:
  using RegressionL1::RegressionL1;
  void Init(const Metadata& md, data_size_t n) override {
    RegressionL2::Init(md, n);
    for (data_size_t i = 0; i < n; ++i) {
      if (std::fabs(label_[i]) < 1) {
        Log::Warning("Met 'abs(label) < 1', will convert them to '1' in MAPE objective and metric");
        break;
      }
    }
    lw_.resize(n);
    for (data_size_t i = 0; i < n; ++i) {
      lw_[i] = 1.0f / std::max(1.0f, std::fabs(label_[i])) * (weights_ ? weights_[i] : 1.0f);
    }
  }
  void GetGradients(const double* s, score_t* g, score_t* h) const override {
#pragma omp parallel for schedule(static)
    for (data_size_t i = 0; i < num_data_; ++i) {
      g[i] = static_cast<score_t>(common::Sign(s[i] - label_[i]) * lw_[i]);
      h[i] = weights_ ? weights_[i] : 1.0f;
    }
  }
  double BoostFromScore(int) const override {
    auto rd = [this](data_size_t i) { return static_cast<double>(label_[i]); };
    auto wr = [this](data_size_t i) { return static_cast<double>(lw_[i]); };
    return static_cast<label_t>(WeightedPercentile(rd, wr, num_data_, 0.5));
  }
  double RenewTreeOutput(double, const std::function<double(const label_t*, int)>& res, const data_size_t* im,
                         const data_size_t* bm, data_size_t n) const override {
    auto rd = [&](data_size_t i) { return res(label_, bm ? bm[im[i]] : im[i]); };
    auto wr = [&](data_size_t i) { return static_cast<double>(lw_[bm ? bm[im[i]] : im[i]]); };
    return WeightedPercentile(rd, wr, n, 0.5);
  }
  bool DeviceRenew(DeviceRenewSpec* d) const override {
    d->alpha = 0.5;
    d->label = label_;
    d->weights = lw_.data();
    return !sqrt_;
  }
  const char* GetName() const override { return "mape"; }
  std::string ToString() const override { return GetName(); }
  bool IsConstantHessian() const override { return true; }
  DeviceGradSpec DeviceSpec() const override {
    auto d = Spec(DeviceGradKind::Mape);
    d.label_weight_arr = lw_.data();
    return d;
  }

 private:
  std::vector<label_t> lw_;
};

class Gamma : public Poisson {
 public:
  using Poisson::Poisson;
  void GetGradients(const double* s, score_t* g, score_t* h) const override {
#pragma omp parallel for schedule(static)
    for (data_size_t i = 0; i < num_data_; ++i) {
      if (weights_) {
        g[i] = static_cast<score_t>(1.0 - label_[i] / std::exp(s[i]) * weights_[i]);
        h[i] = static_cast<score_t>(label_[i] / std::exp(s[i]) * weights_[i]);
      } else {
        g[i] = static_cast<score_t>(1.0 - label_[i] / std::exp(s[i]));
        h[i] = static_cast<score_t>(label_[i] / std::exp(s[i]));
      }
    }
  }
  const char* GetName() const override { return "gamma"; }
  std::string ToString() const override { return GetName(); }
  DeviceGradSpec DeviceSpec() const override { return Spec(DeviceGradKind::Gamma); }
};

class Tweedie : public Poisson {
 public:
  explicit Tweedie(const Config& c) : Poisson(c), rho_(c.tweedie_variance_power) {}
  explicit Tweedie(const std::vector<std::string>& t) : Poisson(t), rho_(1.5) {}
  void GetGradients(const double* s, score_t* g, score_t* h) const override {
#pragma omp parallel for schedule(static)
    for (data_size_t i = 0; i < num_data_; ++i) {
      const double w = weights_ ? weights_[i] : 1.0;
      const double e1 = std::exp((1 - rho_) * s[i]), e2 = std::exp((2 - rho_) * s[i]);
      g[i] = static_cast<score_t>((-label_[i] * e1 + e2) * w);
      h[i] = static_cast<score_t>((-label_[i] * (1 - rho_) * e1 + (2 - rho_) * e2) * w);
    }
  }
  const char* GetName() const override { return "tweedie"; }
  std::string ToString() const override { return GetName(); }
  DeviceGradSpec DeviceSpec() const override {
    auto d = Spec(DeviceGradKind::Tweedie);
    d.p0 = rho_;
    return d;
  }

 private:
  double rho_;
};

// ------------------------------------------------------------------ binary
class BinaryLogloss : public ObjectiveFunction {
 public:
  explicit BinaryLogloss(const Config& c, int pos_class = -1)
      : sigmoid_(c.sigmoid), is_unbalance_(c.is_unbalance), scale_pos_weight_(c.scale_pos_weight),
        pos_class_(pos_class) {
    if (sigmoid_ <= 0.0) Log::Fatal("Sigmoid parameter %f should be greater than zero", sigmoid_);
    if (is_unbalance_ && std::fabs(scale_pos_weight_ - 1.0f) > 1e-6) {
      Log::Fatal("Cannot set is_unbalance and scale_pos_weight at the same time");
    }
  }
  explicit BinaryLogloss(const std::vector<std::string>& t) : sigmoid_(ParseKey(t, "sigmoid", -1)) {
    if (sigmoid_ <= 0.0) Log::Fatal("Sigmoid parameter %f should be greater than zero", sigmoid_);
  }
  bool IsPos(label_t l) const { return pos_class_ < 0 ? l > 0 : static_cast<int>(l) == pos_class_; }
  void Init(const Metadata& md, data_size_t n) override {
    num_data_ = n;
    label_ = md.label();
    weights_ = md.weights();
    data_size_t pos = 0, neg = 0;
#pragma omp parallel for schedule(static) reduction(+ : pos, neg)
    for (data_size_t i = 0; i < n; ++i) {
      if (IsPos(label_[i])) ++pos;
      else ++neg;
    }
    num_pos_ = pos;
    if (Network::num_machines() > 1) {
      pos = Network::GlobalSyncUpBySum(pos);
      neg = Network::GlobalSyncUpBySum(neg);
    }
    need_train_ = true;
    if (neg == 0 || pos == 0) {
      Log::Warning("Contains only one class");
      need_train_ = false;
    }
    Log::Info("Number of positive: %d, number of negative: %d", pos, neg);
    lw_[0] = lw_[1] = 1.0;
    if (is_unbalance_ && pos > 0 && neg > 0) {
      if (pos > neg) lw_[0] = static_cast<double>(pos) / neg;
      else lw_[1] = static_cast<double>(neg) / pos;
    }
    lw_[1] *= scale_pos_weight_;
    if (pos_class_ >= 0) {
      // one-vs-all class labels for the device kernel
      bin_label_.resize(n);
      for (data_size_t i = 0; i < n; ++i) bin_label_[i] = IsPos(label_[i]) ? 1.0f : 0.0f;
    }
  }
  void GetGradients(const double* s, score_t* g, score_t* h) const override {
    if (!need_train_) return;
#pragma omp parallel for schedule(static)
    for (data_size_t i = 0; i < num_data_; ++i) {
      const int is_pos = IsPos(label_[i]);
      const int lab = is_pos ? 1 : -1;
      const double lw = lw_[is_pos];
      const double resp = -lab * sigmoid_ / (1.0f + std::exp(lab * sigmoid_ * s[i]));
      const double ar = std::fabs(resp);
      const double w = weights_ ? weights_[i] : 1.0;
      g[i] = static_cast<score_t>(resp * lw * w);
      h[i] = static_cast<score_t>(ar * (sigmoid_ - ar) * lw * w);
    }
  }
  double BoostFromScore(int) const override {
    double sl = 0, sw = 0;
    if (weights_) {
#pragma omp parallel for schedule(static) reduction(+ : sl, sw)
      for (data_size_t i = 0; i < num_data_; ++i) {
        sl += IsPos(label_[i]) * weights_[i];
        sw += weights_[i];
      }
    } else {
      sw = static_cast<double>(num_data_);
#pragma omp parallel for schedule(static) reduction(+ : sl)
      for (data_size_t i = 0; i < num_data_; ++i) sl += IsPos(label_[i]);
    }
    double p = sl / sw;
    p = std::min(p, 1.0 - kEpsilon);
    p = std::max<double>(p, kEpsilon);
    double init = std::log(p / (1.0f - p)) / sigmoid_;
    Log::Info("[%s:%s]: pavg=%f -> initscore=%f", GetName(), "BoostFromScore", p, init);
    return init;
  }
  bool ClassNeedTrain(int) const override { return need_train_; }
  const char* GetName() const override { return "binary"; }
  void ConvertOutput(const double* in, double* out) const override {
    out[0] = 1.0f / (1.0f + std::exp(-sigmoid_ * in[0]));
  }
  int DeviceOutputKind(double* param) const override {
    *param = sigmoid_;
    return 1;
  }
  std::string ToString() const override {
    std::stringstream s;
    s << GetName() << " sigmoid:" << sigmoid_;
    return s.str();
  }
  bool SkipEmptyClass() const override { return true; }
  bool NeedAccuratePrediction() const override { return false; }
  data_size_t NumPositiveData() const override { return num_pos_; }
  DeviceGradSpec DeviceSpec() const override {
    DeviceGradSpec d;
    d.kind = need_train_ ? DeviceGradKind::Binary : DeviceGradKind::None;
    d.p0 = sigmoid_;
    d.label_weight[0] = lw_[0];
    d.label_weight[1] = lw_[1];
    d.label = pos_class_ >= 0 ? bin_label_.data() : label_;
    d.weights = weights_;
    return d;
  }

 private:
  double sigmoid_;
  bool is_unbalance_ = false;
  double scale_pos_weight_ = 1.0;
  int pos_class_ = -1;
  data_size_t num_data_ = 0;
  data_size_t num_pos_ = 0;
  const label_t* weights_ = nullptr;
  double lw_[2] = {1.0, 1.0};
  bool need_train_ = true;
  std::vector<label_t> bin_label_;
};

// ------------------------------------------------------------------ multiclass
class MulticlassSoftmax : public ObjectiveFunction {
 public:
  explicit MulticlassSoftmax(const Config& c) : num_class_(c.num_class) {
    factor_ = static_cast<double>(num_class_) / (num_class_ - 1.0f);
  }
  explicit MulticlassSoftmax(const std::vector<std::string>& t) {
    num_class_ = static_cast<int>(ParseKey(t, "num_class", -1));
    if (num_class_ < 0) Log::Fatal("Objective should contain num_class field");
    factor_ = static_cast<double>(num_class_) / (num_class_ - 1.0f);
  }
  void Init(const Metadata& md, data_size_t n) override {
    num_data_ = n;
    label_ = md.label();
    weights_ = md.weights();
    label_int_.resize(n);
    probs_.assign(num_class_, 0.0);
    double sw = 0;
    for (data_size_t i = 0; i < n; ++i) {
      label_int_[i] = static_cast<int>(label_[i]);
      if (label_int_[i] < 0 || label_int_[i] >= num_class_) {
        Log::Fatal("Label must be in [0, %d), but found %d in label", num_class_, label_int_[i]);
      }
      if (weights_) {
        probs_[label_int_[i]] += weights_[i];
        sw += weights_[i];
      } else {
        probs_[label_int_[i]] += 1.0;
      }
    }
    if (!weights_) sw = n;
    if (Network::num_machines() > 1) {
      sw = Network::GlobalSyncUpBySum(sw);
      for (int k = 0; k < num_class_; ++k) probs_[k] = Network::GlobalSyncUpBySum(probs_[k]);
    }
    for (int k = 0; k < num_class_; ++k) probs_[k] /= sw;
  }
  void GetGradients(const double* s, score_t* g, score_t* h) const override {
#pragma omp parallel
    {
      std::vector<double> rec(num_class_);
#pragma omp for schedule(static)
      for (data_size_t i = 0; i < num_data_; ++i) {
        for (int k = 0; k < num_class_; ++k) rec[k] = s[static_cast<size_t>(num_data_) * k + i];
        common::Softmax(&rec);
        const double w = weights_ ? weights_[i] : 1.0;
        for (int k = 0; k < num_class_; ++k) {
          const double p = rec[k];
          const size_t idx = static_cast<size_t>(num_data_) * k + i;
          g[idx] = static_cast<score_t>((label_int_[i] == k ? p - 1.0f : p) * w);
          h[idx] = static_cast<score_t>(factor_ * p * (1.0f - p) * w);
        }
      }
    }
  }
  void ConvertOutput(const double* in, double* out) const override { common::Softmax(in, out, num_class_); }
  int DeviceOutputKind(double*) const override { return 4; }
  const char* GetName() const override { return "multiclass"; }
  std::string ToString() const override {
    std::stringstream s;
    s << GetName() << " num_class:" << num_class_;
    return s.str();
  }
  bool SkipEmptyClass() const override { return true; }
  int NumModelPerIteration() const override { return num_class_; }
  int NumPredictOneRow() const override { return num_class_; }
  bool NeedAccuratePrediction() const override { return false; }
  double BoostFromScore(int k) const override { return std::log(std::max<double>(kEpsilon, probs_[k])); }
  bool ClassNeedTrain(int k) const override {
    return !(std::fabs(probs_[k]) <= kEpsilon || std::fabs(probs_[k]) >= 1.0 - kEpsilon);
  }
  DeviceGradSpec DeviceSpec() const override {
    DeviceGradSpec d;
    d.kind = DeviceGradKind::MulticlassSoftmax;
    d.num_class = num_class_;
    d.p0 = factor_;
    d.label = label_;
    d.weights = weights_;
    return d;
  }

 private:
  int num_class_;
  double factor_;
  data_size_t num_data_ = 0;
  const label_t* weights_ = nullptr;
  std::vector<int> label_int_;
  std::vector<double> probs_;
};

class MulticlassOVA : public ObjectiveFunction {
 public:
  explicit MulticlassOVA(const Config& c) : num_class_(c.num_class), sigmoid_(c.sigmoid) {
    for (int k = 0; k < num_class_; ++k) bin_.emplace_back(new BinaryLogloss(c, k));
  }
  explicit MulticlassOVA(const std::vector<std::string>& t) {
    num_class_ = static_cast<int>(ParseKey(t, "num_class", -1));
    sigmoid_ = ParseKey(t, "sigmoid", -1);
    if (num_class_ < 0) Log::Fatal("Objective should contain num_class field");
    if (sigmoid_ <= 0.0) Log::Fatal("Sigmoid parameter %f should be greater than zero", sigmoid_);
  }
  void Init(const Metadata& md, data_size_t n) override {
    num_data_ = n;
    label_ = md.label();
    for (auto& b : bin_) b->Init(md, n);
  }
  void GetGradients(const double* s, score_t* g, score_t* h) const override {
    for (int k = 0; k < num_class_; ++k) {
      const size_t off = static_cast<size_t>(num_data_) * k;
      bin_[k]->GetGradients(s + off, g + off, h + off);
    }
  }
  const char* GetName() const override { return "multiclassova"; }
  void ConvertOutput(const double* in, double* out) const override {
    for (int k = 0; k < num_class_; ++k) out[k] = 1.0f / (1.0f + std::exp(-sigmoid_ * in[k]));
  }
  int DeviceOutputKind(double* param) const override {
    *param = sigmoid_;
    return 5;
  }
  std::string ToString() const override {
    std::stringstream s;
    s << GetName() << " num_class:" << num_class_ << " sigmoid:" << sigmoid_;
    return s.str();
  }
  bool SkipEmptyClass() const override { return true; }
  int NumModelPerIteration() const override { return num_class_; }
  int NumPredictOneRow() const override { return num_class_; }
  bool NeedAccuratePrediction() const override { return false; }
  double BoostFromScore(int k) const override { return bin_[k]->BoostFromScore(0); }
  bool ClassNeedTrain(int k) const override { return bin_[k]->ClassNeedTrain(0); }
  // per-class binary specs are exposed through SubSpec
  DeviceGradSpec DeviceSpec() const override {
    DeviceGradSpec d;
    d.kind = DeviceGradKind::MulticlassOVA;
    d.num_class = num_class_;
    return d;
  }
  const BinaryLogloss* sub(int k) const { return bin_[k].get(); }

 private:
  int num_class_;
  double sigmoid_;
  data_size_t num_data_ = 0;
  std::vector<std::unique_ptr<BinaryLogloss>> bin_;
};

// ------------------------------------------------------------------ cross entropy
class CrossEntropy : public ObjectiveFunction {
 public:
  explicit CrossEntropy(const Config&) {}
  explicit CrossEntropy(const std::vector<std::string>&) {}
  void Init(const Metadata& md, data_size_t n) override {
    num_data_ = n;
    label_ = md.label();
    weights_ = md.weights();
    for (data_size_t i = 0; i < n; ++i) {
      if (label_[i] < 0.0f || label_[i] > 1.0f) Log::Fatal("[%s]: label should be in interval [0, 1]", GetName());
    }
    if (weights_) {
      double sw = 0;
      label_t mn = weights_[0];
      for (data_size_t i = 0; i < n; ++i) {
        sw += weights_[i];
        mn = std::min(mn, weights_[i]);
      }
      if (mn < 0.0f) Log::Fatal("[%s]: at least one weight is negative", GetName());
      if (sw == 0.0) Log::Fatal("[%s]: sum of weights is zero", GetName());
    }
  }
  void GetGradients(const double* s, score_t* g, score_t* h) const override {
#pragma omp parallel for schedule(static)
    for (data_size_t i = 0; i < num_data_; ++i) {
      const double z = 1.0f / (1.0f + std::exp(-s[i]));
      const double w = weights_ ? weights_[i] : 1.0;
      g[i] = static_cast<score_t>((z - label_[i]) * w);
      h[i] = static_cast<score_t>(z * (1.0f - z) * w);
    }
  }
  const char* GetName() const override { return "cross_entropy"; }
  void ConvertOutput(const double* in, double* out) const override { out[0] = 1.0f / (1.0f + std::exp(-in[0])); }
  int DeviceOutputKind(double* param) const override {
    *param = 1.0;
    return 1;
  }
  std::string ToString() const override { return GetName(); }
  double BoostFromScore(int) const override {
    double sl = 0, sw = 0;
    for (data_size_t i = 0; i < num_data_; ++i) {
      const double w = weights_ ? weights_[i] : 1.0;
      sl += label_[i] * w;
      sw += w;
    }
    double p = sl / sw;
    p = std::min(p, 1.0 - kEpsilon);
    p = std::max<double>(p, kEpsilon);
    return std::log(p / (1.0f - p));
  }
  DeviceGradSpec DeviceSpec() const override {
    DeviceGradSpec d;
    d.kind = DeviceGradKind::CrossEntropy;
    d.label = label_;
    d.weights = weights_;
    return d;
  }

 private:
  data_size_t num_data_ = 0;
  const label_t* weights_ = nullptr;
};

class CrossEntropyLambda : public ObjectiveFunction {
 public:
  explicit CrossEntropyLambda(const Config&) {}
  explicit CrossEntropyLambda(const std::vector<std::string>&) {}
  void Init(const Metadata& md, data_size_t n) override {
    num_data_ = n;
    label_ = md.label();
    weights_ = md.weights();
    for (data_size_t i = 0; i < n; ++i) {
      if (label_[i] < 0.0f || label_[i] > 1.0f) Log::Fatal("[%s]: label should be in interval [0, 1]", GetName());
    }
    if (weights_) {
      label_t mn = weights_[0];
      for (data_size_t i = 0; i < n; ++i) mn = std::min(mn, weights_[i]);
      if (mn <= 0.0f) Log::Fatal("[%s]: at least one weight is non-positive", GetName());
    }
  }
  void GetGradients(const double* s, score_t* g, score_t* h) const override {
#pragma omp parallel for schedule(static)
    for (data_size_t i = 0; i < num_data_; ++i) {
      if (!weights_) {
        const double z = 1.0f / (1.0f + std::exp(-s[i]));
        g[i] = static_cast<score_t>(z - label_[i]);
        h[i] = static_cast<score_t>(z * (1.0f - z));
      } else {
        const double w = weights_[i], y = label_[i];
        const double epf = std::exp(s[i]);
        const double hhat = std::log(1.0f + epf);
        const double z = 1.0f - std::exp(-w * hhat);
        const double enf = 1.0f / epf;
        g[i] = static_cast<score_t>((1.0f - y / z) * w / (1.0f + enf));
        const double c = 1.0f / (1.0f - z);
        double d = 1.0f + epf;
        const double a = w * epf / (d * d);
        d = c - 1.0f;
        const double b = (c / (d * d)) * (1.0f + w * epf - c);
        h[i] = static_cast<score_t>(a * (1.0f + y * b));
      }
    }
  }
  const char* GetName() const override { return "cross_entropy_lambda"; }
  void ConvertOutput(const double* in, double* out) const override { out[0] = std::log(1.0f + std::exp(in[0])); }
  std::string ToString() const override { return GetName(); }
  double BoostFromScore(int) const override {
    double sl = 0, sw = 0;
    for (data_size_t i = 0; i < num_data_; ++i) {
      const double w = weights_ ? weights_[i] : 1.0;
      sl += label_[i] * w;
      sw += w;
    }
    const double havg = sl / sw;
    return std::log(std::exp(havg) - 1.0f);
  }
  DeviceGradSpec DeviceSpec() const override {
    DeviceGradSpec d;
    d.kind = DeviceGradKind::CrossEntropyLambda;
    d.label = label_;
    d.weights = weights_;
    return d;
  }

 private:
  data_size_t num_data_ = 0;
  const label_t* weights_ = nullptr;
};

// ------------------------------------------------------------------ ranking
class RankingObjective : public ObjectiveFunction {
 public:
  explicit RankingObjective(const Config& c) : seed_(c.objective_seed) {}
  explicit RankingObjective(const std::vector<std::string>&) : seed_(0) {}
  void Init(const Metadata& md, data_size_t n) override {
    num_data_ = n;
    label_ = md.label();
    weights_ = md.weights();
    qb_ = md.query_boundaries();
    if (qb_ == nullptr) Log::Fatal("Ranking tasks require query information");
    nq_ = md.num_queries();
  }
  void GetGradients(const double* s, score_t* g, score_t* h) const override {
#pragma omp parallel for schedule(guided)
    for (data_size_t q = 0; q < nq_; ++q) {
      const data_size_t b = qb_[q], cnt = qb_[q + 1] - qb_[q];
      OneQuery(q, cnt, label_ + b, s + b, g + b, h + b);
      if (weights_) {
        for (data_size_t j = 0; j < cnt; ++j) {
          g[b + j] = static_cast<score_t>(g[b + j] * weights_[b + j]);
          h[b + j] = static_cast<score_t>(h[b + j] * weights_[b + j]);
        }
      }
    }
  }
  virtual void OneQuery(data_size_t q, data_size_t cnt, const label_t* label, const double* score, score_t* lambdas,
                        score_t* hess) const = 0;
  std::string ToString() const override { return GetName(); }
  bool NeedAccuratePrediction() const override { return false; }

 protected:
  DeviceGradSpec RankSpec(DeviceGradKind k) const {
    DeviceGradSpec d;
    d.kind = k;
    d.label = label_;
    d.weights = weights_;
    d.rank.num_queries = nq_;
    d.rank.query_boundaries = qb_;
    for (data_size_t q = 0; q < nq_; ++q) d.rank.max_query_docs = std::max(d.rank.max_query_docs, qb_[q + 1] - qb_[q]);
    return d;
  }
  int seed_;
  data_size_t nq_ = 0, num_data_ = 0;
  const label_t* weights_ = nullptr;
  const data_size_t* qb_ = nullptr;
};

class LambdarankNDCG : public RankingObjective {
 public:
  explicit LambdarankNDCG(const Config& c)
      : RankingObjective(c), sigmoid_(c.sigmoid), norm_(c.lambdarank_norm), trunc_(c.lambdarank_truncation_level) {
    gain_ = c.label_gain;
    DCG::DefaultLabelGain(&gain_);
    DCG::Init(gain_);
    if (sigmoid_ <= 0.0) Log::Fatal("Sigmoid param %f should be greater than zero", sigmoid_);
  }
  explicit LambdarankNDCG(const std::vector<std::string>& t) : RankingObjective(t) {}
  void Init(const Metadata& md, data_size_t n) override {
    RankingObjective::Init(md, n);
    DCG::CheckLabel(label_, n);
    inv_max_dcg_.resize(nq_);
#pragma omp parallel for schedule(static)
    for (data_size_t q = 0; q < nq_; ++q) {
      inv_max_dcg_[q] = DCG::MaxDCGAtK(trunc_, label_ + qb_[q], qb_[q + 1] - qb_[q]);
      if (inv_max_dcg_[q] > 0.0) inv_max_dcg_[q] = 1.0f / inv_max_dcg_[q];
    }
    min_in_ = -50.0 / sigmoid_ / 2;
    max_in_ = -min_in_;
    table_.resize(kBins);
    idx_factor_ = kBins / (max_in_ - min_in_);
    for (size_t i = 0; i < kBins; ++i) {
      const double x = i / idx_factor_ + min_in_;
      table_[i] = 1.0f / (1.0f + std::exp(x * sigmoid_));
    }
  }
  double Sig(double x) const {
    if (x <= min_in_) return table_[0];
    if (x >= max_in_) return table_[kBins - 1];
    return table_[static_cast<size_t>((x - min_in_) * idx_factor_)];
  }
  void OneQuery(data_size_t q, data_size_t cnt, const label_t* label, const double* score, score_t* lambdas,
                score_t* hess) const override {
    const double inv_max = inv_max_dcg_[q];
    for (data_size_t i = 0; i < cnt; ++i) lambdas[i] = hess[i] = 0.0f;
    std::vector<data_size_t> idx(cnt);
    std::iota(idx.begin(), idx.end(), 0);
    std::stable_sort(idx.begin(), idx.end(), [score](data_size_t a, data_size_t b) { return score[a] > score[b]; });
    const double best = score[idx[0]];
    data_size_t worst_i = cnt - 1;
    if (worst_i > 0 && score[idx[worst_i]] == kMinScore) worst_i -= 1;
    const double worst = score[idx[worst_i]];
    double sum_lambdas = 0;
    for (data_size_t i = 0; i < cnt; ++i) {
      const data_size_t hi = idx[i];
      const int hl = static_cast<int>(label[hi]);
      const double hs = score[hi];
      if (hs == kMinScore) continue;
      const double hg = gain_[hl];
      const double hd = DCG::Discount(i);
      double hsl = 0, hsh = 0;
      for (data_size_t j = 0; j < cnt; ++j) {
        if (i == j) continue;
        const data_size_t lo = idx[j];
        const int ll = static_cast<int>(label[lo]);
        const double ls = score[lo];
        if (hl <= ll || ls == kMinScore) continue;
        const double ds = hs - ls;
        const double dcg_gap = hg - gain_[ll];
        const double pd = std::fabs(hd - DCG::Discount(j));
        double dndcg = dcg_gap * pd * inv_max;
        if (norm_ && best != worst) dndcg /= (0.01f + std::fabs(ds));
        double pl = Sig(ds);
        double ph = pl * (1.0f - pl);
        pl *= -sigmoid_ * dndcg;
        ph *= sigmoid_ * sigmoid_ * dndcg;
        hsl += pl;
        hsh += ph;
        lambdas[lo] -= static_cast<score_t>(pl);
        hess[lo] += static_cast<score_t>(ph);
        sum_lambdas -= 2 * pl;
      }
      lambdas[hi] += static_cast<score_t>(hsl);
      hess[hi] += static_cast<score_t>(hsh);
    }
    if (norm_ && sum_lambdas > 0) {
      const double nf = std::log2(1 + sum_lambdas) / sum_lambdas;
      for (data_size_t i = 0; i < cnt; ++i) {
        lambdas[i] = static_cast<score_t>(lambdas[i] * nf);
        hess[i] = static_cast<score_t>(hess[i] * nf);
      }
    }
  }
  const char* GetName() const override { return "lambdarank"; }
  DeviceGradSpec DeviceSpec() const override {
    auto d = RankSpec(DeviceGradKind::Lambdarank);
    d.rank.inv_max_dcg = inv_max_dcg_.data();
    d.rank.label_gain = gain_.data();
    d.rank.num_label_gain = static_cast<int>(gain_.size());
    d.rank.norm = norm_;
    d.rank.sigmoid = sigmoid_;
    d.rank.sig_min = min_in_;
    d.rank.sig_max = max_in_;
    d.rank.sig_factor = idx_factor_;
    d.rank.sig_table = table_.data();
    d.rank.sig_bins = static_cast<int64_t>(table_.size());
    return d;
  }

 private:
  static constexpr size_t kBins = 1024 * 1024;
  double sigmoid_ = 1;
  bool norm_ = true;
  int trunc_ = 20;
  std::vector<double> gain_, inv_max_dcg_, table_;
  double min_in_ = -50, max_in_ = 50, idx_factor_ = 1;
};

class RankXENDCG : public RankingObjective {
 public:
  explicit RankXENDCG(const Config& c) : RankingObjective(c) {}
  explicit RankXENDCG(const std::vector<std::string>& t) : RankingObjective(t) {}
  void Init(const Metadata& md, data_size_t n) override {
    RankingObjective::Init(md, n);
    rands_.clear();
    for (data_size_t q = 0; q < nq_; ++q) rands_.emplace_back(seed_ + q);
  }
  void OneQuery(data_size_t q, data_size_t cnt, const label_t* label, const double* score, score_t* lambdas,
                score_t* hess) const override {
    if (cnt <= 1) {
      for (data_size_t i = 0; i < cnt; ++i) lambdas[i] = hess[i] = 0.0f;
      return;
    }
    std::vector<double> rho(cnt), params(cnt);
    common::Softmax(score, rho.data(), cnt);
    double inv_den = 0;
    for (data_size_t i = 0; i < cnt; ++i) {
      params[i] = common::PowRec(2.0, static_cast<int>(label[i])) - rands_[q].NextFloat();
      inv_den += params[i];
    }
    inv_den = 1. / std::max<double>(kEpsilon, inv_den);
    double s1 = 0;
    for (data_size_t i = 0; i < cnt; ++i) {
      double term = -params[i] * inv_den + rho[i];
      lambdas[i] = static_cast<score_t>(term);
      params[i] = term / (1. - rho[i]);
      s1 += params[i];
    }
    double s2 = 0;
    for (data_size_t i = 0; i < cnt; ++i) {
      double term = rho[i] * (s1 - params[i]);
      lambdas[i] += static_cast<score_t>(term);
      params[i] = term / (1. - rho[i]);
      s2 += params[i];
    }
    for (data_size_t i = 0; i < cnt; ++i) {
      lambdas[i] += static_cast<score_t>(rho[i] * (s2 - params[i]));
      hess[i] = static_cast<score_t>(rho[i] * (1.0 - rho[i]));
    }
  }
  const char* GetName() const override { return "rank_xendcg"; }
  DeviceGradSpec DeviceSpec() const override {
    auto d = RankSpec(DeviceGradKind::RankXendcg);
    states_.resize(rands_.size());
    for (size_t q = 0; q < rands_.size(); ++q) states_[q] = rands_[q].state();
    d.rank.rng_states = states_.data();
    return d;
  }

 private:
  mutable std::vector<Random> rands_;
  mutable std::vector<unsigned> states_;
};

}  // namespace

ObjectiveFunction* ObjectiveFunction::CreateObjectiveFunction(const std::string& type, const Config& c) {
  if (type == "regression") return new RegressionL2(c);
  if (type == "regression_l1") return new RegressionL1(c);
  if (type == "quantile") return new Quantile(c);
  if (type == "huber") return new Huber(c);
  if (type == "fair") return new Fair(c);
  if (type == "poisson") return new Poisson(c);
  if (type == "binary") return new BinaryLogloss(c);
  if (type == "lambdarank") return new LambdarankNDCG(c);
  if (type == "rank_xendcg") return new RankXENDCG(c);
  if (type == "multiclass") return new MulticlassSoftmax(c);
  if (type == "multiclassova") return new MulticlassOVA(c);
  if (type == "cross_entropy") return new CrossEntropy(c);
  if (type == "cross_entropy_lambda") return new CrossEntropyLambda(c);
  if (type == "mape") return new Mape(c);
  if (type == "gamma") return new Gamma(c);
  if (type == "tweedie") return new Tweedie(c);
  if (type == "custom") return nullptr;
  Log::Fatal("Unknown objective type name: %s", type.c_str());
}

ObjectiveFunction* ObjectiveFunction::CreateObjectiveFunction(const std::string& str) {
  auto t = Tokens(str);
  if (t.empty()) return nullptr;
  const std::string type = ParseObjectiveAlias(t[0]);
  if (type == "regression") return new RegressionL2(t);
  if (type == "regression_l1") return new RegressionL1(t);
  if (type == "quantile") return new Quantile(t);
  if (type == "huber") return new Huber(t);
  if (type == "fair") return new Fair(t);
  if (type == "poisson") return new Poisson(t);
  if (type == "binary") return new BinaryLogloss(t);
  if (type == "lambdarank") return new LambdarankNDCG(t);
  if (type == "rank_xendcg") return new RankXENDCG(t);
  if (type == "multiclass") return new MulticlassSoftmax(t);
  if (type == "multiclassova") return new MulticlassOVA(t);
  if (type == "cross_entropy") return new CrossEntropy(t);
  if (type == "cross_entropy_lambda") return new CrossEntropyLambda(t);
  if (type == "mape") return new Mape(t);
  if (type == "gamma") return new Gamma(t);
  if (type == "tweedie") return new Tweedie(t);
  if (type == "custom") return nullptr;
  Log::Fatal("Unknown objective type name: %s", type.c_str());
}

}  // namespace lgbm_amd
