// Evaluation metrics (reference include/LightGBM/metric.h, src/metric/*.hpp).
// Metrics evaluate the rank-local shard (reference semantics: no Network calls in
// src/metric); `Eval` receives raw scores laid out class-major.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "lgbm_amd/config.h"
#include "lgbm_amd/dataset.h"
#include "lgbm_amd/objective.h"

namespace lgbm_amd {

// a metric the device learner can evaluate on device-resident validation scores
// (kind: src/device/kernels.h kMetric*; 0 = host only)
struct DeviceMetricSpec {
  int kind = 0;     // dev::kMetric* (0: evaluate on the host)
  int convert = 0;  // score -> prediction: 0 identity, 1 sigmoid, 2 sign(s) * s^2, 3 exp,
                    // 4 softmax over the classes, 5 sigmoid per class
  double sigmoid = 1.0;
  double param = 0.0;  // alpha (quantile / huber), fair_c, tweedie_variance_power
  int num_class = 1;   // multiclass metrics: class-major scores
  int top_k = 1;       // multi_error@k
  int nout = 1;        // sums the device returns (Metric::FinishDevice turns them into values)
  const label_t* label = nullptr;  // host pointers, uploaded once per validation set
  const label_t* weights = nullptr;
  // query metrics (NDCG / MAP): boundaries, weights, eval_at, per-query constants ([nq][nk]
  // inverse max DCG, or [nq] relevant documents) and the DCG tables; `key` identifies the
  // metric whose device copies they are
  const void* key = nullptr;
  const data_size_t* qb = nullptr;
  int nq = 0;
  const label_t* qw = nullptr;
  std::vector<int> eval_at;
  std::vector<double> qconst;
  std::vector<double> label_gain, discount;
  data_size_t max_query_docs = 0;  // the longest query (queries past kRankMaxDocs: global scratch)
};

class Metric {
 public:
  // device evaluation of this metric for the objective's output transform (kind 0: none)
  virtual DeviceMetricSpec DeviceSpec(const ObjectiveFunction* objective) const {
    (void)objective;
    return DeviceMetricSpec();
  }
  // the metric's values from the sums the device evaluation returned (DeviceSpec().nout)
  virtual std::vector<double> FinishDevice(const std::vector<double>& sums) const { return sums; }
  virtual ~Metric() = default;
  virtual void Init(const Metadata& metadata, data_size_t num_data) = 0;
  virtual const std::vector<std::string>& GetName() const = 0;
  virtual double factor_to_bigger_better() const = 0;
  virtual std::vector<double> Eval(const double* score, const ObjectiveFunction* objective) const = 0;
  static Metric* CreateMetric(const std::string& type, const Config& config);
};

}  // namespace lgbm_amd
