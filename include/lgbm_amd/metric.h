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
  int kind = 0;
  int convert = 0;  // score -> prediction: 0 identity, 1 sigmoid, 2 sign(s) * s^2
  double sigmoid = 1.0;
  double sum_weights = 0.0;
  const label_t* label = nullptr;  // host pointers, uploaded once per validation set
  const label_t* weights = nullptr;
};

class Metric {
 public:
  // device evaluation of this metric for the objective's output transform (kind 0: none)
  virtual DeviceMetricSpec DeviceSpec(const ObjectiveFunction* objective) const {
    (void)objective;
    return DeviceMetricSpec();
  }
  virtual ~Metric() = default;
  virtual void Init(const Metadata& metadata, data_size_t num_data) = 0;
  virtual const std::vector<std::string>& GetName() const = 0;
  virtual double factor_to_bigger_better() const = 0;
  virtual std::vector<double> Eval(const double* score, const ObjectiveFunction* objective) const = 0;
  static Metric* CreateMetric(const std::string& type, const Config& config);
};

}  // namespace lgbm_amd
