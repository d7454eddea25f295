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

class Metric {
 public:
  virtual ~Metric() = default;
  virtual void Init(const Metadata& metadata, data_size_t num_data) = 0;
  virtual const std::vector<std::string>& GetName() const = 0;
  virtual double factor_to_bigger_better() const = 0;
  virtual std::vector<double> Eval(const double* score, const ObjectiveFunction* objective) const = 0;
  static Metric* CreateMetric(const std::string& type, const Config& config);
};

}  // namespace lgbm_amd
