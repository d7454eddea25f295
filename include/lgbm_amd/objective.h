// Objective functions (gradients/hessians, init score, output transform, leaf renewal).
// Interface mirrors reference include/LightGBM/objective_function.h:19-92; the model
// string of each objective (ToString / the "objective=" model line) is identical so
// that models round-trip with the reference.  Point-wise objectives also expose a
// device description (`DeviceGradSpec`) consumed by the HIP gradient kernel, so the
// device learner never copies scores to the host.
#pragma once

#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "lgbm_amd/config.h"
#include "lgbm_amd/dataset.h"
#include "lgbm_amd/meta.h"

namespace lgbm_amd {

// kinds understood by the device gradient kernel
enum class DeviceGradKind : int {
  None = 0, L2 = 1, L1 = 2, Huber = 3, Fair = 4, Poisson = 5, Quantile = 6, Mape = 7, Gamma = 8, Tweedie = 9,
  Binary = 10, CrossEntropy = 11, CrossEntropyLambda = 12, MulticlassSoftmax = 13, MulticlassOVA = 14,
  Lambdarank = 15, RankXendcg = 16  // listwise: one workgroup per query (src/device/rank_kernels.hip)
};

// query-level tables of the listwise objectives (host pointers, uploaded once)
struct DeviceRankSpec {
  data_size_t num_queries = 0;
  data_size_t max_query_docs = 0;
  const data_size_t* query_boundaries = nullptr;  // [num_queries + 1]
  const double* inv_max_dcg = nullptr;            // [num_queries] (lambdarank)
  const double* label_gain = nullptr;
  int num_label_gain = 0;
  bool norm = true;
  double sigmoid = 1.0, sig_min = -25.0, sig_max = 25.0, sig_factor = 1.0;
  const double* sig_table = nullptr;  // [sig_bins] the sigmoid table (lambdarank)
  int64_t sig_bins = 0;
  const unsigned* rng_states = nullptr;  // [num_queries] per-query LCG states (xendcg); the device owns them after upload
};

// percentile leaf renewal on the device: the residual percentile and its weights
struct DeviceRenewSpec {
  double alpha = 0.5;
  const label_t* label = nullptr;    // host pointers; uploaded by the learner
  const label_t* weights = nullptr;  // null: unweighted percentile
};

struct DeviceGradSpec {
  DeviceGradKind kind = DeviceGradKind::None;
  int num_class = 1;
  double p0 = 0, p1 = 0, p2 = 0;  // kind-specific parameters (sigmoid, alpha, c, rho, ...)
  double label_weight[2] = {1.0, 1.0};
  const label_t* label = nullptr;         // host pointers; uploaded by the learner
  const label_t* weights = nullptr;
  const label_t* label_weight_arr = nullptr;  // per-row factor (MAPE)
  DeviceRankSpec rank;                        // Lambdarank / RankXendcg only
};

class ObjectiveFunction {
 public:
  virtual ~ObjectiveFunction() = default;
  virtual void Init(const Metadata& metadata, data_size_t num_data) = 0;
  virtual void GetGradients(const double* score, score_t* gradients, score_t* hessians) const = 0;
  virtual const char* GetName() const = 0;
  virtual bool IsConstantHessian() const { return false; }
  virtual bool IsRenewTreeOutput() const { return false; }
  // RenewTreeOutput as a device percentile (L1 / quantile / MAPE); false: host only
  virtual bool DeviceRenew(DeviceRenewSpec* spec) const {
    (void)spec;
    return false;
  }
  // new leaf output from the residuals of the rows in the leaf (L1/quantile/MAPE)
  virtual double RenewTreeOutput(double ori_output, const std::function<double(const label_t*, int)>& residual,
                                 const data_size_t* index_mapper, const data_size_t* bagging_mapper,
                                 data_size_t num_data_in_leaf) const {
    (void)residual; (void)index_mapper; (void)bagging_mapper; (void)num_data_in_leaf;
    return ori_output;
  }
  virtual double BoostFromScore(int /*class_id*/) const { return 0.0; }
  virtual bool ClassNeedTrain(int /*class_id*/) const { return true; }
  virtual bool SkipEmptyClass() const { return false; }
  virtual int NumModelPerIteration() const { return 1; }
  virtual int NumPredictOneRow() const { return 1; }
  virtual bool NeedAccuratePrediction() const { return true; }
  virtual data_size_t NumPositiveData() const { return 0; }
  virtual void ConvertOutput(const double* input, double* output) const { output[0] = input[0]; }
  // ConvertOutput as a device-evaluable form: 0 identity, 1 sigmoid(*param * s),
  // 2 sign(s) * s^2 (regression with reg_sqrt), 3 exp(s), 4 softmax over the classes,
  // 5 sigmoid(*param * s) per class; -1 other (host only)
  virtual int DeviceOutputKind(double* param) const {
    (void)param;
    return -1;
  }
  virtual std::string ToString() const = 0;
  // device description; kind None => host gradients (uploaded by the learner)
  virtual DeviceGradSpec DeviceSpec() const { return DeviceGradSpec(); }
  const label_t* label() const { return label_; }

  static ObjectiveFunction* CreateObjectiveFunction(const std::string& type, const Config& config);
  static ObjectiveFunction* CreateObjectiveFunction(const std::string& str);  // from model string

 protected:
  const label_t* label_ = nullptr;
};

}  // namespace lgbm_amd
