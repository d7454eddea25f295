// Boosting drivers: GBDT and its DART / GOSS / RF variants.
// Interface and semantics follow reference include/LightGBM/boosting.h:27-315 and
// src/boosting/{gbdt,dart,goss,rf}.*: BoostFromAverage, per-class trees, bagging with
// one LCG per 1024-row block (seed bagging_seed + block), shrinkage, leaf renewal,
// early stopping on validation metrics, snapshots, text/JSON/if-else model IO.
// With device_type=gpu the training scores and gradients live in HBM, owned by the
// device learner (DeviceTreeLearner); the host keeps only trees and metric mirrors.
#pragma once

#include <fstream>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "lgbm_amd/config.h"
#include "lgbm_amd/dataset.h"
#include "lgbm_amd/device_learner.h"
#include "lgbm_amd/metric.h"
#include "lgbm_amd/objective.h"
#include "lgbm_amd/random.h"
#include "lgbm_amd/tree.h"
#include "lgbm_amd/tree_learner.h"

namespace lgbm_amd {

struct PredictionEarlyStopConfig {
  int round_period = 10;
  double margin_threshold = 10.0;
};

struct PredictionEarlyStopInstance {
  std::function<bool(const double*, int)> callback;
  int round_period = std::numeric_limits<int>::max();
};

PredictionEarlyStopInstance CreatePredictionEarlyStopInstance(const std::string& type,
                                                              const PredictionEarlyStopConfig& cfg);

// host score buffer for one dataset (class-major, num_tree_per_iteration x num_data)
class ScoreUpdater {
 public:
  ScoreUpdater(const Dataset* data, int num_tree_per_iteration);
  // a validation updater may hand its scores to the device learner (slot): updates then run
  // on the device and the host copy is refreshed when it is read
  void AttachDevice(DeviceTreeLearner* dl, int slot);
  int device_slot() const { return device_ != nullptr ? device_slot_ : -1; }
  double* score() {
    SyncFromDevice();
    return score_.data();
  }
  const double* score() const {
    const_cast<ScoreUpdater*>(this)->SyncFromDevice();
    return score_.data();
  }
  data_size_t num_data() const { return num_data_; }
  bool has_init_score() const { return has_init_score_; }
  void AddScore(double v, int tree_id);
  void MultiplyScore(double v, int tree_id);
  void AddScore(const Tree* tree, int tree_id);  // traversal of binned rows
  void AddScore(const Tree* tree, const data_size_t* idx, data_size_t n, int tree_id);
  void AddScore(const TreeLearner* learner, const Tree* tree, int tree_id);
  const Dataset* data() const { return data_; }

 private:
  void SyncFromDevice();
  const Dataset* data_;
  data_size_t num_data_;
  int num_tree_per_iteration_ = 1;
  std::vector<double> score_;
  bool has_init_score_ = false;
  DeviceTreeLearner* device_ = nullptr;
  int device_slot_ = -1;
  bool host_stale_ = false;
};

class GBDT {
 public:
  GBDT();
  virtual ~GBDT();

  // ---- training
  virtual void Init(const Config* config, const Dataset* train_data, const ObjectiveFunction* objective,
                    const std::vector<const Metric*>& training_metrics);
  virtual void ResetTrainingData(const Dataset* train_data, const ObjectiveFunction* objective,
                                 const std::vector<const Metric*>& training_metrics);
  virtual void ResetConfig(const Config* config);
  virtual void AddValidDataset(const Dataset* valid_data, const std::vector<const Metric*>& valid_metrics);
  void Train(int snapshot_freq, const std::string& model_output_path);
  virtual bool TrainOneIter(const score_t* gradients, const score_t* hessians);
  virtual void RollbackOneIter();
  void RefitTree(const std::vector<std::vector<int>>& tree_leaf_prediction);
  virtual bool EvalAndCheckEarlyStopping();
  int GetCurrentIteration() const { return static_cast<int>(models_.size()) / num_tree_per_iteration_; }
  void MergeFrom(const GBDT* other);
  void ShuffleModels(int start_iter, int end_iter);

  // ---- evaluation
  std::vector<double> GetEvalAt(int data_idx);
  virtual const double* GetTrainingScore(int64_t* out_len);
  void GetPredictAt(int data_idx, double* out, int64_t* out_len);
  int64_t GetNumPredictAt(int data_idx) const;
  int GetEvalCounts() const;
  std::vector<std::string> GetEvalNames() const;

  // ---- prediction
  void InitPredict(int start_iteration, int num_iteration, bool is_pred_contrib);
  // InitPredict(start_iteration, num_iteration, false) would change nothing
  bool PredictRangeIs(int start_iteration, int num_iteration) const;
  // normal / raw predictions of a dense float32 / float64 matrix on the MI355X (same results
  // as the host predictor); false if not applicable (no device, too many classes)
  bool PredictDenseOnDevice(const void* data, bool is_double, int64_t nrow, int ncol, bool row_major,
                            int start_iteration, int num_iteration, bool raw, double* out);
  int NumPredictOneRow(int start_iteration, int num_iteration, bool is_pred_leaf, bool is_pred_contrib) const;
  void PredictRaw(const double* features, double* output, const PredictionEarlyStopInstance* es) const;
  void Predict(const double* features, double* output, const PredictionEarlyStopInstance* es) const;
  void PredictLeafIndex(const double* features, double* output) const;
  void PredictContrib(const double* features, double* output) const;
  void PredictRawByMap(const std::unordered_map<int, double>& f, double* output,
                       const PredictionEarlyStopInstance* es) const;
  void PredictByMap(const std::unordered_map<int, double>& f, double* output,
                    const PredictionEarlyStopInstance* es) const;
  void PredictLeafIndexByMap(const std::unordered_map<int, double>& f, double* output) const;
  void PredictContribByMap(const std::unordered_map<int, double>& f,
                           std::vector<std::unordered_map<int, double>>* output) const;

  // ---- model IO
  std::string SaveModelToString(int start_iteration, int num_iteration, int importance_type) const;
  bool SaveModelToFile(int start_iteration, int num_iteration, int importance_type, const char* filename) const;
  bool LoadModelFromString(const char* buffer, size_t len);
  std::string DumpModel(int start_iteration, int num_iteration, int importance_type) const;
  std::string ModelToIfElse(int num_iteration) const;
  bool SaveModelToIfElse(int num_iteration, const char* filename) const;
  std::vector<double> FeatureImportance(int num_iteration, int importance_type) const;
  double GetUpperBoundValue() const;
  double GetLowerBoundValue() const;
  double GetLeafValue(int tree_idx, int leaf_idx) const;
  void SetLeafValue(int tree_idx, int leaf_idx, double val);

  // ---- introspection
  int NumberOfTotalModel() const { return static_cast<int>(models_.size()); }
  int NumModelPerIteration() const { return num_tree_per_iteration_; }
  int NumberOfClasses() const { return num_class_; }
  int MaxFeatureIdx() const { return max_feature_idx_; }
  int LabelIdx() const { return label_idx_; }
  const std::vector<std::string>& FeatureNames() const { return feature_names_; }
  const std::vector<std::string>& FeatureInfos() const { return feature_infos_; }
  const Tree* model(int i) const { return models_[i].get(); }
  DeviceTreeLearner* device_learner() const { return device_learner_; }
  bool average_output() const { return average_output_; }
  const ObjectiveFunction* objective() const { return objective_; }
  std::string SubModelName() const { return "tree"; }
  const char* Name() const { return name_.c_str(); }
  const std::string& loaded_parameter() const { return loaded_parameter_; }
  bool NeedAccuratePrediction() const {
    return objective_ == nullptr || objective_->NeedAccuratePrediction();
  }

  static GBDT* CreateBoosting(const std::string& type, const char* model_filename);

 protected:
  // hook run before gradients are computed from the training score (DART drops trees here)
  virtual void PrepareScoreForGradients() {}
  virtual void Boosting();
  virtual void Bagging(int iter);
  virtual data_size_t BaggingHelper(data_size_t start, data_size_t cnt, data_size_t* buffer);
  void ResetBaggingConfig(const Config* config, bool is_change_dataset);
  double BoostFromAverage(int class_id, bool update_scorer);
  void UpdateScore(const Tree* tree, int cur_tree_id);
  std::string OutputMetric(int iter);
  virtual bool GetIsConstHessian(const ObjectiveFunction* obj) { return obj != nullptr && obj->IsConstantHessian(); }
  // training score helpers (host or device resident)
  void TrainScoreAdd(double v, int tree_id);
  void TrainScoreMultiply(double v, int tree_id);
  void TrainScoreAddTree(const Tree* tree, int tree_id);
  double* HostTrainScore();
  void MarkHostScoreStale() { host_score_fresh_ = false; }
  // run the bagging pass over all rows with `helper`, filling bag_data_indices_
  data_size_t RunBagging(const std::function<data_size_t(data_size_t, data_size_t, data_size_t*)>& helper);

  std::string name_ = "gbdt";
  int iter_ = 0;
  const Dataset* train_data_ = nullptr;
  std::unique_ptr<Config> config_;
  std::unique_ptr<TreeLearner> tree_learner_;
  // LGBM_AMD_ITER_LOG=<path>: one JSON line per boosting iteration (phase times, trees, device
  // collectives); distributed ranks write <path>.rank<r>
  std::unique_ptr<std::ofstream> iter_log_;
  double growth_stats_[7] = {0, 0, 0, 0, 0, 0, 0};
  bool iter_log_checked_ = false;
  void LogIteration(double grad_ms, double bag_ms, const std::vector<double>& tree_ms, double renew_ms,
                    double score_ms, double total_ms, const std::vector<int>& leaves, const std::vector<int>& device,
                    const std::vector<int>& rounds, const std::vector<int>& expansions, const std::vector<int>& graphs,
                    double coll_bytes);
  DeviceTreeLearner* device_learner_ = nullptr;
  // whether the device learner may launch the next iteration's tree before it is asked for:
  // plain boosting whose next tree depends on nothing but this tree's score update -- no
  // bagging, leaf renewal, custom gradients or dropped trees (DART / GOSS / RF: false)
  virtual bool SpeculationSafe(bool own_gradients) const;
  const ObjectiveFunction* objective_ = nullptr;
  std::unique_ptr<ObjectiveFunction> loaded_objective_;
  std::vector<const Metric*> training_metrics_;
  std::vector<std::vector<const Metric*>> valid_metrics_;
  std::unique_ptr<ScoreUpdater> train_score_updater_;
  bool host_score_fresh_ = true;
  std::vector<std::unique_ptr<ScoreUpdater>> valid_score_updater_;
  std::vector<std::vector<double>> best_score_;
  std::vector<std::vector<int>> best_iter_;
  std::vector<std::vector<std::string>> best_msg_;
  std::vector<std::unique_ptr<Tree>> models_;
  int early_stopping_round_ = 0;
  bool es_first_metric_only_ = false;
  int max_feature_idx_ = 0;
  int label_idx_ = 0;
  int num_class_ = 1;
  int num_tree_per_iteration_ = 1;
  data_size_t num_data_ = 0;
  double shrinkage_rate_ = 0.1;
  int num_iteration_for_pred_ = 0;
  int start_iteration_for_pred_ = 0;
  int num_init_iteration_ = 0;
  std::vector<std::string> feature_names_;
  std::vector<std::string> feature_infos_;
  std::vector<int8_t> monotone_constraints_;
  std::vector<score_t> gradients_, hessians_;

 public:
  // the host learner's gradients of the last iteration (tests: device vs host objectives)
  const std::vector<score_t>& host_gradients() const { return gradients_; }
  // LGBM_AMD_BoosterGrowthStats: [trees, device-resident, rounds, expansions, splits, collective bytes,
  // trees launched speculatively]
  const double* growth_stats() const { return growth_stats_; }
  const std::vector<score_t>& host_hessians() const { return hessians_; }
  data_size_t train_num_data() const { return num_data_; }

 protected:
  std::vector<data_size_t> bag_data_indices_;
  data_size_t bag_data_cnt_ = 0;
  std::vector<Random> bagging_rands_;
  static constexpr data_size_t kBaggingRandBlock = 1024;
  bool balanced_bagging_ = false;
  bool need_re_bagging_ = false;
  // device bagging / GOSS: the device generators restart (seed + block) when the host's would
  bool device_sampler_reset_ = true;
  int device_sampler_seed_ = 0;
  // a device draw of the bag (or -1: draw on the host)
  data_size_t DeviceBagging(bool goss);
  // metric j of validation set i: on the device when its scores live there, else on the host
  std::vector<double> EvalValid(int i, int j) const;
  std::vector<double> EvalTrain(const Metric* m);  // device-resident training scores when possible
  std::vector<bool> class_need_train_;
  bool is_constant_hessian_ = false;
  bool average_output_ = false;
  std::string loaded_parameter_;
  std::string forced_splits_text_;
};

class DART : public GBDT {
 public:
  DART() { name_ = "dart"; }
  bool SpeculationSafe(bool) const override { return false; }
  void Init(const Config* config, const Dataset* train_data, const ObjectiveFunction* objective,
            const std::vector<const Metric*>& training_metrics) override;
  void ResetConfig(const Config* config) override;
  bool TrainOneIter(const score_t* gradients, const score_t* hessians) override;
  const double* GetTrainingScore(int64_t* out_len) override;
  bool EvalAndCheckEarlyStopping() override;

 protected:
  void PrepareScoreForGradients() override;

 private:
  void DroppingTrees();
  void Normalize();
  std::vector<double> tree_weight_;
  double sum_weight_ = 0;
  std::vector<int> drop_index_;
  Random random_for_drop_;
  bool is_update_score_cur_iter_ = false;
};

class GOSS : public GBDT {
 public:
  GOSS() { name_ = "goss"; }
  bool SpeculationSafe(bool) const override { return false; }
  void Init(const Config* config, const Dataset* train_data, const ObjectiveFunction* objective,
            const std::vector<const Metric*>& training_metrics) override;
  void ResetTrainingData(const Dataset* train_data, const ObjectiveFunction* objective,
                         const std::vector<const Metric*>& training_metrics) override;
  void ResetConfig(const Config* config) override;
  bool TrainOneIter(const score_t* gradients, const score_t* hessians) override;

 protected:
  void Bagging(int iter) override;
  data_size_t BaggingHelper(data_size_t start, data_size_t cnt, data_size_t* buffer) override;
  bool GetIsConstHessian(const ObjectiveFunction*) override { return false; }

 private:
  void ResetGoss();
};

class RF : public GBDT {
 public:
  bool SpeculationSafe(bool) const override { return false; }
  RF() {
    name_ = "rf";
    average_output_ = true;
  }
  void Init(const Config* config, const Dataset* train_data, const ObjectiveFunction* objective,
            const std::vector<const Metric*>& training_metrics) override;
  void ResetConfig(const Config* config) override;
  void ResetTrainingData(const Dataset* train_data, const ObjectiveFunction* objective,
                         const std::vector<const Metric*>& training_metrics) override;
  bool TrainOneIter(const score_t* gradients, const score_t* hessians) override;
  void RollbackOneIter() override;
  void AddValidDataset(const Dataset* valid_data, const std::vector<const Metric*>& valid_metrics) override;

 protected:
  void Boosting() override;

 private:
  void MultiplyScore(int cur_tree_id, double val);
  std::vector<double> init_scores_;
};

}  // namespace lgbm_amd
