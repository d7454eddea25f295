// Device-resident learner interface (implemented by the MI355X HIP learner in
// src/treelearner/gpu_tree_learner.cpp).  Beyond tree growth, the device learner owns
// the training score / gradient buffers in HBM so that one boosting iteration runs
// without host<->device traffic except the finished tree (SURVEY.md §7.1 principle 1).
// It is a mix-in next to TreeLearner; GBDT discovers it with dynamic_cast.
#pragma once

#include <string>
#include <vector>

#include "lgbm_amd/metric.h"
#include "lgbm_amd/objective.h"
#include "lgbm_amd/tree_learner.h"

namespace lgbm_amd {

// one bagging / GOSS draw on the device (reference gbdt.cpp:162-243, goss.hpp:103-179):
// the generator of 1024-row block b starts at seed + b and persists across draws until
// `reset` (the reference re-creates bagging_rands_ in ResetBaggingConfig / GOSS::ResetGoss)
struct DeviceSampleSpec {
  bool goss = false;
  bool balanced = false;
  bool reset = false;
  int seed = 3;
  double fraction = 1.0, pos_fraction = 1.0, neg_fraction = 1.0;
  double top_rate = 0.2, other_rate = 0.1;
  int num_tree_per_iteration = 1;
  const label_t* label = nullptr;                    // balanced bagging
  std::vector<data_size_t>* host_indices = nullptr;  // if set: the bag (in-bag, then out-of-bag) is copied back
};

class DeviceTreeLearner {
 public:
  virtual ~DeviceTreeLearner() = default;
  // allocate num_tree_per_iteration * num_data score/gradient buffers
  virtual void InitScores(int num_tree_per_iteration, const double* init_score) = 0;
  virtual void SyncScoreToHost(double* host, int tree_id) = 0;  // D2H of one class slice
  virtual void SyncScoreFromHost(const double* host, int tree_id) = 0;
  virtual void AddConstToScore(double v, int tree_id) = 0;
  virtual void MultiplyScore(double v, int tree_id) = 0;
  // after Train(): add the new tree by leaf partition (+ out-of-bag rows by traversal)
  virtual void AddTrainedTreeToScore(const Tree* tree, int tree_id) = 0;
  // a promise for the next Train(): its tree goes into the training scores of class 0 through
  // AddTrainedTreeToScore, after Tree::Shrinkage(shrinkage) and nothing else (GBDT::TrainOneIter
  // without leaf renewal).  The learner may then add it on the device as soon as the splits are
  // known, while the host builds the Tree object (0: no promise)
  virtual void ExpectTrainingScoreUpdate(double shrinkage) { (void)shrinkage; }
  // GBDT's permission, per iteration, to launch the next tree on the device before this
  // Train() returns (plain boosting: no bagging, renewal, custom gradients or dropped trees);
  // the learner checks the next Train()'s inputs against the launch and regrows if they differ
  virtual void AllowSpeculation(bool allowed) { (void)allowed; }
  // any tree, by traversal of the binned training rows
  virtual void AddTreeToScore(const Tree* tree, int tree_id) = 0;
  // device gradients for a point-wise objective; false if the spec is unsupported
  virtual bool ComputeGradients(const DeviceGradSpec& spec, int num_tree_per_iteration) = 0;
  virtual void UploadGradients(const score_t* g, const score_t* h, int64_t n) = 0;
  // draw a bag on the device and make it the learner's bagging data (GOSS also rescales
  // the sampled rows' device gradients); returns the in-bag count
  virtual data_size_t DeviceSample(const DeviceSampleSpec& spec) = 0;
  virtual void DownloadGradients(score_t* g, score_t* h, int64_t n) = 0;
  virtual score_t* device_gradients() = 0;
  virtual score_t* device_hessians() = 0;
  virtual void Synchronize() = 0;
  // validation sets (binned like the training data): rows and scores resident on the device.
  // AddValidData uploads the current host scores ([tree_id][rows]) and returns a slot, or -1
  // if the set can not be scored on the device (its group layout differs)
  virtual int AddValidData(const Dataset* valid, int num_tree_per_iteration, const double* scores) = 0;
  virtual void ValidAddConst(int slot, double v, int tree_id) = 0;
  virtual void ValidMultiply(int slot, double v, int tree_id) = 0;
  virtual void ValidAddTree(int slot, const Tree* tree, int tree_id) = 0;
  virtual void ValidScoreToHost(int slot, double* host) = 0;
  // a metric on the device-resident scores of a validation set: the raw sums of
  // DeviceMetricSpec::nout values (Metric::FinishDevice turns them into the metric's values);
  // false: evaluate on the host
  virtual bool ValidEval(int slot, const DeviceMetricSpec& spec, std::vector<double>* sums) = 0;
  // the same on the device-resident training scores (training metrics every metric_freq
  // iterations without a download of the scores); false: evaluate on the host
  virtual bool TrainEval(const DeviceMetricSpec& spec, std::vector<double>* sums) { return false; }

  // the last tree: grown device-resident, splits applied, bytes moved by device collectives
  struct TreeStats {
    bool device_mode = false;
    int splits = 0;
    int rounds = 0;  // round growth: expansion rounds of the tree (0: one split per step)
    int expansions = 0;  // round growth: nodes expanded (accepted splits + speculation never accepted)
    bool graph = false;  // the tree's kernels (and collectives) were replayed from hipGraphs
    double collective_bytes = 0.0;
    bool speculated = false;  // grown by a launch made when the previous tree ended (AllowSpeculation)
  };
  virtual TreeStats LastTreeStats() const { return TreeStats(); }
  // percentile leaf renewal (L1 / quantile / MAPE) of the tree just grown, on the device from
  // the partition and the device-resident scores of class `tree_id`; false: not possible here
  // (the caller renews on the host)
  virtual bool RenewTreeOutputOnDevice(Tree* tree, const ObjectiveFunction* obj, int tree_id) {
    (void)tree; (void)obj; (void)tree_id;
    return false;
  }

  // test support (tests/test_gpu_kernels.py): the state the last device-grown tree left in HBM.
  // A leaf's rows (partition), its raw fixed-point histogram slot, which histogram bins are
  // meaningful (the slices of features evaluated for the leaf: a feature its parent could not
  // split on is never materialised again) and (sum_g, sum_h, count); false if the last tree
  // was not grown device-resident.
  // `tree` is that last tree: the children of its last split (and of splits whose children
  // can not split further) never get histograms, their bin_valid is all 0.
  virtual bool DebugLeafState(const Tree* tree, int leaf, std::vector<int32_t>* rows, std::vector<long long>* hist,
                              std::vector<int8_t>* bin_valid, double* sums) {
    (void)tree; (void)leaf; (void)rows; (void)hist; (void)bin_valid; (void)sums;
    return false;
  }
  // the per-row (g, h) the histograms were built from and the fixed-point scales (g, h)
  virtual bool DebugGradients(std::vector<float>* g, std::vector<float>* h, double* scales) {
    (void)g; (void)h; (void)scales;
    return false;
  }
  // differential check of every leaf's device best split against the CPU split finder run
  // on the same (dequantised) histogram; a JSON report
  virtual std::string DebugCheckSplits(const Tree* tree) {
    (void)tree;
    return "{}";
  }
};

TreeLearner* CreateDeviceTreeLearner(const std::string& learner_type, const Config* config);

}  // namespace lgbm_amd
