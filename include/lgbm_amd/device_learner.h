// Device-resident learner interface (implemented by the MI355X HIP learner in
// src/treelearner/gpu_tree_learner.cpp).  Beyond tree growth, the device learner owns
// the training score / gradient buffers in HBM so that one boosting iteration runs
// without host<->device traffic except the finished tree (SURVEY.md §7.1 principle 1).
// It is a mix-in next to TreeLearner; GBDT discovers it with dynamic_cast.
#pragma once

#include <vector>

#include "lgbm_amd/objective.h"
#include "lgbm_amd/tree_learner.h"

namespace lgbm_amd {

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
  // any tree, by traversal of the binned training rows
  virtual void AddTreeToScore(const Tree* tree, int tree_id) = 0;
  // device gradients for a point-wise objective; false if the spec is unsupported
  virtual bool ComputeGradients(const DeviceGradSpec& spec, int num_tree_per_iteration) = 0;
  virtual void UploadGradients(const score_t* g, const score_t* h, int64_t n) = 0;
  virtual void DownloadGradients(score_t* g, score_t* h, int64_t n) = 0;
  virtual score_t* device_gradients() = 0;
  virtual score_t* device_hessians() = 0;
  virtual void Synchronize() = 0;
};

TreeLearner* CreateDeviceTreeLearner(const std::string& learner_type, const Config* config);

}  // namespace lgbm_amd
