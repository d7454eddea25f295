// Tree learner interface and factory: {cpu, gpu(MI355X)} x {serial, feature, data, voting}
// (reference include/LightGBM/tree_learner.h:26-102, src/treelearner/tree_learner.cpp).
#pragma once

#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "lgbm_amd/config.h"
#include "lgbm_amd/dataset.h"
#include "lgbm_amd/objective.h"
#include "lgbm_amd/tree.h"

namespace lgbm_amd {

class TreeLearner {
 public:
  virtual ~TreeLearner() = default;
  virtual void Init(const Dataset* train_data, bool is_constant_hessian) = 0;
  virtual void ResetTrainingData(const Dataset* train_data, bool is_constant_hessian) = 0;
  virtual void ResetConfig(const Config* config) = 0;
  virtual void SetForcedSplit(const std::string& json_text) = 0;
  // gradients/hessians: host pointers for CPU learners, device pointers for device learners
  virtual Tree* Train(const score_t* gradients, const score_t* hessians) = 0;
  virtual Tree* FitByExistingTree(const Tree* old_tree, const score_t* gradients, const score_t* hessians) const = 0;
  virtual Tree* FitByExistingTree(const Tree* old_tree, const std::vector<int>& leaf_pred,
                                  const score_t* gradients, const score_t* hessians) = 0;
  virtual void SetBaggingData(const Dataset* subset, const data_size_t* used_indices, data_size_t num_data) = 0;
  // add the just-trained tree's leaf outputs to `out_score` (host, length num_data) by partition
  virtual void AddPredictionToScore(const Tree* tree, double* out_score) const = 0;
  virtual void RenewTreeOutput(Tree* tree, const ObjectiveFunction* obj,
                               const std::function<double(const label_t*, int)>& residual_getter,
                               data_size_t total_num_data, const data_size_t* bag_indices,
                               data_size_t bag_cnt) const = 0;
  virtual bool IsDevice() const { return false; }

  static TreeLearner* CreateTreeLearner(const std::string& learner_type, const std::string& device_type,
                                        const Config* config);
};

}  // namespace lgbm_amd
