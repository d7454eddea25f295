// CPU leaf-wise (best-first) tree learner -- the host reference implementation used
// for device_type=cpu, as the differential-testing oracle of the device learner, and as
// the base of the CPU parallel learners.  Growth loop, histogram subtraction, the
// smaller/larger leaf bookkeeping, forced splits, refit and output renewal follow
// reference src/treelearner/serial_tree_learner.cpp:152-776.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "cegb.h"
#include "col_sampler.h"
#include "lgbm_amd/json.h"
#include "lgbm_amd/split_info.h"
#include "lgbm_amd/tree_learner.h"
#include "monotone_constraints.h"
#include "split_finder.h"

namespace lgbm_amd {

double MonotoneSplitPenalty(int depth, double penalization);

class SerialTreeLearner : public TreeLearner {
 public:
  explicit SerialTreeLearner(const Config* config);
  void Init(const Dataset* train_data, bool is_constant_hessian) override;
  void ResetTrainingData(const Dataset* train_data, bool is_constant_hessian) override;
  void ResetConfig(const Config* config) override;
  void SetForcedSplit(const std::string& json_text) override;
  Tree* Train(const score_t* gradients, const score_t* hessians) override;
  Tree* FitByExistingTree(const Tree* old_tree, const score_t* gradients, const score_t* hessians) const override;
  Tree* FitByExistingTree(const Tree* old_tree, const std::vector<int>& leaf_pred, const score_t* gradients,
                          const score_t* hessians) override;
  void SetBaggingData(const Dataset* subset, const data_size_t* used_indices, data_size_t num_data) override;
  void AddPredictionToScore(const Tree* tree, double* out_score) const override;
  void RenewTreeOutput(Tree* tree, const ObjectiveFunction* obj,
                       const std::function<double(const label_t*, int)>& residual_getter,
                       data_size_t total_num_data, const data_size_t* bag_indices, data_size_t bag_cnt) const override;

 protected:
  struct LeafState {
    int leaf = -1;
    data_size_t num_data = 0;
    double sum_g = 0, sum_h = 0;
    double output = 0;  // leaf output (parent output for smoothing)
  };
  // data partition
  const data_size_t* LeafIndices(int leaf, data_size_t* cnt) const {
    *cnt = leaf_count_[leaf];
    return indices_.data() + leaf_begin_[leaf];
  }
  virtual data_size_t PartitionLeaf(int leaf, int inner_feature, const SplitInfo& s, int new_leaf);
  // the leaf's rows on the host (a device learner first mirrors its partition)
  virtual const data_size_t* HostLeafRows(int leaf, data_size_t* cnt) { return LeafIndices(leaf, cnt); }
  void SetupCegb();
  void PrepareCegbLeaves();  // lazy CEGB costs of the leaves about to be scanned

  virtual void BeforeTrain();
  virtual bool BeforeFindBestSplit(const Tree* tree, int left_leaf, int right_leaf);
  virtual void FindBestSplits(const Tree* tree);
  virtual void ConstructHistograms(const std::vector<int8_t>& feature_used, bool use_subtract);
  int ChooseHistogramThreading(const std::vector<int8_t>& groups, const data_size_t* idx, data_size_t cnt);
  // the histogram mode (0 undecided, 1 col-wise, 2 row-wise); row-wise holds the Dataset's
  // row-major copy while it lasts
  void SetHistMode(int m);
  virtual void FindBestSplitsFromHistograms(const std::vector<int8_t>& feature_used, bool use_subtract,
                                            const Tree* tree);
  virtual void Split(Tree* tree, int best_leaf, int* left_leaf, int* right_leaf);
  virtual data_size_t GetGlobalDataCountInLeaf(int leaf) const { return leaf >= 0 ? leaf_count_[leaf] : 0; }
  // (count, sum g, sum h) of the leaf's local rows; the device learner sums them on the device
  virtual LeafState LocalLeafSums(int leaf) const;
  int ForceSplits(Tree* tree, int* left_leaf, int* right_leaf, int* cur_depth);
  void ComputeBestSplitForFeature(int slot, int inner, const std::vector<int8_t>& node_used, const LeafState& ls,
                                  int depth, SplitInfo* best);
  // evaluate one feature histogram with explicit params; returns splittability
  // meta: the feature's metadata and extra_trees generator (default meta_[inner]; the voting
  // learner's global scans pass their own generator set)
  bool EvalFeature(hist_t* hist, int inner, const SplitParams& p, const LeafState& ls, int depth, SplitInfo* best,
                   const FeatureMeta* meta = nullptr);
  void SplitInner(Tree* tree, int best_leaf, int* left_leaf, int* right_leaf, bool update_cnt);
  // a leaf's histogram (the leaf must hold a pool slot: BeforeFindBestSplit assigns them)
  std::vector<hist_t>& LeafHist(int leaf) { return hist_pool_[leaf_slot_[leaf]]; }
  hist_t* FeatureHist(int leaf, int inner) { return LeafHist(leaf).data() + 2 * data_->FeatureHistOffset(inner); }
  void InitFeatureMeta();
  // intermediate monotone constraints: a leaf whose bounds another split tightened gets its
  // best split recomputed from its stored histogram (reference RecomputeBestSplitForLeaf)
  void RecomputeBestSplitForLeaf(const Tree* tree, int leaf);
  std::vector<int8_t> GroupsUsed(const std::vector<int8_t>& feature_used) const;

  const Config* config_;
  const Dataset* data_ = nullptr;
  data_size_t num_data_ = 0;
  int num_features_ = 0;
  SplitParams params_;
  std::vector<FeatureMeta> meta_;
  ColSampler col_sampler_;
  std::unique_ptr<CostEffectiveGB> cegb_;  // cost-effective gradient boosting (null: off)
  LeafConstraints constraints_;
  std::vector<SplitInfo> best_split_per_leaf_;

  // histogram pool (reference HistogramPool, feature_histogram.hpp:1061-1301): full
  // histograms in slots, leaves mapped to slots; the parent's slot moves to its larger child.
  // histogram_pool_size (MB) bounds the slots below num_leaves: the least recently used leaf
  // is evicted, and a child whose parent was evicted is histogrammed from its rows
  void ResetPool();
  void PoolTouch(int leaf);
  void PoolAssign(int leaf, int keep_leaf);  // a slot for `leaf`, never evicting keep_leaf
  void PoolMove(int from_leaf, int to_leaf);
  std::vector<std::vector<hist_t>> hist_pool_;
  std::vector<int> leaf_slot_;         // leaf -> slot (-1: not cached)
  std::vector<int> slot_leaf_;         // slot -> leaf (-1: free)
  std::vector<long long> slot_stamp_;  // last use (LRU)
  long long pool_clock_ = 0;
  std::vector<std::vector<char>> splittable_;  // per leaf, per inner feature
  // the step's smaller / larger leaf ids (their histograms: LeafHist)
  int smaller_slot_ = -1, larger_slot_ = -1;
  // CPU histogram threading (reference Dataset::TestMultiThreadingMethod): 0 undecided (auto),
  // 1 col-wise (threads over feature groups), 2 row-wise (threads over row blocks)
  int hist_mode_ = 0;
  // data_->RetainRowMajor() taken (SetHistMode; not given back at destruction: the Dataset may
  // be freed first, and it frees the copy itself)
  bool holds_row_major_ = false;
  Dataset::RowWiseScratch row_scratch_;  // this learner's row-wise per-thread histograms
  bool has_parent_hist_ = false;
  LeafState smaller_, larger_;

  // partition
  std::vector<data_size_t> indices_;
  std::vector<data_size_t> leaf_begin_, leaf_count_;
  std::vector<data_size_t> tmp_left_, tmp_right_;
  const data_size_t* bag_indices_ = nullptr;
  data_size_t bag_cnt_ = 0;
  bool use_bag_ = false;

  const score_t* gradients_ = nullptr;
  const score_t* hessians_ = nullptr;
  Json forced_split_;
  std::string forced_split_text_;  // (the JSON text forced_split_ was parsed from)
  bool has_forced_split_ = false;
  // features owned by this rank (feature-parallel); empty = all
  std::vector<int8_t> feature_mask_;
};

}  // namespace lgbm_amd
