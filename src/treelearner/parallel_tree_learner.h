// CPU distributed tree learners over the host Network layer
// (reference src/treelearner/parallel_tree_learner.h:23-190):
//  * FeatureParallel: every rank holds all rows; features are dealt out by bin count and
//    only the best split per rank is exchanged (allgather of SplitInfo).
//  * DataParallel: rows are sharded; local histograms of the smaller leaf are
//    reduce-scattered so each rank owns the global histograms of a feature block, finds
//    the best split there, and the per-rank bests are allgathered.
//  * VotingParallel (PV-Tree): local top_k voting per leaf, global vote by
//    count-weighted gain, then only the elected features' histograms are reduced.
#pragma once

#include <vector>

#include "serial_tree_learner.h"

namespace lgbm_amd {

// fixed-size wire format of a SplitInfo (categorical thresholds padded to max_cat)
size_t SplitInfoWireSize(int max_cat_threshold);
void SplitInfoToWire(const SplitInfo& s, int max_cat_threshold, char* out);
void SplitInfoFromWire(const char* in, SplitInfo* s);
// allgather both leaves' local best splits and keep the global best of each
void SyncUpGlobalBestSplit(SplitInfo* smaller_best, SplitInfo* larger_best, int max_cat_threshold);

class FeatureParallelTreeLearner : public SerialTreeLearner {
 public:
  explicit FeatureParallelTreeLearner(const Config* config) : SerialTreeLearner(config) {}
  void Init(const Dataset* train_data, bool is_constant_hessian) override;

 protected:
  void BeforeTrain() override;
  void FindBestSplitsFromHistograms(const std::vector<int8_t>& used, bool use_subtract, const Tree* tree) override;

 private:
  int rank_ = 0, num_machines_ = 1;
};

class DataParallelTreeLearner : public SerialTreeLearner {
 public:
  explicit DataParallelTreeLearner(const Config* config) : SerialTreeLearner(config) {}
  void Init(const Dataset* train_data, bool is_constant_hessian) override;
  void ResetConfig(const Config* config) override;

 protected:
  void BeforeTrain() override;
  void FindBestSplits(const Tree* tree) override;
  void Split(Tree* tree, int best_leaf, int* left_leaf, int* right_leaf) override;
  data_size_t GetGlobalDataCountInLeaf(int leaf) const override {
    return leaf >= 0 ? global_count_[leaf] : 0;
  }

 private:
  int rank_ = 0, num_machines_ = 1;
  std::vector<data_size_t> global_count_;
  std::vector<int8_t> aggregated_;          // features whose global histogram this rank owns
  std::vector<comm_size_t> block_start_, block_len_;
  std::vector<size_t> write_pos_, read_pos_;  // byte offsets per inner feature
  comm_size_t reduce_scatter_size_ = 0;
  std::vector<char> in_buf_, out_buf_;
};

// Base = SerialTreeLearner (host histograms) or GPUTreeLearner in host-assisted growth
// (device histograms and partitions), as the reference instantiates
// VotingParallelTreeLearner<SerialTreeLearner | GPUTreeLearner>
// (voting_parallel_tree_learner.cpp:456-458).
template <typename Base>
class VotingParallelTreeLearner : public Base {
 public:
  explicit VotingParallelTreeLearner(const Config* config) : Base(config) {}
  void Init(const Dataset* train_data, bool is_constant_hessian) override;
  void ResetConfig(const Config* config) override;

 protected:
  using LeafState = typename SerialTreeLearner::LeafState;
  void BeforeTrain() override;
  bool BeforeFindBestSplit(const Tree* tree, int left_leaf, int right_leaf) override;
  void FindBestSplits(const Tree* tree) override;
  void Split(Tree* tree, int best_leaf, int* left_leaf, int* right_leaf) override;
  data_size_t GetGlobalDataCountInLeaf(int leaf) const override {
    return leaf >= 0 ? global_count_[leaf] : 0;
  }

 private:
  void InitLocalParams();
  void GlobalVoting(int leaf, const std::vector<LightSplitInfo>& splits, std::vector<int>* out) const;

  int rank_ = 0, num_machines_ = 1, top_k_ = 20;
  SplitParams local_params_;
  // the global scans' feature metadata: a second extra_trees generator set, seeded like meta_
  // (reference voting_parallel_tree_learner.cpp:61-90 feature_metas_), drawn only by the rank
  // that owns an elected histogram
  std::vector<FeatureMeta> global_meta_;
  LeafState global_smaller_, global_larger_;
  std::vector<data_size_t> global_count_;
  std::vector<hist_t> global_small_hist_, global_large_hist_;
  std::vector<char> in_buf_, out_buf_;
};

}  // namespace lgbm_amd
