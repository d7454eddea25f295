// MI355X tree learner: host orchestration of the HIP kernels in src/device/.
//
// Two growth modes share the same HBM state (row-major bin matrix, packed gradients,
// partition indices, histogram pool):
//  * device-resident (default): the whole tree -- split selection included -- runs as
//    a fixed kernel sequence on one stream (optionally replayed from a hipGraph); the
//    host reads the split records back once per tree.
//  * host-assisted: the SerialTreeLearner loop runs on the host and only histogram
//    construction, row partitioning and leaf sums are offloaded.  Used for features the
//    device split scan does not implement (forced splits, interaction constraints,
//    extra_trees, per-node column sampling, CEGB, categorical features with > 1024
//    categories) and under the voting-parallel learner.
// The reference's GPU learner (src/treelearner/gpu_tree_learner.cpp, OpenCL) offloads
// only the histogram build; this learner keeps the training scores, gradients and the
// data partition resident on the device across iterations.
#pragma once

#include <hip/hip_runtime_api.h>

#include <memory>
#include <string>
#include <set>
#include <unordered_map>
#include <vector>

#include "../device/kernels.h"
#include "lgbm_amd/device_learner.h"
#include "lgbm_amd/tuning.h"
#include "serial_tree_learner.h"

namespace lgbm_amd {

class GPUTreeLearner : public SerialTreeLearner, public DeviceTreeLearner {
 public:
  // serial: one device; data: rows sharded across ranks (owner-blocked reduce-scatter of the
  // histograms, reference data_parallel_tree_learner.cpp); feature: every rank holds all
  // rows and builds / scans only its own features (feature_parallel_tree_learner.cpp)
  // voting: rows sharded; each rank scans its local histograms, the ranks elect top_k features
  // per leaf and only their histograms are summed (reference voting_parallel_tree_learner.cpp)
  enum class Mode { kSerial, kData, kFeature, kVoting };
  GPUTreeLearner(const Config* config, Mode mode);
  explicit GPUTreeLearner(const Config* config) : GPUTreeLearner(config, Mode::kSerial) {}
  // host-assisted growth for every tree (the voting-parallel learner scans on the host)
  void ForceHostMode() { force_host_mode_ = true; }
  // device-resident voting (before Init); host-assisted trees keep the wrapper's host voting
  void UseDeviceVoting() { mode_ = Mode::kVoting; }
  ~GPUTreeLearner() override;

  // TreeLearner
  void Init(const Dataset* train_data, bool is_constant_hessian) override;
  void ResetTrainingData(const Dataset* train_data, bool is_constant_hessian) override;
  void ResetConfig(const Config* config) override;
  Tree* Train(const score_t* gradients, const score_t* hessians) override;
  void SetBaggingData(const Dataset* subset, const data_size_t* used_indices, data_size_t num_data) override;
  void AddPredictionToScore(const Tree* tree, double* out_score) const override;
  void RenewTreeOutput(Tree* tree, const ObjectiveFunction* obj,
                       const std::function<double(const label_t*, int)>& residual_getter, data_size_t total_num_data,
                       const data_size_t* bag_indices, data_size_t bag_cnt) const override;
  bool IsDevice() const override { return true; }

  // DeviceTreeLearner
  void InitScores(int num_tree_per_iteration, const double* init_score) override;
  void SyncScoreToHost(double* host, int tree_id) override;
  void SyncScoreFromHost(const double* host, int tree_id) override;
  void AddConstToScore(double v, int tree_id) override;
  void MultiplyScore(double v, int tree_id) override;
  void AddTrainedTreeToScore(const Tree* tree, int tree_id) override;
  void ExpectTrainingScoreUpdate(double shrinkage) override { expect_shrinkage_ = shrinkage; }
  void AllowSpeculation(bool allowed) override { spec_allowed_ = allowed; }
  void AddTreeToScore(const Tree* tree, int tree_id) override;
  bool ComputeGradients(const DeviceGradSpec& spec, int num_tree_per_iteration) override;
  void UploadGradients(const score_t* g, const score_t* h, int64_t n) override;
  data_size_t DeviceSample(const DeviceSampleSpec& spec) override;
  void DownloadGradients(score_t* g, score_t* h, int64_t n) override;
  score_t* device_gradients() override { return d_grad_; }
  score_t* device_hessians() override { return d_hess_; }
  void Synchronize() override;
  int AddValidData(const Dataset* valid, int num_tree_per_iteration, const double* scores) override;
  void ValidAddConst(int slot, double v, int tree_id) override;
  void ValidMultiply(int slot, double v, int tree_id) override;
  void ValidAddTree(int slot, const Tree* tree, int tree_id) override;
  void ValidScoreToHost(int slot, double* host) override;
  bool ValidEval(int slot, const DeviceMetricSpec& spec, std::vector<double>* sums) override;
  bool TrainEval(const DeviceMetricSpec& spec, std::vector<double>* sums) override;
  bool DebugLeafState(const Tree* tree, int leaf, std::vector<int32_t>* rows, std::vector<long long>* hist,
                      std::vector<int8_t>* bin_valid, double* sums) override;
  bool DebugGradients(std::vector<float>* g, std::vector<float>* h, double* scales) override;
  std::string DebugCheckSplits(const Tree* tree) override;  // gpu_self_check.cpp
  bool RenewTreeOutputOnDevice(Tree* tree, const ObjectiveFunction* obj, int tree_id) override;
  TreeStats LastTreeStats() const override { return last_stats_; }

  bool device_mode() const { return device_mode_; }

 protected:
  // host-assisted mode hooks
  void BeforeTrain() override;
  void ConstructHistograms(const std::vector<int8_t>& feature_used, bool use_subtract) override;
  data_size_t PartitionLeaf(int leaf, int inner_feature, const SplitInfo& s, int new_leaf) override;
  const data_size_t* HostLeafRows(int leaf, data_size_t* cnt) override {
    DownloadPartitionToHost();
    return LeafIndices(leaf, cnt);
  }
  void Split(Tree* tree, int best_leaf, int* left_leaf, int* right_leaf) override;
  data_size_t GetGlobalDataCountInLeaf(int leaf) const override;
  LeafState LocalLeafSums(int leaf) const override;

 private:
  void UploadData();
  void FreeAll();
  void FreeBuffers();
  void DecideMode();
  Tree* TrainDeviceMode(bool speculated = false);
  void EnqueueTree(const dev::KArgs& a);
  void DestroyGraph();
  void KernelFloorProbe(const dev::KArgs& a);
  void MaterializeSplitGradients();
  static bool FuseNextGradients();
  // the fused score walk (+ next gradients) applies to a tree of this many leaves
  bool FusedScoreWalk(int num_leaves, int tree_id) const;
  // the promised score update of the tree of the first nsplit device records (TreeFromRecords)
  void EarlyScoreUpdate(int nsplit, double shrinkage);
  static bool SameGradArgs(const dev::GradArgs& x, const dev::GradArgs& y);
  void ReportKernelTrace(int num_splits);
  void BuildRangeHistogram(int leaf, int slot);
  void DownloadPartitionToHost() const;
  void AllreduceRoot();
  void WatchdogSync();
  void AllreduceAbsMax();
  void UploadRankTables(const DeviceRankSpec& r, DeviceGradKind kind);
  void AllocSplittable();
  void UploadInteractionMasks();  // (re)allocate the splittable rows: all 1, leaf i -> row i (resets d_leaves_)
  // tree records for the traversal kernels (staged in d_tree_*; the host vectors must stay
  // alive until the stream is synchronised)
  dev::DevTree StageTree(const Tree* tree);
  bool UseSparseRows(int wpr) const;
  bool SetupForcedSplits();  // KArgs::forced_*; false: the forced splits need host-assisted growth
  // feature-parallel forced splits: each rank's records gathered after the scans (data-parallel
  // rejects forced splits as the reference does; voting keeps them host-assisted)
  bool ForcedGathered() const { return distributed_ && !data_parallel_ && !voting_ && world_ > 1; }
  void UploadSparseRows();
  std::vector<uint8_t> RowMajorBins(const Dataset* d, int row_words) const;
  template <typename T>
  T* Alloc(size_t n);

  // round growth (speculative multi-leaf expansion, src/device/round_kernels.hip): up to
  // round_k_ leaves expanded per round; trees whose split order depends on more than each
  // leaf's own rows (per-node sampling, extra_trees draws, CEGB, forced splits) and the
  // distributed learners grow one split per step
  bool RoundGrowth(const dev::KArgs& a) const;
  bool CegbRounds(const dev::KArgs& a) const;  // CEGB penalties on round growth (this tree)
  int RunRounds(dev::KArgs a);  // the tree's splits; h_rec_ holds their records
  struct RoundLaunch {  // a launched round tree (LaunchRounds), as its wait needs it
    dev::KArgs a{};
    int launched = 0;  // rounds enqueued
    int seg = 1;
    bool graph = false;
  };
  RoundLaunch LaunchRounds(dev::KArgs a);
  void LaunchSegment(const RoundLaunch& rl);
  int WaitRounds(RoundLaunch* rl);
  // Speculative next tree (one process, plain round growth, GBDT's permission): when a tree's
  // last plan is seen, its score walk (+ the next gradients) is already enqueued, and so is
  // the next tree -- its scales, root and provisioned rounds -- before the host returns
  // through GBDT.  The next Train() only waits for it if its inputs are the ones the launch
  // assumed (the walk's gradients, nothing reset); otherwise the launched tree is drained and
  // the tree grown again with the same feature sample.
  bool SpeculationEligible(const dev::KArgs& a, bool rounds) const;
  void LaunchSpeculative();
  void DropSpeculation();  // drain a launched next tree, restore the column sampler
  bool spec_allowed_ = false;
  bool spec_live_ = false;
  RoundLaunch spec_;
  std::unique_ptr<ColSampler> spec_sampler_;  // the sampler before the launched tree's draw
  uint64_t state_epoch_ = 0;     // bumped by every reset of the learner's inputs
  uint64_t spec_epoch_ = 0;
  bool grad_from_prefetch_ = false;  // the last ComputeGradients took the score walk's gradients
  void EnqueueRoot(const dev::KArgs& a);
  void EnqueueRound(const dev::KArgs& a);
  double RoundCollectiveBytes() const;  // device collectives of one distributed round
  long long* d_round_send_ = nullptr;
  long long* d_round_owned_ = nullptr;
  void AllocRoundState();
  void SizeRoundPools(int n_leaves);
  void ReadHist(const dev::Leaf& lf, int leaf, std::vector<long long>* raw) const;  // (self checks)
  int round_k_ = 1;
  int round_vmax_ = 0;      // speculation levels below the leaves (index buffers: + 2)
  int hist_slots_ = 0;      // histogram pool slots (round growth: one per expansion + the root's)
  int split_rows_ = 0;      // rows of the splittable flags (round growth: the tree's nodes)
  dev::Round* d_round_ = nullptr;
  dev::Round* h_round_ = nullptr;
  // KArgs::host_out (fine-grained pinned): the finished tree's scalars and split records, written
  // by its last plan; the host waits on its flag (one process)
  int32_t* h_tree_out_ = nullptr;
  bool tree_out_used_ = false;  // the last round tree's records are in h_tree_out_
  dev::RNode* d_rnode_ = nullptr;
  dev::FeatureBest* d_cbest_ = nullptr;
  uint32_t* d_cbest_cat_ = nullptr;
  uint32_t* d_child_cnt_ = nullptr;
  std::vector<hipGraphExec_t> round_root_execs_;  // [n]: root + n rounds (captured on first use)
  hipGraphExec_t round_seg_exec_ = nullptr;        // round_seg_ rounds
  int round_graph_rows_ = -1, round_graph_identity_ = -1, round_graph_root_mode_ = -1;
  // provisioning of the enqueued rounds (RunRounds): history length, margin, rounds per segment
  // graph, rounds in the root graph (0: the provisioned count rounded up to segments)
  size_t round_hist_n_ = tuning::kRoundHistory;
  int round_margin_ = 0, round_seg_ = tuning::kRoundSegment, round_root_fixed_ = 0;
  std::vector<int> round_hist_;  // rounds of the last round_hist_n_ trees (the next one enqueues their max + margin)
  bool last_tree_rounds_ = false;
  // per-tree round width (LGBM_AMD_ROUND_K unset): the last round tree's speculation outcome
  bool k_adapt_ = false;
  bool k_adapt_checked_ = false;  // (the 4M rows-per-rank threshold, applied at the first tree)
  int32_t k_cur_host_ = 0;
  int prev_expansions_ = 0, prev_splits_ = 0;
  // round growth vs one split per step, chosen by timing (AutoGrowthRounds)
  enum { kAutoUnset, kAutoProbe, kAutoRounds, kAutoSteps };
  int auto_state_ = kAutoUnset, auto_tree_ = 0;
  double auto_rounds_ms_ = 1e300;
  bool AutoGrowthRounds();
  void AutoGrowthRecord(double ms);
  void DestroyStepGraph();
  void DestroyRoundGraphs();

  void SetupOwnership();
  void GatherFeatureBests();
  void ReduceScatterStep(int parity);
  Mode mode_ = Mode::kSerial;
  bool data_parallel_ = false;  // kData on more than one rank (global counts from the split estimates)
  bool voting_ = false;         // kVoting on more than one rank
  void SetupCegb();
  // intermediate monotone constraints on the device (KArgs::mt_*, Params::mono_inter)
  void SetupMonoInter();
  size_t fb_slots_ = 0;
  int mt_cap_ = 0;
  int32_t* d_mt_leaf_parent_ = nullptr;
  int32_t* d_mt_node_ = nullptr;
  int8_t* d_mt_in_sub_ = nullptr;
  int32_t* d_mt_upd_ = nullptr;
  TreeStats last_stats_;
  double split_collective_bytes_ = 0.0;  // device collectives per split step (distributed)
  double root_collective_bytes_ = 0.0;
  int8_t* d_cegb_used_ = nullptr;
  double* d_cegb_coupled_ = nullptr;
  dev::FeatureBest* d_cegb_mem_ = nullptr;
  uint32_t* d_cegb_mem_cat_ = nullptr;
  // CEGB lazy penalties (KArgs::cegb_lazy): per-feature costs, paid bitset, unpaid counts
  double* d_cegb_lazy_ = nullptr;
  uint32_t* d_cegb_paid_ = nullptr;
  int32_t* d_cegb_cnt_ = nullptr;
  int32_t* d_cegb_scratch_ = nullptr;
  std::vector<char> h_cegb_used_;
  void* d_renew_scratch_ = nullptr;  // percentile renewal (RenewTreeOutputOnDevice)
  int64_t* d_renew_off_ = nullptr;
  double* d_renew_out_ = nullptr;
  const label_t* renew_weight_src_ = nullptr;
  float* d_renew_weights_ = nullptr;
  int vote_k_ = 0;
  double* d_root_local_ = nullptr;      // voting: this rank's root sums
  dev::VoteEntry* d_vote_buf_ = nullptr;  // [world][2][vote_k]
  int32_t* d_vote_list_ = nullptr;        // [2][vote_k]
  long long* d_vote_hist_ = nullptr;      // [2][vote_k][max_feature_bins][2]
  void VoteExchange(const dev::KArgs& glob, bool root);
  // voting: the arguments of the global scan of the elected features (Params::vote_phase 2)
  dev::KArgs VoteGlobalArgs(const dev::KArgs& a, int pick_in_find) const;
  // voting rounds: proposals of every child of the round -> allgather -> elections + elected
  // local histograms -> all-reduce (one of each per round)
  void RoundVoteExchange(const dev::KArgs& glob);
  bool distributed_ = false;    // kData / kFeature on more than one rank
  int world_ = 1, rank_ = 0;
  // feature ownership (distributed): storage-group blocks balanced by bins (SetupOwnership);
  // data-parallel with feature_fraction < 1: re-assigned per tree over the used groups
  struct OwnerLayout {
    std::vector<int> feats, cats;              // this rank's features / categorical ones
    std::vector<int32_t> fb_index, owned_off, rs_pos;
    int max_block = 0, max_feats = 0;          // largest rank block (bins) / feature count
  };
  OwnerLayout BuildOwnerLayout(const std::vector<int>& group_owner) const;  // (owner -1: not scanned)
  void UploadOwnerLayout(const OwnerLayout& layout);
  void OwnershipForTree();
  OwnerLayout static_layout_;
  bool dyn_owner_ = false, owner_layout_static_ = true;
  int cat_cap_ = 1;
  std::vector<int32_t> group_off_, feat_hist_off_;
  int32_t* d_owned_off_ = nullptr;
  std::vector<int> owned_feats_;
  int max_owned_ = 0;           // features of the largest owner (feat_best block of a rank per side)
  int owned_bin_lo_ = 0;
  int rs_block_ = 0;            // padded owner block, histogram bins
  int num_cat_total_ = 0;
  int32_t* d_feat_list_ = nullptr;
  int32_t* d_fb_index_ = nullptr;
  int32_t* d_rs_pos_ = nullptr;
  int32_t* d_owned_cats_ = nullptr;
  long long* d_owned_hist_ = nullptr;
  bool device_mode_ = true;
  bool mode_decided_ = false;  // the first decision is logged too
  bool force_host_mode_ = false;
  double* d_leaf_sums_ = nullptr;
  double* d_root_blk_ = nullptr;  // RootSum's per-workgroup partials
  int device_id_ = 0;
  hipStream_t stream_ = nullptr;
  dev::KArgs args_{};
  std::vector<void*> allocs_;
  // device buffers
  void* d_bins_ = nullptr;
  dev::Feature* d_feat_ = nullptr;
  int32_t* d_group_off_ = nullptr;
  int8_t* d_tree_mask_ = nullptr;
  int8_t* d_node_mask_ = nullptr;       // per-node feature samples of the current tree
  int8_t* d_splittable_ = nullptr;      // [num_leaves][num_features] (KArgs::splittable)
  int8_t* d_parent_flags_ = nullptr;    // [num_features]
  int32_t* d_cat_list_ = nullptr;       // categorical features (KArgs::cat_list)
  dev::IcMask* d_feat_icmask_ = nullptr;  // KArgs::feat_icmask
  std::vector<int8_t> h_node_mask_;     // (kept alive for the async upload)
  // per-node sampling under interaction constraints (bynode_kernels.hip): node pool, generator
  // state, scratch row
  int32_t* d_bynode_pool_ = nullptr;
  uint32_t* d_bynode_rng_ = nullptr;
  int32_t* d_bynode_scratch_ = nullptr;
  std::vector<int32_t> h_bynode_pool_;
  uint32_t h_bynode_rng_ = 0;
  uint32_t* d_xt_base_ = nullptr;       // extra_trees: per-feature generator states, tree start
  int32_t* d_xt_cum_ = nullptr;         // extra_trees: draws per feature after each step
  std::vector<uint32_t> h_xt_base_;
  std::vector<int32_t> h_xt_cum_;
  // voting extra_trees: every rank's global-scan generator set (ResetVoteXt), its device states
  // per tree and running draw counts (KArgs::xt_base_glob / xt_cum_glob)
  std::vector<Random> xt_glob_rand_;
  std::vector<uint32_t> h_xt_base_glob_;
  uint32_t* d_xt_base_glob_ = nullptr;
  int32_t* d_xt_cum_glob_ = nullptr;
  void ResetVoteXt();
  void AllocVoteXt(int n_leaves);
  void VoteXtAdvance();
  dev::GH* d_gh_ = nullptr;
  int32_t* d_idx_ = nullptr;
  int32_t* d_tmp_ = nullptr;
  int32_t* d_oob_ = nullptr;
  int32_t* d_bag_ = nullptr;  // pristine in-bag rows (the partition permutes d_idx_)
  dev::Leaf* d_leaves_ = nullptr;
  dev::Step* d_step_ = nullptr;
  uint32_t* d_find_sub_ = nullptr;  // KArgs::find_sub
  dev::SplitRecord* d_rec_ = nullptr;
  DeviceSplit* d_best_ = nullptr;
  long long* d_hist_ = nullptr;
  long long* d_scratch_ = nullptr;
  double* d_scales_ = nullptr;
  uint32_t* d_absmax_ = nullptr;
  uint8_t* d_bins_col_ = nullptr;
  // row layout (KArgs::bin_bytes / word_g0): per group its byte in a row and width, the
  // word holding it; per word its first group (+ sentinel) and width
  std::vector<int32_t> h_gbyte_, h_word_of_group_, h_word_g0_;
  std::vector<int8_t> h_gwide_, h_word_wide_;
  std::vector<int8_t> h_gnib_;  // 4-bit storage: 2 / 3 the group's low / high half-byte (0: 8 / 16-bit)
  bool nibbles_ = false;        // every group stored in 4 bits (KArgs::nibbles)
  int32_t* d_word_g0_ = nullptr;
  int8_t* d_word_wide_ = nullptr;
  // row-sparse training storage (KArgs::sp_ptr / sp_bin) instead of the word matrix
  bool sparse_rows_ = false;
  int64_t* d_sp_ptr_ = nullptr;
  uint16_t* d_sp_bin_ = nullptr;
  int sp_team_ = 4;  // KArgs::sp_team
  // device forced-split schedule (SetupForcedSplits), rebuilt when the JSON text changes
  std::string forced_text_built_;
  bool forced_ok_ = false;
  int32_t* d_forced_i32_ = nullptr;
  dev::FeatureBest* d_forced_best_ = nullptr;
  uint32_t* d_forced_cat_ = nullptr;
  dev::FeatureBest* d_feat_best_ = nullptr;
  uint32_t* d_feat_cat_ = nullptr;  // category sets of the per-feature categorical bests
  uint32_t* h_absmax_ = nullptr;
  double* h_scales_ = nullptr;
  int rows_cap_ = 4096;      // rows per histogram row block (packed fixed-point headroom)
  int hist_units_ = 1;       // 1 packed (g | h) u64 per bin, 2 wide int64 g / h (WideHistograms)
  static bool WideHistograms(const Config& c);
  int root_grid_ = 512;
  int split_grid_ = 256;
  int blk_min_rows_ = 2048;
  unsigned long long* d_partials_ = nullptr;  // per-workgroup partial histograms
  std::vector<dev::Feature> h_feats_;          // host copy of the feature records
  hipGraphExec_t graph_exec_ = nullptr;        // captured tree (single-process device mode)
  long long* d_ktrace_ = nullptr;              // LGBM_AMD_KTRACE timestamps
  int graph_rows_ = -1;
  int graph_identity_ = -1;
  int graph_root_mode_ = -1;
  int graph_xt_ = -1;
  bool graph_capture_failed_ = false;  // RCCL collectives could not be captured: eager trees
  bool gh_fresh_ = false;         // d_gh_ / absmax / root partials written by the gradient kernel
  bool split_stale_ = false;      // d_grad_ / d_hess_ behind d_gh_ (MaterializeSplitGradients)
  // point-wise device gradients: the last gradient kernel's arguments; the score walk after a
  // tree may compute the next iteration's gradients with them (grad_prefetched_), which the
  // next ComputeGradients then takes instead of launching; any other score change drops them
  dev::GradArgs last_grad_{};
  bool last_grad_fusable_ = false;
  bool grad_prefetched_ = false;
  int grad_parts_ = 0;  // per-workgroup partials (max_parts / root_parts) of the last gradients
  bool root_from_parts_ = false;  // this tree's gradients came packed from the gradient kernel
  double* d_root_parts_ = nullptr;
  float* d_max_parts_ = nullptr;
  double* d_root_ = nullptr;
  double* d_score_ = nullptr;
  float* d_grad_ = nullptr;
  float* d_hess_ = nullptr;
  double* d_leaf_values_ = nullptr;
  float* d_label_ = nullptr;
  float* d_weights_ = nullptr;
  float* d_label_weight_ = nullptr;
  const label_t* uploaded_label_src_ = nullptr;
  const label_t* uploaded_weight_src_ = nullptr;
  const label_t* uploaded_lw_src_ = nullptr;
  // listwise objectives: query tables (uploaded once) and the xendcg generators
  int32_t* d_qb_ = nullptr;
  double* d_inv_max_dcg_ = nullptr;
  double* d_label_gain_ = nullptr;
  double* d_discount_ = nullptr;
  double* d_sig_table_ = nullptr;  // lambdarank: the objective's sigmoid table
  // listwise queries of more than kRankMaxDocs documents and their global scratch (RankArgs::big_*)
  int32_t* d_rank_big_q_ = nullptr;
  int32_t rank_num_big_ = 0;
  double *d_rank_big_d0_ = nullptr, *d_rank_big_d1_ = nullptr, *d_rank_big_dh_ = nullptr;
  int32_t rank_max_docs_ = 0;             // most documents of a query staged in LDS
  float2* d_rank_pairs_ = nullptr;        // lambdarank pair scratch (RankArgs::pair_buf), or null
  int64_t* d_rank_pair_off_ = nullptr;
  float* d_rank_big_f_ = nullptr;
  int32_t *d_rank_big_i0_ = nullptr, *d_rank_big_i1_ = nullptr, *d_rank_big_i2_ = nullptr;
  uint32_t* d_rank_rng_ = nullptr;
  const data_size_t* uploaded_qb_src_ = nullptr;
  // device row sampling (bagging / GOSS)
  uint32_t* d_sample_rng_ = nullptr;
  uint8_t* d_sample_codes_ = nullptr;
  int32_t* d_sample_cnt_ = nullptr;
  int32_t* d_sample_off_ = nullptr;
  int32_t* d_bag_count_ = nullptr;  // in-bag rows of the current bag (read by the root kernels)
  bool sample_seeded_ = false;
  // validation sets on the device (own allocations: they survive ResetTrainingData)
  struct ValidSet {
    void* bins = nullptr;
    double* score = nullptr;
    data_size_t num_data = 0;
    int ntpi = 1;
    float* label = nullptr;    // metric inputs, uploaded on the first device evaluation
    float* weights = nullptr;
    const void* label_src = nullptr;    // the host arrays they were uploaded from
    const void* weights_src = nullptr;
    bool negative_weights = false;      // (AUC carries the class in the weight's sign: host then)
    void* metric_scratch = nullptr;
    data_size_t metric_scratch_rows = 0;  // rows metric_scratch is sized for (AUC)
    double* metric_out = nullptr;
    struct QueryInputs {  // one query metric's device inputs (NDCG / MAP)
      int32_t* qb = nullptr;
      float* qw = nullptr;
      int32_t* eval_at = nullptr;
      double* qconst = nullptr;
      double* label_gain = nullptr;
      double* discount = nullptr;
      void* scratch = nullptr;
      bool big = false;  // a query longer than the LDS staging
    };
    std::unordered_map<const void*, QueryInputs> queries;
    std::set<int> logged_kinds;  // metric kinds evaluated here so far (debug log)
  };
  std::vector<ValidSet> valid_;
  int train_eval_slot_ = -1;  // valid_ entry over the training scores (d_score_; no bins)
  std::vector<void*> valid_allocs_;
  void ReleaseValidInputs(ValidSet* vs);  // frees a set's metric inputs (not its bins / scores)
  // tree upload for the score traversal: one blob (node arrays, category sets, leaf values)
  // per tree, one H2D copy from a ring of pinned staging slots (each reused once its event --
  // recorded after its copy -- has completed: no stream synchronisation per tree)
  struct StageSlot {
    char* host = nullptr;
    size_t cap = 0;
    hipEvent_t done = nullptr;
  };
  static constexpr int kStageSlots = 4;
  StageSlot stage_slots_[kStageSlots];
  int stage_next_ = 0;
  char* d_tree_blob_ = nullptr;
  // ExpectTrainingScoreUpdate: the promised shrinkage of the next tree; the tree the device
  // added to the training scores early (its leaves; 0: none) and its DevTree blob
  double expect_shrinkage_ = 0.0, train_shrink_ = 0.0;
  int early_scored_leaves_ = 0;
  char* d_early_blob_ = nullptr;
  hipEvent_t rec_event_ = nullptr;  // the split records' copy (round growth)
  size_t tree_blob_cap_ = 0;
  unsigned long long* d_tree_bm_ = nullptr;  // per-node decision bitmaps (score traversal)
  int32_t* d_tree_bm_meta_ = nullptr;
  int tree_bm_cap_ = 0;
  // pinned host staging
  int8_t* h_mask_ = nullptr;
  dev::SplitRecord* h_rec_ = nullptr;
  dev::Step* h_step_ = nullptr;
  double* h_root_ = nullptr;
  // sizes
  int num_groups_ = 0;
  int total_bins_ = 0;
  int num_tree_per_iteration_ = 1;
  data_size_t root_rows_ = 0;
  data_size_t oob_cnt_ = 0;
  std::vector<data_size_t> global_count_;
  mutable bool host_partition_fresh_ = false;
  bool in_trained_update_ = false;
};

}  // namespace lgbm_amd
