// MI355X tree learner: round growth orchestration -- pools, the round sequence and its
// collectives, the growth-mode choice and the host loop over round segments (round_kernels.hip).
#include <atomic>
#include <chrono>
#include <thread>

#include "gpu_learner_internal.h"
#include "lgbm_amd/tuning.h"

namespace lgbm_amd {

// histogram slots and splittable rows (nodes) of a tree: one slot per leaf, or -- round
// growth -- one per expansion (the root's, then the histogrammed child's of each), two nodes
// per expansion; 3 * num_leaves expansions leave the speculation 2 * num_leaves of waste,
// 2 * num_leaves when the slots would pass 16 GiB
void GPUTreeLearner::SizeRoundPools(int n_leaves) {
  hist_slots_ = n_leaves;
  split_rows_ = n_leaves;
  if (round_k_ > 1) {
    const double slot_bytes = 16.0 * static_cast<double>(total_bins_);
    const int per = slot_bytes * 3.0 * n_leaves > 16.0 * (1ull << 30) ? 2 : 3;
    hist_slots_ = per * n_leaves;
    split_rows_ = 2 * per * n_leaves;
  }
  args_.round_nodes = split_rows_;
  args_.round_emax = std::min(hist_slots_ - 1, (split_rows_ - 1) / 2);
  args_.round_vmax = round_vmax_;
}

void GPUTreeLearner::AllocRoundState() {
  dev::KArgs& a = args_;
  a.rnode = nullptr;
  a.cbest = nullptr;
  a.cbest_cat = nullptr;
  a.child_cnt = nullptr;
  a.round_bynode = 0;
  a.node_fb = nullptr;
  a.leaf_rows = nullptr;
  a.round_xt = 0;
  a.node_pre = nullptr;
  a.round_cegb = 0;
  a.node_fb_cat = nullptr;
  a.node_cat_slot = nullptr;
  a.node_cat_slots = 0;
  if (round_k_ <= 1) return;
  d_round_ = Alloc<dev::Round>(1);
  d_rnode_ = Alloc<dev::RNode>(split_rows_);
  d_cbest_ = Alloc<dev::FeatureBest>(split_rows_);
  if (a.round_vote) a.rnode_lsum = Alloc<double>(2 * static_cast<size_t>(split_rows_));  // (voting: local node sums)
  d_cbest_cat_ = Alloc<uint32_t>(static_cast<size_t>(split_rows_) * kMaxCatWords);
  const size_t cnt = 2 * static_cast<size_t>(dev::kMaxRoundExp) * (dev::kFindSub + 1) * dev::kFindSubStride;
  d_child_cnt_ = Alloc<uint32_t>(cnt);
  HIPCHECK(hipMemset(d_child_cnt_, 0, sizeof(uint32_t) * cnt));
  HIPCHECK(hipMemset(d_round_, 0, sizeof(dev::Round)));
  if (h_round_ == nullptr) {
    HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&h_round_), sizeof(dev::Round), hipHostMallocDefault));
  }
  if (h_tree_out_ != nullptr) (void)hipHostFree(h_tree_out_);
  HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&h_tree_out_),
                         sizeof(int32_t) * dev::kHostOutHeaderWords +
                             sizeof(dev::SplitRecord) * std::max(1, config_->num_leaves - 1),
                         hipHostMallocCoherent));
  a.rnode = d_rnode_;
  a.cbest = d_cbest_;
  a.cbest_cat = d_cbest_cat_;
  a.child_cnt = d_child_cnt_;
  round_hist_.clear();
  // per-node sampling on round growth (KArgs::round_bynode): one process or the data- /
  // feature-parallel learners (every rank draws the same samples; k_round_childbest completes
  // each rank's per-node results and flags from the gathered records), no interaction
  // constraints (categorical features: their category sets are kept per node)
  bool any_cat = false;
  for (int f = 0; f < num_features_; ++f) any_cat = any_cat || data_->FeatureBinMapper(f)->bin_type() == BinType::Categorical;
  const bool base_rounds = config_->interaction_constraints_vector.empty() && !voting_;
  const bool simple_rounds = base_rounds && !any_cat;
  // (categorical features: each node keeps its categorical features' category sets)
  std::vector<int32_t> cat_slot(std::max(1, num_features_), -1);
  int ncs = 0;
  for (int f = 0; f < num_features_; ++f) {
    if (data_->FeatureBinMapper(f)->bin_type() == BinType::Categorical) cat_slot[f] = ncs++;
  }
  const double cat_bytes = static_cast<double>(split_rows_) * ncs * kMaxCatWords * sizeof(uint32_t);
  const bool bynode = config_->feature_fraction_bynode < 1.0 && base_rounds && cat_bytes <= 2.0 * (1ull << 30) &&
                      !tuning::Off(tuning::Knob::ByNodeRounds);
  // extra_trees on round growth (KArgs::round_xt): also no CEGB or forced splits, at most
  // kXtLaneFeatures * 64 features (the replay's draw counters), prefix tables under 8 GiB
  const double pre_bytes = static_cast<double>(split_rows_) * total_bins_ * sizeof(dev::XtPre);
  const bool xt = config_->extra_trees && simple_rounds && !distributed_ && !CostEffectiveGB::Enabled(*config_) &&
                  config_->forcedsplits_filename.empty() && num_features_ <= 4 * 64 &&
                  pre_bytes <= 8.0 * (1ull << 30) && !tuning::Off(tuning::Knob::XtRounds);
  // CEGB coupled penalties on round growth (KArgs::round_cegb): also no lazy penalties or
  // monotone constraints (the replay subtracts the penalties from raw candidates)
  const bool mono = std::any_of(config_->monotone_constraints.begin(), config_->monotone_constraints.end(),
                                [](int8_t m) { return m != 0; });
  const bool cegb = CostEffectiveGB::Enabled(*config_) && !config_->cegb_penalty_feature_coupled.empty() &&
                    config_->cegb_penalty_feature_lazy.empty() && simple_rounds && !mono &&
                    !tuning::Off(tuning::Knob::CegbRounds);
  const size_t nf = static_cast<size_t>(std::max(1, num_features_));
  if (bynode || xt || cegb) {
    a.leaf_rows = Alloc<int8_t>(static_cast<size_t>(config_->num_leaves) * nf);
    HIPCHECK(hipMemset(a.leaf_rows, 1, static_cast<size_t>(config_->num_leaves) * nf));  // (SerialTreeLearner::Init)
  }
  if (bynode || cegb) a.node_fb = Alloc<dev::FeatureBest>(static_cast<size_t>(split_rows_) * nf);
  if (bynode) a.round_bynode = 1;
  if (bynode && ncs > 0) {
    a.node_fb_cat = Alloc<uint32_t>(static_cast<size_t>(split_rows_) * ncs * kMaxCatWords);
    int32_t* slots = Alloc<int32_t>(cat_slot.size());
    HIPCHECK(hipMemcpy(slots, cat_slot.data(), sizeof(int32_t) * cat_slot.size(), hipMemcpyHostToDevice));
    a.node_cat_slot = slots;
    a.node_cat_slots = ncs;
  }
  if (cegb) a.round_cegb = 1;
  if (xt) {
    a.node_pre = Alloc<dev::XtPre>(static_cast<size_t>(split_rows_) * total_bins_);
    a.round_xt = 1;
    a.plan_in_find = 0;  // (the extra_trees replay is compiled into k_round_plan only)
  }
}

// one round: single process, every kernel back to back; distributed, the histograms
// reduce-scattered to their owners (data-parallel) and the per-feature results of every rank
// gathered before the children's bests and the plan -- two collectives per round where one
// split per step took two per split (reference data_parallel_tree_learner.cpp:154-247)
void GPUTreeLearner::EnqueueRound(const dev::KArgs& a) {
  if (!distributed_) {
    dev::RoundStep(a, stream_);
    return;
  }
  DeviceComm* dc = Network::device_comm();
  // a finished tree's remaining rounds skip their collectives on every rank (Round::done is
  // replicated state); communicators that cannot skip run them.  The guard is cleared on every
  // exit of this scope: a throw between here and the last collective (a failed launch caught
  // by the graph capture) must not leave later collectives guarded by a stale flag
  struct SkipGuardScope {
    DeviceComm* dc;
    ~SkipGuardScope() { dc->SetSkipGuard(nullptr); }
  } guard_scope{dc};
  dc->SetSkipGuard(&d_round_->done);
  if (voting_) {
    // the local scan of every child of the round, one vote for all of them, the global scan of
    // the elected features (reference voting_parallel_tree_learner.cpp:300-343, per round)
    const dev::KArgs glob = VoteGlobalArgs(a, 0);
    dev::RoundSplitReduce(a, stream_);
    dev::RoundFind(a, stream_);
    RoundVoteExchange(glob);
    dev::RoundFindElected(glob, stream_);
    dc->SetSkipGuard(nullptr);
    dev::RoundChildBestAndPlan(glob, stream_);
    return;
  }
  const size_t owned = static_cast<size_t>(round_k_) * rs_block_ * 2;
  // (the owner-major send buffer was cleared by the previous round's split scans, or by the root)
  dev::RoundSplitReduce(a, stream_);
  if (data_parallel_) dc->ReduceScatterSumI64(d_round_send_, d_round_owned_, owned, stream_);
  dev::RoundFind(a, stream_);
  const size_t per = 2 * static_cast<size_t>(round_k_) * std::max(1, max_owned_);
  char* fb = reinterpret_cast<char*>(d_feat_best_);
  dc->Allgather(fb + per * sizeof(dev::FeatureBest) * rank_, fb, per * sizeof(dev::FeatureBest), stream_);
  if (num_cat_total_ > 0) {
    char* fc = reinterpret_cast<char*>(d_feat_cat_);
    const size_t cb = per * kMaxCatWords * sizeof(uint32_t);
    dc->Allgather(fc + cb * rank_, fc, cb, stream_);
  }
  dc->SetSkipGuard(nullptr);  // (the plan's kernels are not collectives)
  dev::RoundChildBestAndPlan(a, stream_);
}

void GPUTreeLearner::RoundVoteExchange(const dev::KArgs& glob) {
  DeviceComm* dc = Network::device_comm();  // (round growth runs with a device communicator only)
  dev::RoundVoteLocal(glob, stream_);
  const size_t prop_bytes = sizeof(dev::VoteEntry) * 2 * static_cast<size_t>(round_k_) * vote_k_;
  char* vb = reinterpret_cast<char*>(d_vote_buf_);
  dc->Allgather(vb + prop_bytes * rank_, vb, prop_bytes, stream_);
  dev::RoundVoteElect(glob, stream_);
  dc->AllreduceSumI64(d_vote_hist_, 2 * static_cast<size_t>(round_k_) * vote_k_ * 2 * glob.p.max_feature_bins, stream_);
}

double GPUTreeLearner::RoundCollectiveBytes() const {
  if (!distributed_) return 0.0;
  if (voting_) {
    const double sides = 2.0 * round_k_ * vote_k_;
    return sides * sizeof(dev::VoteEntry) * world_ + sides * 2.0 * args_.p.max_feature_bins * sizeof(long long);
  }
  const double per = 2.0 * round_k_ * std::max(1, max_owned_) *
                     (sizeof(dev::FeatureBest) + (num_cat_total_ > 0 ? kMaxCatWords * sizeof(uint32_t) : 0)) * world_;
  return per + (data_parallel_ ? sizeof(long long) * 2.0 * round_k_ * rs_block_ * world_ : 0.0);
}

// ---------------------------------------------------------------- round growth
// Round growth or one split per step (the trees are the same): rounds trade the per-split
// latency chain for speculative work, which on large data (Criteo-shaped 255-leaf trees from
// ~50M rows per GPU, profiles/r04_speculation_big_shards.md) costs more than the latency it
// hides.  From 16M rows per rank (LGBM_AMD_ROUND_AUTO=1: always, 0: never) trees 1-2 are timed
// with rounds and tree 4 with one split per step (3 captures its graph); the faster mode grows
// every later tree.  Distributed ranks sum their times first, so all of them switch together.
bool GPUTreeLearner::AutoGrowthRounds() {
  if (auto_state_ == kAutoUnset) {
    const char* e = tuning::Get(tuning::Knob::RoundAuto);
    double rows = static_cast<double>(num_data_);
    if (distributed_ && Network::num_machines() > 1) {
      std::vector<double> v{rows};
      rows = Network::GlobalSum(v)[0] / Network::num_machines();
    }
    const bool on = e != nullptr ? e[0] == '1' : rows >= tuning::kRoundAutoRows;
    auto_state_ = on ? kAutoProbe : kAutoRounds;
    auto_tree_ = 0;
  }
  if (auto_state_ == kAutoSteps) return false;
  if (auto_state_ == kAutoProbe) return !(auto_tree_ == 3 || auto_tree_ == 4);
  return true;
}

void GPUTreeLearner::AutoGrowthRecord(double ms) {
  if (auto_state_ != kAutoProbe) return;
  if (auto_tree_ == 1 || auto_tree_ == 2) auto_rounds_ms_ = std::min(auto_rounds_ms_, ms);
  if (auto_tree_ == 4) {
    std::vector<double> v{auto_rounds_ms_, ms};
    if (distributed_ && Network::num_machines() > 1) v = Network::GlobalSum(v);
    auto_state_ = v[1] < 0.97 * v[0] ? kAutoSteps : kAutoRounds;
    Log::Info("device learner: growth timed at %.2f ms per tree with rounds, %.2f with one split per step: %s",
              v[0] / std::max(1, distributed_ ? Network::num_machines() : 1),
              v[1] / std::max(1, distributed_ ? Network::num_machines() : 1),
              auto_state_ == kAutoSteps ? "one split per step from here on" : "rounds");
  }
  ++auto_tree_;
}

bool GPUTreeLearner::RoundGrowth(const dev::KArgs& a) const {
  if (round_k_ <= 1 || d_round_ == nullptr) return false;
  if (distributed_ && Network::device_comm() == nullptr) return false;  // (host collectives: one split per step)
  // the split order depends on more than each leaf's own rows: per-node feature samples and
  // extra_trees draws are consumed in the sequential order, CEGB's coupled penalties change
  // other leaves' gains, forced splits follow their own schedule
  // (per-node sampling without interaction constraints folds each node's sample at the replay:
  // KArgs::round_bynode)
  if (a.node_mask != nullptr && !(a.round_bynode && a.bynode_rng == nullptr)) return false;
  if ((a.xt_base != nullptr && !a.round_xt) || a.forced_n > 0 || a.p.mono_inter) return false;
  if (a.p.cegb && !CegbRounds(a)) return false;
  return true;
}

// CEGB on round growth (one process or data- / feature-parallel, no lazy penalties).  A scan subtracts the split penalty,
// tradeoff * penalty_split * rows, which depends on the node's own rows only.  A coupled
// penalty depends on whether the model has used the feature, and a feature's first use refunds
// the other leaves' remembered candidates (CostEfficientGradientBoosting::UpdateLeafBestSplits):
// both change within a tree only while some feature of the tree's sample is still unused.  So a
// tree grows in rounds once every feature of its sample is used -- its splits cannot use a new
// feature, the coupled terms are 0 and no refund happens; the candidates a refund would read
// later are of features outside this tree's sample (not scanned here).  Earlier trees grow one
// split per step, as do all trees with lazy penalties.
bool GPUTreeLearner::CegbRounds(const dev::KArgs& a) const {
  if (voting_ || a.cegb_lazy != nullptr || cegb_ == nullptr) return false;
  if (a.cegb_coupled == nullptr || a.round_cegb) return true;  // (round_cegb: refunds in the replay)
  const std::vector<char>& used = cegb_->used_in_split();
  for (int f = 0; f < num_features_; ++f) {
    if (h_mask_[f] && (f >= static_cast<int>(used.size()) || !used[f])) return false;
  }
  return true;
}

// One root graph (the root + a number of rounds, one cached graph per count) and segment graphs
// of round_seg_ rounds are enqueued up to the provisioned count (the most rounds of the recent
// trees + margin); the host then checks the Round record and adds segments until the tree is
// done (a finished tree's kernels exit at once: an over-provisioned round costs ~12 us, a
// missing one a host round trip and a graph launch per segment)

int GPUTreeLearner::RunRounds(dev::KArgs a) {
  RoundLaunch rl = LaunchRounds(a);
  return WaitRounds(&rl);
}

// the tree's root graph and its provisioned rounds, enqueued without waiting (also the
// speculative launch of the next tree, LaunchSpeculative)
GPUTreeLearner::RoundLaunch GPUTreeLearner::LaunchRounds(dev::KArgs a) {
  common::ScopedTimer timer("GPUTreeLearner::LaunchRounds");
  a.rd = d_round_;
  // one process: the tree's last plan hands its records and scalars to the host directly
  a.host_out = (!distributed_ && !tuning::Off(tuning::Knob::HostOut)) ? h_tree_out_ : nullptr;
  volatile int32_t* flag = a.host_out;
  if (flag != nullptr) {
    flag[0] = 0;  // (the previous tree's writer is long done: the host waited for it)
    std::atomic_thread_fence(std::memory_order_seq_cst);
  }
  if (k_adapt_ && !k_adapt_checked_) {
    k_adapt_checked_ = true;
    double rows = static_cast<double>(num_data_);
    if (distributed_ && Network::num_machines() > 1) {
      std::vector<double> v{rows};
      rows = Network::GlobalSum(v)[0] / Network::num_machines();
    }
    k_adapt_ = rows >= tuning::kRoundAdaptRows;
  }
  if (k_adapt_) {
    // this tree's round width (Round::k_cur: the captured graphs are sized for round_k_)
    k_cur_host_ = (prev_splits_ <= 0 || prev_expansions_ <= prev_splits_ + 2) ? round_k_ : std::min(round_k_, tuning::kRoundWidthNarrow);
    HIPCHECK(hipMemcpyAsync(&d_round_->k_cur, &k_cur_host_, sizeof(int32_t), hipMemcpyHostToDevice, stream_));
  }
  a.pick_in_find = 0;  // the root's split scan only publishes; RoundRootPlan picks
  // (LGBM_AMD_KTRACE: k_round_split's phase times of one workgroup per round)
  if (a.ktrace != nullptr) HIPCHECK(hipMemsetAsync(a.ktrace, 0, sizeof(long long) * dev::kTraceSlots * config_->num_leaves, stream_));
  const char* ng = tuning::Get(tuning::Knob::NoGraph);
  // distributed: the collectives are captured with the kernels when the communicator allows it
  // (RCCL); the in-process communicator rendezvouses on the host, so its rounds run eagerly
  DeviceComm* dc = distributed_ ? Network::device_comm() : nullptr;
  const bool use_graph = !(ng != nullptr && ng[0] == '1') && (dc == nullptr || dc->CaptureSafe()) && !graph_capture_failed_;
  const int root_mode = (root_from_parts_ && !use_bag_) ? 1 : 0;
  auto capture = [&](hipGraphExec_t* exec, bool root, int rounds) {
    hipGraph_t g = nullptr;
    HIPCHECK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
    std::string why;
    try {
      if (root) EnqueueRoot(a);
      for (int r = 0; r < rounds; ++r) EnqueueRound(a);
    } catch (const std::exception& e) {
      why = e.what();
    }
    hipError_t ec = hipStreamEndCapture(stream_, &g);
    if (why.empty() && ec == hipSuccess) ec = hipGraphInstantiate(exec, g, nullptr, nullptr, 0);
    if (g != nullptr) (void)hipGraphDestroy(g);
    if (!why.empty() || ec != hipSuccess) {
      if (why.empty()) why = hipGetErrorString(ec);
      (void)hipGetLastError();
      *exec = nullptr;
      if (!distributed_) Log::Fatal("device learner: capturing the round graphs failed: %s", why.c_str());
      Log::Warning("device learner: capturing the round collectives failed (%s); launching rounds eagerly", why.c_str());
      graph_capture_failed_ = true;
      return false;
    }
    return true;
  };
  const int L = config_->num_leaves;
  static const int env_hist = tuning::Int(tuning::Knob::RoundHist, 0), env_margin = tuning::Int(tuning::Knob::RoundMargin, -99),
                   env_seg = tuning::Int(tuning::Knob::RoundSeg, 0), env_root = tuning::Int(tuning::Knob::RoundRoot, -1);
  if (env_hist > 0) round_hist_n_ = static_cast<size_t>(env_hist);
  if (env_margin > -99) round_margin_ = env_margin;
  if (env_seg > 0) round_seg_ = env_seg;
  if (env_root >= 0) round_root_fixed_ = env_root;
  const int seg = round_seg_;
  // rounds to enqueue: the most rounds of the last trees (+ margin)
  int want = tuning::kRoundFirstTree;
  if (!round_hist_.empty()) want = *std::max_element(round_hist_.begin(), round_hist_.end()) + round_margin_;
  want = std::max(1, std::min(want, L - 1));
  // the root graph: a fixed number of rounds, or exactly the provisioned count (one cached graph
  // per count; rounding up to whole segments ran ~1.5 no-op rounds of three launches per tree);
  // segment graphs make up the rest before the host first looks at the Round record
  const int root_rounds = round_root_fixed_ > 0 ? std::min(round_root_fixed_, want) : want;
  bool graph = use_graph;
  if (graph && (round_seg_exec_ == nullptr || round_graph_rows_ != a.num_rows ||
                round_graph_identity_ != a.root_identity || round_graph_root_mode_ != root_mode)) {
    if (dc != nullptr) dc->HostBarrier();
    DestroyRoundGraphs();
    graph = capture(&round_seg_exec_, false, seg);
    if (!graph) DestroyRoundGraphs();
    round_graph_rows_ = a.num_rows;
    round_graph_identity_ = a.root_identity;
    round_graph_root_mode_ = root_mode;
  }
  if (graph) {
    if (static_cast<int>(round_root_execs_.size()) <= root_rounds) round_root_execs_.resize(root_rounds + 1, nullptr);
    if (round_root_execs_[root_rounds] == nullptr) {
      if (dc != nullptr) dc->HostBarrier();
      graph = capture(&round_root_execs_[root_rounds], true, root_rounds);
      if (!graph) DestroyRoundGraphs();
    }
  }
  RoundLaunch rl;
  rl.a = a;
  rl.graph = graph;
  rl.seg = seg;
  if (graph) {
    common::ScopedTimer launch_timer("GPUTreeLearner::RootGraphLaunch");
    HIPCHECK(hipGraphLaunch(round_root_execs_[root_rounds], stream_));
  } else {
    EnqueueRoot(a);
    for (int r = 0; r < root_rounds; ++r) EnqueueRound(a);
  }
  rl.launched = root_rounds;
  while (rl.launched < want) {  // (asynchronous: enqueued while the root graph runs)
    LaunchSegment(rl);
    rl.launched += seg;
  }
  return rl;
}

void GPUTreeLearner::LaunchSegment(const RoundLaunch& rl) {
  if (rl.graph) {
    common::ScopedTimer launch_timer("GPUTreeLearner::SegmentGraphLaunch");
    HIPCHECK(hipGraphLaunch(round_seg_exec_, stream_));
  } else {
    for (int r = 0; r < rl.seg; ++r) EnqueueRound(rl.a);
  }
}

// the host side of a launched tree: wait for its last plan (more segments if the provisioned
// rounds did not finish it), then its counters
int GPUTreeLearner::WaitRounds(RoundLaunch* rlp) {
  common::ScopedTimer timer("GPUTreeLearner::RunRounds");
  RoundLaunch& rl = *rlp;
  const dev::KArgs& a = rl.a;
  volatile int32_t* flag = a.host_out;
  const int L = config_->num_leaves, seg = rl.seg;
  int& launched = rl.launched;
  auto launch_seg = [&]() { LaunchSegment(rl); };
  last_stats_.graph = rl.graph;
  // the host reads the Round record's scalars only (done, splits, rounds, nodes); the split
  // records follow once the tree is done (TrainDeviceMode)
  constexpr size_t kRoundHeader = offsetof(dev::Round, cur);
  tree_out_used_ = flag != nullptr;
  if (flag != nullptr) {
    // spin on the flag (it is set while the stream may still run the tree's surplus rounds);
    // every ~20 us look whether the stream ran dry without it: then the tree needs more rounds
    // (a pause per read; past the first millisecond the thread yields between reads, so a long
    // tree does not hold a host core the OpenMP host work could use; time_out bounds the wait)
    const auto t0 = std::chrono::steady_clock::now();
    auto last = t0;
    const double limit_s = 60.0 * std::max(1, config_->time_out);
    for (;;) {
      if (flag[0] != 0) break;
      __builtin_ia32_pause();
      const auto now = std::chrono::steady_clock::now();
      if (now - last < std::chrono::microseconds(20)) {
        if (now - t0 > std::chrono::milliseconds(1)) std::this_thread::yield();
        continue;
      }
      last = now;
      const hipError_t q = hipStreamQuery(stream_);
      if (q == hipErrorNotReady) {
        if (std::chrono::duration<double>(now - t0).count() > limit_s) {
          Log::Fatal("device learner: the tree's rounds did not finish within time_out=%d min", config_->time_out);
        }
        continue;
      }
      HIPCHECK(q);
      if (flag[0] != 0) break;
      if (launched > 2 * L + seg) {
        Log::Fatal("device learner: round growth did not finish the tree after %d rounds", launched);
      }
      launch_seg();
      launched += seg;
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    h_round_->done = 1;
    h_round_->nsplit = flag[1];
    h_round_->rounds = flag[2];
    h_round_->next_frow = flag[3];
    h_round_->bynode_next = flag[4];
  } else {
    for (;;) {
      HIPCHECK(hipMemcpyAsync(h_round_, d_round_, kRoundHeader, hipMemcpyDeviceToHost, stream_));
      WatchdogSync();
      if (h_round_->done) break;
      if (launched > 2 * L + seg) {
        Log::Fatal("device learner: round growth did not finish the tree after %d rounds (%d splits)", launched,
                   h_round_->nsplit);
      }
      launch_seg();
      launched += seg;
    }
  }
  if (a.ktrace != nullptr) {
    std::vector<long long> t(static_cast<size_t>(L) * dev::kTraceSlots);
    HIPCHECK(hipMemcpy(t.data(), a.ktrace, sizeof(long long) * t.size(), hipMemcpyDeviceToHost));
    static const char* names[] = {"stage", "side", "resv", "write", "gather", "tail", "store"};
    // plans: slot 16 entry time, 17..21 phase times (loads, replay, prediction with the records
    // of the accepted splits / changed leaves beside it and then the expansions' records,
    // barrier, sizing + plan stores), 22 accepted, 23 planned, 25 the split scan's start
    for (int r = 0; r <= h_round_->rounds && r < L; ++r) {
      const long long* o = &t[static_cast<size_t>(r) * dev::kTraceSlots];
      if (o[16] == 0) continue;
      std::fprintf(stderr, "plan %d: scan->plan %.2f loads=%.2f replay=%.2f predict+records=%.2f (predict %.2f) sync=%.2f sizing+stores=%.2f us; accepted %lld planned %lld\n",
                   r, o[25] != 0 ? (o[16] - o[25]) / 100.0 : 0.0, o[17] / 100.0, o[18] / 100.0, o[19] / 100.0, o[24] / 100.0,
                   o[20] / 100.0, o[21] / 100.0, o[22], o[23]);
      if (o[26] != 0) {  // the planning workgroup's scan path, from the first scan workgroup's start
        auto us = [&](int k) { return (o[k] - o[25]) / 100.0; };
        std::fprintf(stderr, "  planner wg: entry %.2f loaded %.2f staged %.2f scanned %.2f arrived %.2f folded %.2f plan %.2f us\n",
                     us(26), us(27), us(28), us(29), us(30), us(31), us(16));
        if (o[12] != 0) {  // (LGBM_FIND_PHASES builds: the scan's phases)
          std::fprintf(stderr, "  planner scan: begin %.2f prefix %.2f candidates %.2f argmax %.2f us\n", us(12), us(13),
                       us(14), us(15));
        }
      }
    }
    for (int r = 1; r <= h_round_->rounds && r < L; ++r) {
      const long long* o = &t[static_cast<size_t>(r) * dev::kTraceSlots];
      std::string line = "round " + std::to_string(r) + " exp " + std::to_string(o[10]) + " blocks " +
                         std::to_string(o[11]) + " wg0: subtiles " + std::to_string(o[7]) + " rows " +
                         std::to_string(o[8]) + " us";
      char buf[64];
      for (int k = 0; k < 7; ++k) {
        std::snprintf(buf, sizeof(buf), " %s=%.2f", names[k], o[k] / 100.0);
        line += buf;
      }
      std::snprintf(buf, sizeof(buf), " total=%.2f", o[9] / 100.0);
      std::fprintf(stderr, "%s%s\n", line.c_str(), buf);
    }
  }
  // the next tree enqueues the most rounds of the last round_hist_n_ trees (+ margin)
  round_hist_.push_back(h_round_->rounds);
  while (round_hist_.size() > round_hist_n_) round_hist_.erase(round_hist_.begin());
  last_stats_.rounds = h_round_->rounds;
  last_stats_.expansions = (h_round_->next_frow - 1) / 2;
  prev_expansions_ = last_stats_.expansions;
  prev_splits_ = h_round_->nsplit;
  // (every enqueued round's collectives run; a finished tree's exit at once)
  last_stats_.collective_bytes = distributed_ ? root_collective_bytes_ + RoundCollectiveBytes() * launched : 0.0;
  return h_round_->nsplit;
}

// a leaf's raw histogram: its slot, or -- round growth, for a node whose pending expansion
// reused its slot for the subtracted child -- per feature the sum over its children where the
// node evaluated the feature (its children materialised it), recursively; elsewhere the
// node's slot, which its subtracted descendants inherit without touching that feature's bins
// (self checks only)
void GPUTreeLearner::ReadHist(const dev::Leaf& lf, int leaf, std::vector<long long>* raw) const {
  (void)leaf;
  const size_t nh = 2 * static_cast<size_t>(total_bins_);
  raw->assign(nh, 0);
  auto read_slot = [&](int slot, std::vector<long long>* out) {
    out->resize(nh);
    HIPCHECK(hipMemcpy(out->data(), d_hist_ + static_cast<size_t>(slot) * nh, sizeof(long long) * nh,
                       hipMemcpyDeviceToHost));
  };
  if (d_rnode_ == nullptr || last_stats_.rounds == 0 || lf.frow < 0) {  // (one split per step: Leaf::frow is no node)
    read_slot(lf.slot, raw);
    return;
  }
  std::function<void(int, std::vector<long long>*)> node_hist = [&](int n, std::vector<long long>* out) {
    dev::RNode r{};
    HIPCHECK(hipMemcpy(&r, d_rnode_ + n, sizeof(r), hipMemcpyDeviceToHost));
    read_slot(r.st.slot, out);
    if (!r.expanded) return;
    dev::RNode c{};
    HIPCHECK(hipMemcpy(&c, d_rnode_ + r.child, sizeof(c), hipMemcpyDeviceToHost));
    const int md = config_->min_data_in_leaf;
    const int lc = r.total_left, rc = r.count - r.total_left;
    // (children of an expansion that cannot be split are not histogrammed)
    if ((config_->max_depth > 0 && c.st.depth >= config_->max_depth) || (lc < 2 * md && rc < 2 * md)) return;
    std::vector<int8_t> flags(num_features_);
    HIPCHECK(hipMemcpy(flags.data(), d_splittable_ + static_cast<size_t>(n) * num_features_, num_features_,
                       hipMemcpyDeviceToHost));
    std::vector<long long> h0, h1;
    node_hist(r.child, &h0);
    node_hist(r.child + 1, &h1);
    for (int f = 0; f < num_features_; ++f) {
      if (!flags[f]) continue;
      const size_t off = 2 * static_cast<size_t>(data_->FeatureHistOffset(f));
      const size_t len = 2 * static_cast<size_t>(data_->FeatureHistSize(f));
      for (size_t i = off; i < off + len; ++i) (*out)[i] = h0[i] + h1[i];
    }
  };
  node_hist(lf.frow, raw);
}

}  // namespace lgbm_amd
