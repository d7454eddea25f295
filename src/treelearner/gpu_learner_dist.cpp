// MI355X tree learner: distributed parts -- feature ownership, the root / histogram / record
// collectives of the one-split-per-step sequence and the voting exchange.
#include "gpu_learner_internal.h"
#include "lgbm_amd/tuning.h"

namespace lgbm_amd {

// Feature ownership of the distributed learners (reference data_parallel_tree_learner.cpp
// BeforeTrain :61-123 assigns the tree's used features to the least-loaded rank by bins).
// Here a rank owns whole storage groups; its groups' bins, packed in group order, are its
// block of the owner-major reduce-scatter buffer (rs_pos), and its features are gathered
// rank-major after each scan (fb_index).  The static layout cuts the groups into `world`
// contiguous blocks balanced by bins,
//   owner(group g) = min(world - 1, mid(g) * world / total_bins), monotone in g;
// data-parallel training with feature_fraction < 1 re-assigns the tree's used groups every
// tree, greedily to the rank with the fewest bins so far (OwnershipForTree), inside the
// capacities the static layout sized the buffers and graphs for.
GPUTreeLearner::OwnerLayout GPUTreeLearner::BuildOwnerLayout(const std::vector<int>& gown) const {
  OwnerLayout L;
  std::vector<int> load(world_, 0), gpos(num_groups_, -1);
  for (int g = 0; g < num_groups_; ++g) {
    if (gown[g] < 0) continue;
    gpos[g] = load[gown[g]];
    load[gown[g]] += group_off_[g + 1] - group_off_[g];
  }
  L.max_block = *std::max_element(load.begin(), load.end());
  std::vector<int> count(world_, 0), local(num_features_, -1);
  for (int f = 0; f < num_features_; ++f) {
    const int o = gown[data_->Feature2Group(f)];
    if (o < 0) continue;
    local[f] = count[o]++;
    if (o == rank_) L.feats.push_back(f);
  }
  L.max_feats = *std::max_element(count.begin(), count.end());
  L.fb_index.assign(std::max(1, num_features_), 0);
  L.owned_off.assign(std::max(1, num_features_), 0);
  for (int f = 0; f < num_features_; ++f) {
    const int g = data_->Feature2Group(f), o = gown[g];
    if (o < 0) continue;  // (never read: the feature is not scanned this tree)
    L.fb_index[f] = o * 2 * max_owned_ + local[f];
    L.owned_off[f] = gpos[g] + (feat_hist_off_[f] - group_off_[g]);
  }
  L.rs_pos.assign(std::max(1, total_bins_), -1);
  for (int g = 0; g < num_groups_; ++g) {
    if (gown[g] < 0) continue;
    for (int b = group_off_[g]; b < group_off_[g + 1]; ++b) L.rs_pos[b] = gown[g] * rs_block_ + gpos[g] + (b - group_off_[g]);
  }
  for (int f : L.feats) {
    if (data_->FeatureBinMapper(f)->bin_type() == BinType::Categorical) L.cats.push_back(f);
  }
  return L;
}

void GPUTreeLearner::UploadOwnerLayout(const OwnerLayout& L) {
  std::vector<int32_t> fl(std::max(1, max_owned_), -1), cl(std::max(1, cat_cap_), -1);
  std::copy(L.feats.begin(), L.feats.end(), fl.begin());
  std::copy(L.cats.begin(), L.cats.end(), cl.begin());
  HIPCHECK(hipMemcpyAsync(d_feat_list_, fl.data(), sizeof(int32_t) * fl.size(), hipMemcpyHostToDevice, stream_));
  HIPCHECK(hipMemcpyAsync(d_owned_cats_, cl.data(), sizeof(int32_t) * cl.size(), hipMemcpyHostToDevice, stream_));
  HIPCHECK(hipMemcpyAsync(d_fb_index_, L.fb_index.data(), sizeof(int32_t) * L.fb_index.size(), hipMemcpyHostToDevice,
                          stream_));
  HIPCHECK(hipMemcpyAsync(d_owned_off_, L.owned_off.data(), sizeof(int32_t) * L.owned_off.size(),
                          hipMemcpyHostToDevice, stream_));
  HIPCHECK(hipMemcpyAsync(d_rs_pos_, L.rs_pos.data(), sizeof(int32_t) * L.rs_pos.size(), hipMemcpyHostToDevice,
                          stream_));
  HIPCHECK(hipStreamSynchronize(stream_));  // (the host vectors are temporaries)
}

void GPUTreeLearner::SetupOwnership() {
  owned_feats_.clear();
  max_owned_ = 0;
  rs_block_ = 0;
  owned_bin_lo_ = 0;
  dyn_owner_ = false;
  if (!distributed_ || mode_ == Mode::kVoting) return;
  group_off_.assign(num_groups_ + 1, total_bins_);
  for (int g = 0; g < num_groups_; ++g) group_off_[g] = static_cast<int32_t>(data_->group_bin_boundary(g));
  feat_hist_off_.assign(std::max(1, num_features_), 0);
  for (int f = 0; f < num_features_; ++f) feat_hist_off_[f] = static_cast<int32_t>(data_->FeatureHistOffset(f));
  std::vector<int> gown(num_groups_);
  std::vector<int> lo(world_, -1), hi(world_, -1);
  int max_group_bins = 1, max_group_feats = 1;
  std::vector<int> gfeats(num_groups_, 0);
  for (int f = 0; f < num_features_; ++f) max_group_feats = std::max(max_group_feats, ++gfeats[data_->Feature2Group(f)]);
  for (int g = 0; g < num_groups_; ++g) {
    const long long mid2 = static_cast<long long>(group_off_[g]) + group_off_[g + 1];
    gown[g] = static_cast<int>(std::min<long long>(world_ - 1, mid2 * world_ / (2LL * std::max(1, total_bins_))));
    const int r = gown[g];
    if (lo[r] < 0) lo[r] = group_off_[g];
    hi[r] = group_off_[g + 1];
    max_group_bins = std::max(max_group_bins, group_off_[g + 1] - group_off_[g]);
  }
  int prev_end = 0;
  for (int r = 0; r < world_; ++r) {
    if (lo[r] < 0) lo[r] = hi[r] = prev_end;  // a rank without groups: empty block
    prev_end = hi[r];
    rs_block_ = std::max(rs_block_, hi[r] - lo[r]);
  }
  owned_bin_lo_ = lo[rank_];
  std::vector<int> count(world_, 0);
  for (int f = 0; f < num_features_; ++f) count[gown[data_->Feature2Group(f)]]++;
  for (int r = 0; r < world_; ++r) max_owned_ = std::max(max_owned_, count[r]);
  // per-tree ownership: blocks of the greedy assignment fit avg + one group (bins); the feature
  // capacity leaves room for an uneven count -- a tree whose assignment exceeds either keeps
  // the static layout
  dyn_owner_ = mode_ == Mode::kData && config_->feature_fraction < 1.0 &&
               !(tuning::Get(tuning::Knob::StaticOwners) != nullptr && tuning::Get(tuning::Knob::StaticOwners)[0] == '1');
  int ncat = 0;
  for (int f = 0; f < num_features_; ++f) ncat += data_->FeatureBinMapper(f)->bin_type() == BinType::Categorical ? 1 : 0;
  if (dyn_owner_) {
    rs_block_ = std::max(rs_block_, (total_bins_ + world_ - 1) / world_ + max_group_bins);
    max_owned_ = std::min(num_features_, std::max(max_owned_, (3 * num_features_ + 2 * world_ - 1) / (2 * world_) +
                                                                    max_group_feats));
  }
  rs_block_ = std::max(rs_block_, 1);
  max_owned_ = std::max(max_owned_, 1);
  static_layout_ = BuildOwnerLayout(gown);
  owned_feats_ = static_layout_.feats;
  cat_cap_ = dyn_owner_ ? std::max(1, ncat) : std::max<int>(1, static_layout_.cats.size());
  d_feat_list_ = Alloc<int32_t>(std::max(1, max_owned_));
  d_fb_index_ = Alloc<int32_t>(std::max(1, num_features_));
  d_rs_pos_ = Alloc<int32_t>(std::max(1, total_bins_));
  d_owned_cats_ = Alloc<int32_t>(cat_cap_);
  d_owned_off_ = Alloc<int32_t>(std::max(1, num_features_));
  UploadOwnerLayout(static_layout_);
  owner_layout_static_ = true;
  d_owned_hist_ = Alloc<long long>(2 * static_cast<size_t>(rs_block_));
  const size_t fb_bytes = 2 * static_cast<size_t>(max_owned_) *
                          (sizeof(dev::FeatureBest) + (num_cat_total_ > 0 ? kMaxCatWords * sizeof(uint32_t) : 0));
  const double rs_bytes = mode_ == Mode::kData ? sizeof(long long) * 2.0 * rs_block_ * world_ : 0.0;
  split_collective_bytes_ = rs_bytes + static_cast<double>(fb_bytes) * world_;
  root_collective_bytes_ = split_collective_bytes_ + 3 * sizeof(double) + 3 * sizeof(uint32_t);
  if (mode_ == Mode::kData) {
    Log::Info("data-parallel device learner, rank %d of %d: %d features, histogram bins [%d, %d)%s; per split "
              "reduce-scatter %zu bytes in / %zu out, split-record allgather %zu bytes per rank",
              rank_, world_, static_cast<int>(owned_feats_.size()), lo[rank_], hi[rank_],
              dyn_owner_ ? " (re-assigned per tree over the used features)" : "",
              sizeof(long long) * 2 * static_cast<size_t>(rs_block_) * world_,
              sizeof(long long) * 2 * static_cast<size_t>(rs_block_), fb_bytes);
  } else {
    Log::Info("feature-parallel device learner, rank %d of %d: %d features, histogram bins [%d, %d); per split "
              "split-record allgather %zu bytes per rank", rank_, world_, static_cast<int>(owned_feats_.size()),
              lo[rank_], hi[rank_], fb_bytes);
  }
}

// the tree's used groups to the rank with the fewest bins so far, in group order (every rank
// computes the same assignment from the same bytree sample)
void GPUTreeLearner::OwnershipForTree() {
  if (!dyn_owner_) return;
  std::vector<int> gown(num_groups_, -1), load(world_, 0);
  std::vector<char> used(num_groups_, 0);
  for (int f = 0; f < num_features_; ++f) {
    if (h_mask_[f]) used[data_->Feature2Group(f)] = 1;
  }
  for (int g = 0; g < num_groups_; ++g) {
    if (!used[g]) continue;
    const int r = static_cast<int>(std::min_element(load.begin(), load.end()) - load.begin());
    gown[g] = r;
    load[r] += group_off_[g + 1] - group_off_[g];
  }
  OwnerLayout L = BuildOwnerLayout(gown);
  int ncats_max = 0;
  {
    std::vector<int> cc(world_, 0);
    for (int f = 0; f < num_features_; ++f) {
      const int o = gown[data_->Feature2Group(f)];
      if (o >= 0 && data_->FeatureBinMapper(f)->bin_type() == BinType::Categorical) ncats_max = std::max(ncats_max, ++cc[o]);
    }
  }
  const bool fits = L.max_block <= rs_block_ && L.max_feats <= max_owned_ && ncats_max <= cat_cap_;
  if (!fits) {
    if (!owner_layout_static_) UploadOwnerLayout(static_layout_);
    owner_layout_static_ = true;
    owned_feats_ = static_layout_.feats;
    Log::Debug("per-tree ownership exceeds the layout's capacity (block %d / %d bins, %d / %d features): static owners",
               L.max_block, rs_block_, L.max_feats, max_owned_);
    return;
  }
  UploadOwnerLayout(L);
  owner_layout_static_ = false;
  owned_feats_ = L.feats;
  Log::Debug("rank %d owns %zu of the tree's features (%d bins, largest block %d)", rank_, L.feats.size(),
             load[rank_], L.max_block);
}

void GPUTreeLearner::AllreduceRoot() {
  if (!(data_parallel_ || voting_) || Network::num_machines() <= 1) return;
  // voting: the local scan of the root needs this rank's sums too
  if (voting_) HIPCHECK(hipMemcpyAsync(d_root_local_, d_root_, sizeof(double) * 3, hipMemcpyDeviceToDevice, stream_));
  DeviceComm* dc = Network::device_comm();
  if (dc != nullptr) {
    dc->AllreduceSumF64(d_root_, 3, stream_);
    return;
  }
  HIPCHECK(hipMemcpyAsync(h_root_, d_root_, sizeof(double) * 3, hipMemcpyDeviceToHost, stream_));
  HIPCHECK(hipStreamSynchronize(stream_));
  auto v = Network::GlobalSum(std::vector<double>(h_root_, h_root_ + 3));
  std::copy(v.begin(), v.end(), h_root_);
  HIPCHECK(hipMemcpyAsync(d_root_, h_root_, sizeof(double) * 3, hipMemcpyHostToDevice, stream_));
}

// data-parallel: this rank's owner block of the step's histogram, summed over every rank
// (reference data_parallel_tree_learner.cpp:154-173 ReduceScatter into feature owners)
void GPUTreeLearner::ReduceScatterStep(int parity) {
  if (!data_parallel_) return;
  DeviceComm* dc = Network::device_comm();
  long long* send = d_scratch_ + static_cast<size_t>(parity & 1) * args_.scratch_stride;
  const size_t block = 2 * static_cast<size_t>(rs_block_);
  if (dc != nullptr) {
    dc->ReduceScatterSumI64(send, d_owned_hist_, block, stream_);  // exact: fixed-point integers
    return;
  }
  // host collectives: the whole padded buffer, summed on the host
  std::vector<long long> h(block * world_);
  HIPCHECK(hipMemcpyAsync(h.data(), send, sizeof(long long) * h.size(), hipMemcpyDeviceToHost, stream_));
  HIPCHECK(hipStreamSynchronize(stream_));
  auto v = Network::GlobalSum(h);
  HIPCHECK(hipMemcpyAsync(d_owned_hist_, v.data() + block * rank_, sizeof(long long) * block, hipMemcpyHostToDevice,
                          stream_));
  HIPCHECK(hipStreamSynchronize(stream_));
}

// distributed: every rank's per-feature results (and category sets), rank-major, so each
// rank picks the same split (reference SyncUpGlobalBestSplit, parallel_tree_learner.h:190)
void GPUTreeLearner::GatherFeatureBests() {
  if (!distributed_ || voting_) return;
  DeviceComm* dc = Network::device_comm();
  const size_t fb_bytes = 2 * static_cast<size_t>(max_owned_) * sizeof(dev::FeatureBest);
  const size_t cat_bytes = 2 * static_cast<size_t>(max_owned_) * kMaxCatWords * sizeof(uint32_t);
  char* fb = reinterpret_cast<char*>(d_feat_best_);
  char* fc = reinterpret_cast<char*>(d_feat_cat_);
  // feature-parallel forced splits: the owners' records of every forced node (KArgs::forced_all)
  const dev::KArgs& fa = args_;
  const size_t ff_bytes = fa.forced_world > 1 ? sizeof(dev::FeatureBest) * fa.forced_n : 0;
  const size_t fcat_bytes = fa.forced_world > 1 ? sizeof(uint32_t) * kMaxCatWords * fa.forced_n : 0;
  char* ff = reinterpret_cast<char*>(d_forced_best_);
  char* ffc = reinterpret_cast<char*>(d_forced_cat_);
  if (dc != nullptr) {
    dc->Allgather(fb + fb_bytes * rank_, fb, fb_bytes, stream_);
    if (num_cat_total_ > 0) dc->Allgather(fc + cat_bytes * rank_, fc, cat_bytes, stream_);
    if (ff_bytes > 0) {
      dc->Allgather(ff + ff_bytes * rank_, ff, ff_bytes, stream_);
      if (num_cat_total_ > 0) dc->Allgather(ffc + fcat_bytes * rank_, ffc, fcat_bytes, stream_);
    }
    return;
  }
  auto host_gather = [&](char* d, size_t bytes) {
    std::vector<char> all(bytes * world_);
    HIPCHECK(hipMemcpyAsync(all.data() + bytes * rank_, d + bytes * rank_, bytes, hipMemcpyDeviceToHost, stream_));
    HIPCHECK(hipStreamSynchronize(stream_));
    std::vector<char> mine(all.begin() + bytes * rank_, all.begin() + bytes * (rank_ + 1));
    Network::Allgather(mine.data(), static_cast<comm_size_t>(bytes), all.data());
    HIPCHECK(hipMemcpyAsync(d, all.data(), all.size(), hipMemcpyHostToDevice, stream_));
    HIPCHECK(hipStreamSynchronize(stream_));
  };
  host_gather(fb, fb_bytes);
  if (num_cat_total_ > 0) host_gather(fc, cat_bytes);
  if (ff_bytes > 0) {
    host_gather(ff, ff_bytes);
    if (num_cat_total_ > 0) host_gather(ffc, fcat_bytes);
  }
}

void GPUTreeLearner::AllreduceAbsMax() {
  if (!(data_parallel_ || voting_) || Network::num_machines() <= 1) return;
  DeviceComm* dc = Network::device_comm();
  if (dc != nullptr) {
    dc->AllreduceMaxU32(d_absmax_, 4, stream_);  // non-negative float bits order like the floats; [3]: a flag
    return;
  }
  HIPCHECK(hipMemcpyAsync(h_absmax_, d_absmax_, sizeof(uint32_t) * 4, hipMemcpyDeviceToHost, stream_));
  HIPCHECK(hipStreamSynchronize(stream_));
  for (int k = 0; k < 4; ++k) h_absmax_[k] = Network::GlobalSyncUpByMax(h_absmax_[k]);
  HIPCHECK(hipMemcpyAsync(d_absmax_, h_absmax_, sizeof(uint32_t) * 4, hipMemcpyHostToDevice, stream_));
}

dev::KArgs GPUTreeLearner::VoteGlobalArgs(const dev::KArgs& a, int pick_in_find) const {
  dev::KArgs glob = a;
  glob.p.vote_phase = 2;
  glob.p.sp = params_;
  glob.pick_in_find = pick_in_find;
  glob.num_scan = vote_k_;
  return glob;
}

// voting: proposals -> allgather -> election + elected local histograms -> all-reduce
// (reference voting_parallel_tree_learner.cpp:300-343); the global scan follows
void GPUTreeLearner::VoteExchange(const dev::KArgs& glob, bool root) {
  dev::VoteLocal(glob, stream_, root);
  DeviceComm* dc = Network::device_comm();
  const size_t prop_bytes = sizeof(dev::VoteEntry) * 2 * static_cast<size_t>(vote_k_);
  char* vb = reinterpret_cast<char*>(d_vote_buf_);
  if (dc != nullptr) {
    dc->Allgather(vb + prop_bytes * rank_, vb, prop_bytes, stream_);
  } else {
    std::vector<char> all(prop_bytes * world_);
    HIPCHECK(hipMemcpyAsync(all.data() + prop_bytes * rank_, vb + prop_bytes * rank_, prop_bytes,
                            hipMemcpyDeviceToHost, stream_));
    HIPCHECK(hipStreamSynchronize(stream_));
    std::vector<char> mine(all.begin() + prop_bytes * rank_, all.begin() + prop_bytes * (rank_ + 1));
    Network::Allgather(mine.data(), static_cast<comm_size_t>(prop_bytes), all.data());
    HIPCHECK(hipMemcpyAsync(vb, all.data(), all.size(), hipMemcpyHostToDevice, stream_));
  }
  dev::VoteElect(glob, stream_, root);
  const size_t n = static_cast<size_t>(2 * vote_k_) * 2 * glob.p.max_feature_bins;
  if (dc != nullptr) {
    dc->AllreduceSumI64(d_vote_hist_, n, stream_);  // exact: fixed-point integers
  } else {
    std::vector<long long> h(n);
    HIPCHECK(hipMemcpyAsync(h.data(), d_vote_hist_, sizeof(long long) * n, hipMemcpyDeviceToHost, stream_));
    HIPCHECK(hipStreamSynchronize(stream_));
    h = Network::GlobalSum(h);
    HIPCHECK(hipMemcpyAsync(d_vote_hist_, h.data(), sizeof(long long) * n, hipMemcpyHostToDevice, stream_));
    HIPCHECK(hipStreamSynchronize(stream_));
  }
}

}  // namespace lgbm_amd
