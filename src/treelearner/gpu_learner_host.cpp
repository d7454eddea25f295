// MI355X tree learner: host-assisted growth (the CPU learner's loop over device histograms)
// and the host mirror of the device partition.
#include "gpu_learner_internal.h"

namespace lgbm_amd {

// ---------------------------------------------------------------- host-assisted mode
void GPUTreeLearner::BeforeTrain() {
  col_sampler_.ResetByTree();
  dev::KArgs a = args_;
  if (use_bag_) {
    HIPCHECK(hipMemcpyAsync(d_idx_, d_bag_, sizeof(int32_t) * bag_cnt_, hipMemcpyDeviceToDevice, stream_));
    a.num_rows = bag_cnt_;
  } else {
    dev::Iota(d_idx_, num_data_, stream_);
    a.num_rows = num_data_;
  }
  a.root_identity = 0;
  root_rows_ = a.num_rows;
  dev::TreeBegin(a, stream_);
  dev::RootSum(a, stream_);
  HIPCHECK(hipMemcpyAsync(h_root_, d_root_, sizeof(double) * 3, hipMemcpyDeviceToHost, stream_));
  HIPCHECK(hipStreamSynchronize(stream_));
  double sg = h_root_[0], sh = h_root_[1], cnt = h_root_[2];
  if (data_parallel_ && Network::num_machines() > 1) {
    auto v = Network::GlobalSum(std::vector<double>{sg, sh, cnt});
    sg = v[0];
    sh = v[1];
    cnt = v[2];
  }
  std::fill(leaf_begin_.begin(), leaf_begin_.end(), 0);
  std::fill(leaf_count_.begin(), leaf_count_.end(), 0);
  leaf_count_[0] = a.num_rows;
  global_count_.assign(config_->num_leaves, 0);
  global_count_[0] = static_cast<data_size_t>(cnt);
  constraints_.Init(config_->num_leaves);
  for (auto& s : best_split_per_leaf_) s.Reset();
  smaller_ = LeafState{0, static_cast<data_size_t>(cnt), sg, sh, 0.0};
  larger_ = LeafState{};
  larger_.leaf = -1;
}

// host-assisted growth keeps every leaf's rows in index buffer 0 at [leaf_begin, +count)
SerialTreeLearner::LeafState GPUTreeLearner::LocalLeafSums(int leaf) const {
  LeafState ls;
  ls.leaf = leaf;
  ls.num_data = leaf_count_[leaf];
  if (ls.num_data <= 0) return ls;
  dev::KArgs a = args_;
  a.idx = d_idx_ + leaf_begin_[leaf];
  a.num_rows = ls.num_data;
  a.num_rows_dev = nullptr;
  a.root_identity = 0;
  a.root = d_leaf_sums_;
  dev::RootSum(a, stream_);
  double h[3];
  HIPCHECK(hipMemcpyAsync(h, d_leaf_sums_, sizeof(double) * 3, hipMemcpyDeviceToHost, stream_));
  HIPCHECK(hipStreamSynchronize(stream_));
  ls.sum_g = h[0];
  ls.sum_h = h[1];
  return ls;
}

data_size_t GPUTreeLearner::GetGlobalDataCountInLeaf(int leaf) const {
  if (leaf < 0) return 0;
  return data_parallel_ ? global_count_[leaf] : leaf_count_[leaf];
}

void GPUTreeLearner::BuildRangeHistogram(int leaf, int slot) {
  dev::KArgs a = args_;
  a.range_begin = leaf_begin_[leaf];
  a.num_rows = leaf_count_[leaf];
  const size_t n = 2 * static_cast<size_t>(total_bins_);
  HIPCHECK(hipMemsetAsync(d_scratch_, 0, sizeof(long long) * n, stream_));
  if (a.num_rows > 0) dev::HistRange(a, stream_);  // partials + reduction into scratch buffer 0
  std::vector<long long> h(n);
  HIPCHECK(hipMemcpyAsync(h.data(), d_scratch_, sizeof(long long) * n, hipMemcpyDeviceToHost, stream_));
  HIPCHECK(hipMemcpyAsync(h_scales_, d_scales_, sizeof(double) * 4, hipMemcpyDeviceToHost, stream_));
  HIPCHECK(hipStreamSynchronize(stream_));
  if (data_parallel_ && Network::num_machines() > 1) h = Network::GlobalSum(h);
  std::vector<hist_t>& dst = LeafHist(slot);
  const double ig = h_scales_[2], ih = h_scales_[3];
  for (size_t i = 0; i < n; i += 2) {
    dst[i] = static_cast<double>(h[i]) * ig;
    dst[i + 1] = static_cast<double>(h[i + 1]) * ih;
  }
}

void GPUTreeLearner::ConstructHistograms(const std::vector<int8_t>&, bool use_subtract) {
  common::ScopedTimer timer("GPUTreeLearner::ConstructHistograms");
  BuildRangeHistogram(smaller_.leaf, smaller_slot_);
  if (larger_slot_ >= 0 && !use_subtract) BuildRangeHistogram(larger_.leaf, larger_slot_);
}

data_size_t GPUTreeLearner::PartitionLeaf(int leaf, int inner, const SplitInfo& s, int new_leaf) {
  const data_size_t begin = leaf_begin_[leaf];
  const data_size_t cnt = leaf_count_[leaf];
  dev::Step& st = *h_step_;
  std::memset(&st, 0, sizeof(st));
  st.cs.leaf = leaf;
  st.cs.new_leaf = new_leaf;
  st.cs.part_begin = begin;
  st.cs.part_count = cnt;
  st.cs.src_buf = 0;  // host mode keeps every leaf in buffer 0 (copied back below)
  SplitInfo si = s;
  si.inner_feature = inner;
  si.ToDevice(&st.cs.split, data_->FeatureBinMapper(inner)->bin_type() == BinType::Categorical);
  st.cs.feat = h_feats_[inner];
  HIPCHECK(hipMemcpyAsync(d_step_, h_step_, sizeof(dev::Step), hipMemcpyHostToDevice, stream_));
  dev::KArgs a = args_;
  a.host_mode = 1;
  dev::Partition(a, stream_);
  if (cnt > 0) {
    HIPCHECK(hipMemcpyAsync(d_idx_ + begin, d_tmp_ + begin, sizeof(int32_t) * cnt, hipMemcpyDeviceToDevice, stream_));
  }
  HIPCHECK(hipMemcpyAsync(h_step_, d_step_, sizeof(dev::Step), hipMemcpyDeviceToHost, stream_));
  HIPCHECK(hipStreamSynchronize(stream_));
  const data_size_t left = h_step_->cur_left;
  host_partition_fresh_ = false;
  leaf_count_[leaf] = left;
  leaf_begin_[new_leaf] = begin + left;
  leaf_count_[new_leaf] = cnt - left;
  return left;
}

void GPUTreeLearner::Split(Tree* tree, int best_leaf, int* left_leaf, int* right_leaf) {
  if (!data_parallel_) {
    SplitInner(tree, best_leaf, left_leaf, right_leaf, true);
    return;
  }
  SplitInner(tree, best_leaf, left_leaf, right_leaf, false);
  const SplitInfo& s = best_split_per_leaf_[best_leaf];
  global_count_[*left_leaf] = s.left_count;
  global_count_[*right_leaf] = s.right_count;
}

// ---------------------------------------------------------------- partition mirror
void GPUTreeLearner::DownloadPartitionToHost() const {
  if (host_partition_fresh_) return;
  auto* self = const_cast<GPUTreeLearner*>(this);
  const int L = config_->num_leaves;
  if (!device_mode_) {
    // host-assisted growth keeps the partition in buffer 0 and its ranges on the host
    HIPCHECK(hipMemcpyAsync(self->indices_.data(), d_idx_, sizeof(int32_t) * root_rows_, hipMemcpyDeviceToHost,
                            stream_));
    HIPCHECK(hipStreamSynchronize(stream_));
    host_partition_fresh_ = true;
    return;
  }
  std::vector<dev::Leaf> leaves(L);
  HIPCHECK(hipMemcpyAsync(leaves.data(), d_leaves_, sizeof(dev::Leaf) * L, hipMemcpyDeviceToHost, stream_));
  HIPCHECK(hipStreamSynchronize(stream_));
  // each leaf's rows sit in the index buffer its last split wrote (Leaf::buf)
  const int num_leaves_now = last_stats_.splits + 1;  // (either growth mode)
  for (int l = 0; l < L; ++l) {
    self->leaf_begin_[l] = leaves[l].begin;
    self->leaf_count_[l] = l < num_leaves_now ? leaves[l].count : 0;
    if (self->leaf_count_[l] <= 0) continue;
    const int32_t* srcbuf = leaves[l].buf == 0 ? d_idx_ : d_tmp_ + static_cast<int64_t>(leaves[l].buf - 1) * num_data_;
    HIPCHECK(hipMemcpyAsync(self->indices_.data() + leaves[l].begin, srcbuf + leaves[l].begin,
                            sizeof(int32_t) * leaves[l].count, hipMemcpyDeviceToHost, stream_));
  }
  HIPCHECK(hipStreamSynchronize(stream_));
  host_partition_fresh_ = true;
}

void GPUTreeLearner::AddPredictionToScore(const Tree* tree, double* out_score) const {
  DownloadPartitionToHost();
  SerialTreeLearner::AddPredictionToScore(tree, out_score);
}

void GPUTreeLearner::RenewTreeOutput(Tree* tree, const ObjectiveFunction* obj,
                                     const std::function<double(const label_t*, int)>& residual,
                                     data_size_t total_num_data, const data_size_t* bag_indices,
                                     data_size_t bag_cnt) const {
  if (obj == nullptr || !obj->IsRenewTreeOutput()) return;
  if (spec_live_) Log::Fatal("device learner: leaf renewal after the next tree was launched (speculation not allowed)");
  DownloadPartitionToHost();
  SerialTreeLearner::RenewTreeOutput(tree, obj, residual, total_num_data, bag_indices, bag_cnt);
}

}  // namespace lgbm_amd
