// CPU distributed learners (see parallel_tree_learner.h).
// feature-parallel: reference src/treelearner/feature_parallel_tree_learner.cpp:23-75
// data-parallel:    reference src/treelearner/data_parallel_tree_learner.cpp:22-255
// voting-parallel:  reference src/treelearner/voting_parallel_tree_learner.cpp:15-452
#include "parallel_tree_learner.h"

#include <type_traits>

#include <omp.h>

#include <algorithm>
#include <cstring>

#include "lgbm_amd/log.h"
#include "lgbm_amd/network.h"
#include "gpu_tree_learner.h"

namespace lgbm_amd {

namespace {

struct WireHeader {
  int32_t feature, inner_feature;
  uint32_t threshold;
  int32_t left_count, right_count, num_cat;
  double left_output, right_output, gain;
  double lsg, lsh, rsg, rsh;
  int8_t default_left, monotone_type, pad[6];
};

void HistSumReducer(const char* src, char* dst, int, comm_size_t len) {
  const hist_t* s = reinterpret_cast<const hist_t*>(src);
  hist_t* d = reinterpret_cast<hist_t*>(dst);
  const comm_size_t n = len / static_cast<comm_size_t>(sizeof(hist_t));
  for (comm_size_t i = 0; i < n; ++i) d[i] += s[i];
}

// greedy bin-balanced assignment of the tree's features to ranks
std::vector<std::vector<int>> DistributeFeatures(const Dataset* data, const std::vector<int8_t>& used, int nm,
                                                 bool exclude_offset_bin) {
  std::vector<std::vector<int>> dist(nm);
  std::vector<int> bins(nm, 0);
  for (int i = 0; i < data->num_total_features(); ++i) {
    const int inner = data->InnerFeatureIndex(i);
    if (inner < 0 || !used[inner]) continue;
    const int m = static_cast<int>(std::min_element(bins.begin(), bins.end()) - bins.begin());
    dist[m].push_back(inner);
    int nb = data->FeatureBinMapper(inner)->num_bin();
    if (exclude_offset_bin && data->FeatureBinMapper(inner)->GetMostFreqBin() == 0) nb -= 1;
    bins[m] += nb;
  }
  return dist;
}

}  // namespace

size_t SplitInfoWireSize(int max_cat) { return sizeof(WireHeader) + sizeof(uint32_t) * std::max(0, max_cat); }

void SplitInfoToWire(const SplitInfo& s, int max_cat, char* out) {
  WireHeader h;
  std::memset(&h, 0, sizeof(h));
  h.feature = s.feature;
  h.inner_feature = s.inner_feature;
  h.threshold = s.threshold;
  h.left_count = s.left_count;
  h.right_count = s.right_count;
  h.num_cat = std::min(s.num_cat_threshold, max_cat);
  h.left_output = s.left_output;
  h.right_output = s.right_output;
  h.gain = s.gain;
  h.lsg = s.left_sum_gradient;
  h.lsh = s.left_sum_hessian;
  h.rsg = s.right_sum_gradient;
  h.rsh = s.right_sum_hessian;
  h.default_left = s.default_left ? 1 : 0;
  h.monotone_type = s.monotone_type;
  std::memcpy(out, &h, sizeof(h));
  std::memset(out + sizeof(h), 0, sizeof(uint32_t) * std::max(0, max_cat));
  if (h.num_cat > 0) std::memcpy(out + sizeof(h), s.cat_threshold.data(), sizeof(uint32_t) * h.num_cat);
}

void SplitInfoFromWire(const char* in, SplitInfo* s) {
  WireHeader h;
  std::memcpy(&h, in, sizeof(h));
  s->feature = h.feature;
  s->inner_feature = h.inner_feature;
  s->threshold = h.threshold;
  s->left_count = h.left_count;
  s->right_count = h.right_count;
  s->num_cat_threshold = h.num_cat;
  s->left_output = h.left_output;
  s->right_output = h.right_output;
  s->gain = h.gain;
  s->left_sum_gradient = h.lsg;
  s->left_sum_hessian = h.lsh;
  s->right_sum_gradient = h.rsg;
  s->right_sum_hessian = h.rsh;
  s->default_left = h.default_left != 0;
  s->monotone_type = h.monotone_type;
  s->cat_threshold.resize(h.num_cat);
  if (h.num_cat > 0) std::memcpy(s->cat_threshold.data(), in + sizeof(h), sizeof(uint32_t) * h.num_cat);
}

void SyncUpGlobalBestSplit(SplitInfo* smaller, SplitInfo* larger, int max_cat) {
  if (Network::num_machines() <= 1) return;
  const size_t sz = SplitInfoWireSize(max_cat);
  std::vector<char> in(2 * sz), out(2 * sz);
  SplitInfoToWire(*smaller, max_cat, in.data());
  SplitInfoToWire(*larger, max_cat, in.data() + sz);
  Network::Allreduce(in.data(), static_cast<comm_size_t>(2 * sz), static_cast<int>(sz), out.data(),
                     [](const char* src, char* dst, int ts, comm_size_t len) {
                       for (comm_size_t used = 0; used < len; used += ts) {
                         WireHeader a, b;
                         std::memcpy(&a, src + used, sizeof(a));
                         std::memcpy(&b, dst + used, sizeof(b));
                         LightSplitInfo la, lb;
                         la.feature = a.feature;
                         la.gain = a.gain;
                         lb.feature = b.feature;
                         lb.gain = b.gain;
                         if (la > lb) std::memcpy(dst + used, src + used, ts);
                       }
                     });
  SplitInfoFromWire(out.data(), smaller);
  SplitInfoFromWire(out.data() + sz, larger);
}

// ------------------------------------------------------------------ feature parallel
void FeatureParallelTreeLearner::Init(const Dataset* train_data, bool is_constant_hessian) {
  SerialTreeLearner::Init(train_data, is_constant_hessian);
  rank_ = Network::rank();
  num_machines_ = Network::num_machines();
}

void FeatureParallelTreeLearner::BeforeTrain() {
  SerialTreeLearner::BeforeTrain();
  auto dist = DistributeFeatures(data_, col_sampler_.is_feature_used_bytree(), num_machines_, false);
  feature_mask_.assign(num_features_, 0);
  for (int f : dist[rank_]) feature_mask_[f] = 1;
}

void FeatureParallelTreeLearner::FindBestSplitsFromHistograms(const std::vector<int8_t>& used, bool use_subtract,
                                                              const Tree* tree) {
  SerialTreeLearner::FindBestSplitsFromHistograms(used, use_subtract, tree);
  SplitInfo sb = best_split_per_leaf_[smaller_.leaf], lb;
  if (larger_.leaf >= 0) lb = best_split_per_leaf_[larger_.leaf];
  SyncUpGlobalBestSplit(&sb, &lb, config_->max_cat_threshold);
  best_split_per_leaf_[smaller_.leaf] = sb;
  if (larger_.leaf >= 0) best_split_per_leaf_[larger_.leaf] = lb;
}

// ------------------------------------------------------------------ data parallel
void DataParallelTreeLearner::Init(const Dataset* train_data, bool is_constant_hessian) {
  SerialTreeLearner::Init(train_data, is_constant_hessian);
  rank_ = Network::rank();
  num_machines_ = Network::num_machines();
  const size_t hist_bytes = 2 * sizeof(hist_t) * data_->num_total_bin();
  const size_t split_bytes = 2 * SplitInfoWireSize(config_->max_cat_threshold);
  in_buf_.resize(std::max(hist_bytes, split_bytes));
  out_buf_.resize(std::max(hist_bytes, split_bytes));
  aggregated_.assign(num_features_, 0);
  block_start_.assign(num_machines_, 0);
  block_len_.assign(num_machines_, 0);
  write_pos_.assign(num_features_, 0);
  read_pos_.assign(num_features_, 0);
  global_count_.assign(config_->num_leaves, 0);
}

void DataParallelTreeLearner::ResetConfig(const Config* config) {
  SerialTreeLearner::ResetConfig(config);
  global_count_.assign(config_->num_leaves, 0);
}

void DataParallelTreeLearner::BeforeTrain() {
  SerialTreeLearner::BeforeTrain();
  const auto& bytree = col_sampler_.is_feature_used_bytree();
  auto dist = DistributeFeatures(data_, bytree, num_machines_, true);
  std::fill(aggregated_.begin(), aggregated_.end(), 0);
  for (int f : dist[rank_]) aggregated_[f] = 1;
  const size_t entry = 2 * sizeof(hist_t);
  size_t pos = 0;
  reduce_scatter_size_ = 0;
  for (int m = 0; m < num_machines_; ++m) {
    block_start_[m] = static_cast<comm_size_t>(pos);
    for (int f : dist[m]) {
      write_pos_[f] = pos;
      pos += entry * data_->FeatureHistSize(f);
    }
    block_len_[m] = static_cast<comm_size_t>(pos) - block_start_[m];
  }
  reduce_scatter_size_ = static_cast<comm_size_t>(pos);
  size_t rp = 0;
  for (int f : dist[rank_]) {
    read_pos_[f] = rp;
    rp += entry * data_->FeatureHistSize(f);
  }
  // global root statistics
  struct Sum {
    double n, g, h;
  } local{static_cast<double>(smaller_.num_data), smaller_.sum_g, smaller_.sum_h}, global{0, 0, 0};
  Network::Allreduce(reinterpret_cast<char*>(&local), sizeof(Sum), sizeof(Sum), reinterpret_cast<char*>(&global),
                     [](const char* src, char* dst, int, comm_size_t) {
                       Sum a, b;
                       std::memcpy(&a, src, sizeof(Sum));
                       std::memcpy(&b, dst, sizeof(Sum));
                       b.n += a.n;
                       b.g += a.g;
                       b.h += a.h;
                       std::memcpy(dst, &b, sizeof(Sum));
                     });
  smaller_.num_data = static_cast<data_size_t>(global.n);
  smaller_.sum_g = global.g;
  smaller_.sum_h = global.h;
  global_count_[0] = smaller_.num_data;
}

void DataParallelTreeLearner::FindBestSplits(const Tree* tree) {
  const auto& bytree = col_sampler_.is_feature_used_bytree();
  ConstructHistograms(bytree, true);
  const size_t entry = 2 * sizeof(hist_t);
#pragma omp parallel for schedule(static)
  for (int f = 0; f < num_features_; ++f) {
    if (!bytree[f]) continue;
    std::memcpy(in_buf_.data() + write_pos_[f], FeatureHist(smaller_slot_, f), entry * data_->FeatureHistSize(f));
  }
  Network::ReduceScatter(in_buf_.data(), reduce_scatter_size_, sizeof(hist_t), block_start_.data(), block_len_.data(),
                         out_buf_.data(), static_cast<comm_size_t>(out_buf_.size()), &HistSumReducer);
  std::vector<int8_t> used(num_features_, 0);
  for (int f = 0; f < num_features_; ++f) {
    if (!aggregated_[f]) continue;
    used[f] = 1;
    std::memcpy(FeatureHist(smaller_slot_, f), out_buf_.data() + read_pos_[f], entry * data_->FeatureHistSize(f));
  }
  SerialTreeLearner::FindBestSplitsFromHistograms(used, true, tree);
  SplitInfo sb = best_split_per_leaf_[smaller_.leaf], lb;
  if (larger_.leaf >= 0) lb = best_split_per_leaf_[larger_.leaf];
  SyncUpGlobalBestSplit(&sb, &lb, config_->max_cat_threshold);
  best_split_per_leaf_[smaller_.leaf] = sb;
  if (larger_.leaf >= 0) best_split_per_leaf_[larger_.leaf] = lb;
}

void DataParallelTreeLearner::Split(Tree* tree, int best_leaf, int* left_leaf, int* right_leaf) {
  SplitInner(tree, best_leaf, left_leaf, right_leaf, false);
  const SplitInfo& s = best_split_per_leaf_[best_leaf];
  global_count_[*left_leaf] = s.left_count;
  global_count_[*right_leaf] = s.right_count;
}

// ------------------------------------------------------------------ voting parallel
template <typename Base>
void VotingParallelTreeLearner<Base>::InitLocalParams() {
  Config local = *this->config_;
  local.min_data_in_leaf /= num_machines_;
  local.min_sum_hessian_in_leaf /= num_machines_;
  local_params_ = MakeSplitParams(local);
}

template <typename Base>
void VotingParallelTreeLearner<Base>::Init(const Dataset* train_data, bool is_constant_hessian) {
  if constexpr (std::is_base_of<DeviceTreeLearner, Base>::value) {
    // device-resident trees run the whole exchange on the device (GPUTreeLearner kVoting);
    // host-assisted ones (per-node sampling, extra_trees, forced splits, CEGB) use this class's
    // host loop between the device histogram builds
    this->UseDeviceVoting();
  }
  Base::Init(train_data, is_constant_hessian);
  rank_ = Network::rank();
  num_machines_ = Network::num_machines();
  top_k_ = std::min(this->config_->top_k, this->num_features_);
  InitLocalParams();
  global_meta_ = this->meta_;  // (freshly seeded: Random(extra_seed + feature))
  global_count_.assign(this->config_->num_leaves, 0);
  global_small_hist_.assign(2 * this->data_->num_total_bin(), 0.0);
  global_large_hist_.assign(2 * this->data_->num_total_bin(), 0.0);
  in_buf_.resize(std::max<size_t>(4 * sizeof(hist_t) * this->data_->num_total_bin(),
                                  2 * SplitInfoWireSize(this->config_->max_cat_threshold)));
  out_buf_.resize(in_buf_.size());
}

template <typename Base>
void VotingParallelTreeLearner<Base>::ResetConfig(const Config* config) {
  Base::ResetConfig(config);
  top_k_ = std::min(this->config_->top_k, this->num_features_);
  InitLocalParams();
  global_meta_ = this->meta_;  // (both generator sets reseeded, as the reference's ResetConfig)
  global_count_.assign(this->config_->num_leaves, 0);
}

template <typename Base>
void VotingParallelTreeLearner<Base>::BeforeTrain() {
  Base::BeforeTrain();
  double loc[3] = {static_cast<double>(this->smaller_.num_data), this->smaller_.sum_g, this->smaller_.sum_h};
  auto glob = Network::GlobalSum(std::vector<double>(loc, loc + 3));
  global_smaller_ = LeafState{0, static_cast<data_size_t>(glob[0]), glob[1], glob[2], 0.0};
  global_larger_ = LeafState{};
  global_count_[0] = global_smaller_.num_data;
}

template <typename Base>
bool VotingParallelTreeLearner<Base>::BeforeFindBestSplit(const Tree* tree, int left_leaf, int right_leaf) {
  if (!Base::BeforeFindBestSplit(tree, left_leaf, right_leaf)) return false;
  if (right_leaf < 0) return true;
  // leaf roles follow the global counts; statistics for local voting are local
  const int small = this->GetGlobalDataCountInLeaf(left_leaf) < this->GetGlobalDataCountInLeaf(right_leaf) ? left_leaf : right_leaf;
  const int large = small == left_leaf ? right_leaf : left_leaf;
  this->smaller_ = this->LocalLeafSums(small);
  this->larger_ = this->LocalLeafSums(large);
  this->smaller_.output = global_smaller_.output;
  this->larger_.output = global_larger_.output;
  return true;
}

template <typename Base>
void VotingParallelTreeLearner<Base>::GlobalVoting(int leaf, const std::vector<LightSplitInfo>& splits,
                                             std::vector<int>* out) const {
  out->clear();
  if (leaf < 0) return;
  const score_t mean = this->GetGlobalDataCountInLeaf(leaf) / static_cast<score_t>(num_machines_);
  std::vector<LightSplitInfo> best(this->data_->num_total_features());
  for (const auto& s : splits) {
    if (s.feature < 0) continue;
    const double g = s.gain * (s.left_count + s.right_count) / mean;
    if (g > best[s.feature].gain) {
      best[s.feature] = s;
      best[s.feature].gain = g;
    }
  }
  std::stable_sort(best.begin(), best.end(), std::greater<LightSplitInfo>());
  for (int i = 0; i < std::min<int>(top_k_, static_cast<int>(best.size())); ++i) {
    if (best[i].gain == kMinScore || best[i].feature == -1) continue;
    out->push_back(best[i].feature);
  }
}

template <typename Base>
void VotingParallelTreeLearner<Base>::FindBestSplits(const Tree* tree) {
  // 1) local histograms + local per-feature best splits (local statistics & params)
  std::vector<int8_t> used(this->num_features_, 0);
  const auto& bytree = this->col_sampler_.is_feature_used_bytree();
  for (int f = 0; f < this->num_features_; ++f) {
    if (!bytree[f]) continue;
    if (this->has_parent_hist_ && !this->splittable_[this->larger_slot_][f]) {
      this->splittable_[this->smaller_slot_][f] = 0;
      continue;
    }
    used[f] = 1;
  }
  this->ConstructHistograms(used, this->has_parent_hist_);
  this->PrepareCegbLeaves();
  std::vector<SplitInfo> sbest(this->num_features_), lbest(this->num_features_);
  const int sdepth = tree->leaf_depth(this->smaller_.leaf);
  const int ldepth = this->larger_.leaf >= 0 ? tree->leaf_depth(this->larger_.leaf) : 0;
#pragma omp parallel for schedule(static)
  for (int f = 0; f < this->num_features_; ++f) {
    if (!used[f]) continue;
    this->data_->FixHistogram(f, this->smaller_.sum_g, this->smaller_.sum_h, this->FeatureHist(this->smaller_slot_, f));
    this->splittable_[this->smaller_slot_][f] = this->EvalFeature(this->FeatureHist(this->smaller_slot_, f), f, local_params_, this->smaller_, sdepth,
                                                &sbest[f]) ? 1 : 0;
    if (this->larger_.leaf < 0) continue;
    hist_t* lh = this->FeatureHist(this->larger_slot_, f);
    if (this->has_parent_hist_) {
      const hist_t* sh = this->FeatureHist(this->smaller_slot_, f);
      const int n = 2 * this->data_->FeatureHistSize(f);
      for (int i = 0; i < n; ++i) lh[i] -= sh[i];
    } else {
      this->data_->FixHistogram(f, this->larger_.sum_g, this->larger_.sum_h, lh);
    }
    this->splittable_[this->larger_slot_][f] = this->EvalFeature(lh, f, local_params_, this->larger_, ldepth, &lbest[f]) ? 1 : 0;
  }
  // 2) local top-k, allgather, global vote
  auto topk = [&](std::vector<SplitInfo> v) {
    std::stable_sort(v.begin(), v.end(), [](const SplitInfo& a, const SplitInfo& b) { return a > b; });
    std::vector<LightSplitInfo> out(top_k_);
    for (int i = 0; i < top_k_ && i < static_cast<int>(v.size()); ++i) {
      out[i].feature = v[i].feature;
      out[i].gain = v[i].gain;
      out[i].left_count = v[i].left_count;
      out[i].right_count = v[i].right_count;
    }
    return out;
  };
  auto st = topk(sbest), lt = topk(lbest);
  std::vector<LightSplitInfo> mine;
  for (int i = 0; i < top_k_; ++i) {
    mine.push_back(st[i]);
    mine.push_back(lt[i]);
  }
  std::vector<LightSplitInfo> all(mine.size() * num_machines_);
  Network::Allgather(reinterpret_cast<char*>(mine.data()), static_cast<comm_size_t>(sizeof(LightSplitInfo) * mine.size()),
                     reinterpret_cast<char*>(all.data()));
  std::vector<LightSplitInfo> sg, lg;
  for (size_t i = 0; i < all.size(); i += 2) {
    sg.push_back(all[i]);
    lg.push_back(all[i + 1]);
  }
  std::vector<int> stop, ltop;
  GlobalVoting(this->smaller_.leaf, sg, &stop);
  GlobalVoting(this->larger_.leaf, lg, &ltop);
  // 3) reduce-scatter the elected histograms (alternating smaller/larger, even split)
  std::vector<int8_t> s_agg(this->num_features_, 0), l_agg(this->num_features_, 0);
  std::vector<size_t> s_read(this->num_features_, 0), l_read(this->num_features_, 0);
  std::vector<comm_size_t> bstart(num_machines_, 0), blen(num_machines_, 0);
  const size_t total = stop.size() + ltop.size();
  const size_t avg = (total + num_machines_ - 1) / num_machines_;
  size_t used_n = 0, si = 0, li = 0, rs = 0;
  const size_t entry = 2 * sizeof(hist_t);
  for (int m = 0; m < num_machines_; ++m) {
    size_t cur = 0, cnt = 0;
    const size_t want = std::min(avg, total - used_n);
    while (cnt < want) {
      if (si < stop.size()) {
        const int f = this->data_->InnerFeatureIndex(stop[si++]);
        ++cnt;
        const size_t bytes = entry * this->data_->FeatureHistSize(f);
        if (m == rank_) {
          s_agg[f] = 1;
          s_read[f] = cur;
        }
        std::memcpy(in_buf_.data() + rs, this->FeatureHist(this->smaller_slot_, f), bytes);
        cur += bytes;
        rs += bytes;
      }
      if (cnt >= want) break;
      if (li < ltop.size()) {
        const int f = this->data_->InnerFeatureIndex(ltop[li++]);
        ++cnt;
        const size_t bytes = entry * this->data_->FeatureHistSize(f);
        if (m == rank_) {
          l_agg[f] = 1;
          l_read[f] = cur;
        }
        std::memcpy(in_buf_.data() + rs, this->FeatureHist(this->larger_slot_, f), bytes);
        cur += bytes;
        rs += bytes;
      }
    }
    used_n += cnt;
    blen[m] = static_cast<comm_size_t>(cur);
    if (m + 1 < num_machines_) bstart[m + 1] = bstart[m] + blen[m];
  }
  Network::ReduceScatter(in_buf_.data(), static_cast<comm_size_t>(rs), sizeof(hist_t), bstart.data(), blen.data(),
                         out_buf_.data(), static_cast<comm_size_t>(out_buf_.size()), &HistSumReducer);
  // 4) best splits on the global histograms this rank owns (global statistics & params)
  auto s_node = this->col_sampler_.GetByNode(tree, global_smaller_.leaf);
  std::vector<int8_t> l_node;
  if (global_larger_.leaf >= 0) l_node = this->col_sampler_.GetByNode(tree, global_larger_.leaf);
  const int nt = omp_get_max_threads();
  std::vector<SplitInfo> sb(nt), lb(nt);
#pragma omp parallel for schedule(static)
  for (int f = 0; f < this->num_features_; ++f) {
    const int tid = omp_get_thread_num();
    const size_t off = 2 * static_cast<size_t>(this->data_->FeatureHistOffset(f));
    const size_t bytes = entry * this->data_->FeatureHistSize(f);
    if (s_agg[f] && s_node[f]) {
      hist_t* h = global_small_hist_.data() + off;
      std::memcpy(h, out_buf_.data() + s_read[f], bytes);
      this->data_->FixHistogram(f, global_smaller_.sum_g, global_smaller_.sum_h, h);
      this->EvalFeature(h, f, this->params_, global_smaller_, sdepth, &sb[tid], &global_meta_[f]);
    }
    if (l_agg[f] && global_larger_.leaf >= 0 && l_node[f]) {
      hist_t* h = global_large_hist_.data() + off;
      std::memcpy(h, out_buf_.data() + l_read[f], bytes);
      this->data_->FixHistogram(f, global_larger_.sum_g, global_larger_.sum_h, h);
      this->EvalFeature(h, f, this->params_, global_larger_, ldepth, &lb[tid], &global_meta_[f]);
    }
  }
  SplitInfo bs, bl;
  for (int t = 0; t < nt; ++t) {
    if (sb[t] > bs) bs = sb[t];
    if (lb[t] > bl) bl = lb[t];
  }
  SyncUpGlobalBestSplit(&bs, &bl, this->config_->max_cat_threshold);
  // (the reference stores this rank's bests before the sync and copies back a larger leaf's
  // synced best only when it found a split; the sync is a max over the ranks, so a larger leaf
  // without one keeps "no split" -- never its parent's stale best, which it would split again)
  this->best_split_per_leaf_[global_smaller_.leaf] = bs;
  if (global_larger_.leaf >= 0) this->best_split_per_leaf_[global_larger_.leaf] = bl;
}

template <typename Base>
void VotingParallelTreeLearner<Base>::Split(Tree* tree, int best_leaf, int* left_leaf, int* right_leaf) {
  this->SplitInner(tree, best_leaf, left_leaf, right_leaf, false);
  const SplitInfo& s = this->best_split_per_leaf_[best_leaf];
  global_count_[*left_leaf] = s.left_count;
  global_count_[*right_leaf] = s.right_count;
  // this->SplitInner set this->smaller_/this->larger_ from the (global) split statistics
  global_smaller_ = this->smaller_;
  global_larger_ = this->larger_;
}

template class VotingParallelTreeLearner<SerialTreeLearner>;
template class VotingParallelTreeLearner<GPUTreeLearner>;

}  // namespace lgbm_amd
