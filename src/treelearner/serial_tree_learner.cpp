// CPU serial tree learner (see serial_tree_learner.h).
#include "serial_tree_learner.h"

#include <omp.h>

#include <algorithm>
#include <cmath>
#include <queue>
#include <unordered_map>

#include "lgbm_amd/common.h"
#include "lgbm_amd/log.h"
#include "lgbm_amd/network.h"

namespace lgbm_amd {

double MonotoneSplitPenalty(int depth, double penalization) {
  if (penalization >= depth + 1.) return kEpsilon;
  if (penalization <= 1.) return 1. - penalization / std::pow(2., depth) + kEpsilon;
  return 1. - std::pow(2, penalization - 1. - depth) + kEpsilon;
}

SerialTreeLearner::SerialTreeLearner(const Config* config) : config_(config), col_sampler_(config) {}

void SerialTreeLearner::InitFeatureMeta() {
  meta_.resize(num_features_);
  for (int i = 0; i < num_features_; ++i) {
    const BinMapper* m = data_->FeatureBinMapper(i);
    FeatureMeta& fm = meta_[i];
    fm.num_bin = m->num_bin();
    fm.default_bin = m->GetDefaultBin();
    fm.missing_type = m->missing_type();
    fm.offset = m->GetMostFreqBin() == 0 ? 1 : 0;
    fm.bin_type = m->bin_type();
    const int real = data_->RealFeatureIndex(i);
    fm.monotone_type = config_->monotone_constraints.empty() ? 0 : config_->monotone_constraints[real];
    fm.penalty = config_->feature_contri.empty() ? 1.0 : config_->feature_contri[real];
    fm.rand = Random(config_->extra_seed + i);
  }
  params_ = MakeSplitParams(*config_);
}

void SerialTreeLearner::Init(const Dataset* train_data, bool /*is_constant_hessian*/) {
  data_ = train_data;
  num_data_ = data_->num_data();
  num_features_ = data_->num_features();
  InitFeatureMeta();
  col_sampler_.SetTrainingData(data_);
  best_split_per_leaf_.assign(config_->num_leaves, SplitInfo());
  constraints_.Init(config_->num_leaves, config_);
  ResetPool();
  splittable_.assign(config_->num_leaves, std::vector<char>(num_features_, 1));
  SetHistMode(config_->force_row_wise ? 2 : config_->force_col_wise ? 1 : 0);
  indices_.resize(num_data_);
  leaf_begin_.assign(config_->num_leaves, 0);
  leaf_count_.assign(config_->num_leaves, 0);
  tmp_left_.resize(num_data_);
  tmp_right_.resize(num_data_);
  SetupCegb();
  Log::Info("Number of data points in the train set: %d, number of used features: %d", num_data_, num_features_);
}

void SerialTreeLearner::SetHistMode(int m) {
  if (m == 2 && !holds_row_major_) data_->RetainRowMajor();
  if (m != 2 && holds_row_major_) data_->ReleaseRowMajor();
  holds_row_major_ = m == 2;
  hist_mode_ = m;
}

void SerialTreeLearner::ResetTrainingData(const Dataset* train_data, bool) {
  const int mode = hist_mode_;
  SetHistMode(0);  // (the hold moves to the new Dataset)
  data_ = train_data;
  SetHistMode(mode);
  num_data_ = data_->num_data();
  LGBM_CHECK_EQ(num_features_, data_->num_features());
  indices_.resize(num_data_);
  tmp_left_.resize(num_data_);
  tmp_right_.resize(num_data_);
  col_sampler_.SetTrainingData(data_);
  use_bag_ = false;
  SetupCegb();
}

void SerialTreeLearner::SetupCegb() {
  if (!CostEffectiveGB::Enabled(*config_)) return;
  if (!cegb_) cegb_.reset(new CostEffectiveGB());
  cegb_->Init(config_, data_);
}

void SerialTreeLearner::PrepareCegbLeaves() {
  if (!cegb_ || config_->cegb_penalty_feature_lazy.empty()) return;
  for (int leaf : {smaller_.leaf, larger_.leaf}) {
    if (leaf < 0) continue;
    data_size_t cnt = 0;
    const data_size_t* rows = HostLeafRows(leaf, &cnt);
    cegb_->PrepareLeaf(leaf, rows, cnt);
  }
}

void SerialTreeLearner::ResetConfig(const Config* config) {
  const bool leaves_changed = config_->num_leaves != config->num_leaves;
  config_ = config;
  if (leaves_changed) {
    best_split_per_leaf_.assign(config_->num_leaves, SplitInfo());
    splittable_.assign(config_->num_leaves, std::vector<char>(num_features_, 1));
    leaf_begin_.assign(config_->num_leaves, 0);
    leaf_count_.assign(config_->num_leaves, 0);
  }
  ResetPool();
  if (config_->force_row_wise) SetHistMode(2);
  else if (config_->force_col_wise) SetHistMode(1);
  col_sampler_.SetConfig(config_);
  constraints_.Init(config_->num_leaves, config_);
  InitFeatureMeta();
  SetupCegb();
}

void SerialTreeLearner::ResetPool() {
  const size_t total_bins = data_->num_total_bin();
  int slots = config_->num_leaves;
  if (config_->histogram_pool_size > 0) {  // (reference SerialTreeLearner::Init's cache size)
    const double bytes = sizeof(hist_t) * 2.0 * static_cast<double>(total_bins);
    slots = static_cast<int>(config_->histogram_pool_size * 1024 * 1024 / bytes);
  }
  slots = std::min(config_->num_leaves, std::max(2, slots));
  if (static_cast<int>(hist_pool_.size()) != slots) {
    hist_pool_.assign(slots, std::vector<hist_t>(2 * total_bins, 0.0));
    if (slots < config_->num_leaves) {
      Log::Info("Histogram pool: %d of %d leaves' histograms cached (histogram_pool_size=%g MB)", slots,
                config_->num_leaves, config_->histogram_pool_size);
    }
  }
  leaf_slot_.assign(config_->num_leaves, -1);
  slot_leaf_.assign(slots, -1);
  slot_stamp_.assign(slots, 0);
  pool_clock_ = 0;
}

void SerialTreeLearner::PoolTouch(int leaf) {
  if (leaf_slot_[leaf] >= 0) slot_stamp_[leaf_slot_[leaf]] = ++pool_clock_;
}

void SerialTreeLearner::PoolAssign(int leaf, int keep_leaf) {
  if (leaf_slot_[leaf] >= 0) {
    PoolTouch(leaf);
    return;
  }
  int best = -1;
  for (int k = 0; k < static_cast<int>(slot_leaf_.size()); ++k) {
    if (slot_leaf_[k] < 0) {
      best = k;
      break;
    }
    if (slot_leaf_[k] == keep_leaf) continue;
    if (best < 0 || slot_stamp_[k] < slot_stamp_[best]) best = k;
  }
  if (slot_leaf_[best] >= 0) leaf_slot_[slot_leaf_[best]] = -1;  // evict the least recently used
  slot_leaf_[best] = leaf;
  leaf_slot_[leaf] = best;
  slot_stamp_[best] = ++pool_clock_;
}

void SerialTreeLearner::PoolMove(int from_leaf, int to_leaf) {
  const int k = leaf_slot_[from_leaf];
  if (leaf_slot_[to_leaf] >= 0) slot_leaf_[leaf_slot_[to_leaf]] = -1;
  leaf_slot_[to_leaf] = k;
  leaf_slot_[from_leaf] = -1;
  if (k >= 0) {
    slot_leaf_[k] = to_leaf;
    slot_stamp_[k] = ++pool_clock_;
  }
}

void SerialTreeLearner::SetForcedSplit(const std::string& json_text) {
  has_forced_split_ = false;
  forced_split_text_ = json_text;
  if (json_text.empty()) return;
  forced_split_ = Json::Parse(json_text);
  has_forced_split_ = forced_split_.is_object() && forced_split_.has("feature");
}

void SerialTreeLearner::SetBaggingData(const Dataset*, const data_size_t* used_indices, data_size_t n) {
  bag_indices_ = used_indices;
  bag_cnt_ = n;
  use_bag_ = used_indices != nullptr && n < num_data_;
}

void SerialTreeLearner::BeforeTrain() {
  col_sampler_.ResetByTree();
  ResetPool();  // every leaf's slot is free at the root
  // partition: every used row in leaf 0
  std::fill(leaf_begin_.begin(), leaf_begin_.end(), 0);
  std::fill(leaf_count_.begin(), leaf_count_.end(), 0);
  data_size_t n = num_data_;
  if (use_bag_) {
    n = bag_cnt_;
    std::copy(bag_indices_, bag_indices_ + n, indices_.begin());
  } else {
#pragma omp parallel for schedule(static)
    for (data_size_t i = 0; i < n; ++i) indices_[i] = i;
  }
  leaf_count_[0] = n;
  constraints_.Init(config_->num_leaves, config_);
  for (auto& s : best_split_per_leaf_) s.Reset();
  double sg = 0, sh = 0;
  if (use_bag_) {
#pragma omp parallel for schedule(static) reduction(+ : sg, sh)
    for (data_size_t i = 0; i < n; ++i) {
      sg += gradients_[indices_[i]];
      sh += hessians_[indices_[i]];
    }
  } else {
#pragma omp parallel for schedule(static) reduction(+ : sg, sh)
    for (data_size_t i = 0; i < n; ++i) {
      sg += gradients_[i];
      sh += hessians_[i];
    }
  }
  smaller_ = LeafState{0, n, sg, sh, 0.0};
  larger_ = LeafState{};
  larger_.leaf = -1;
}

Tree* SerialTreeLearner::Train(const score_t* gradients, const score_t* hessians) {
  common::ScopedTimer timer("SerialTreeLearner::Train");
  gradients_ = gradients;
  hessians_ = hessians;
  BeforeTrain();
  const bool track = !config_->interaction_constraints_vector.empty();
  std::unique_ptr<Tree> tree(new Tree(config_->num_leaves, track));
  int left_leaf = 0, right_leaf = -1, cur_depth = 1;
  int init_splits = ForceSplits(tree.get(), &left_leaf, &right_leaf, &cur_depth);
  for (int split = init_splits; split < config_->num_leaves - 1; ++split) {
    if (BeforeFindBestSplit(tree.get(), left_leaf, right_leaf)) FindBestSplits(tree.get());
    int best_leaf = 0;
    for (int i = 1; i < static_cast<int>(best_split_per_leaf_.size()); ++i) {
      if (best_split_per_leaf_[i] > best_split_per_leaf_[best_leaf]) best_leaf = i;
    }
    const SplitInfo& b = best_split_per_leaf_[best_leaf];
    if (b.gain <= 0.0) {
      Log::Warning("No further splits with positive gain, best gain: %f", b.gain);
      break;
    }
    Split(tree.get(), best_leaf, &left_leaf, &right_leaf);
    cur_depth = std::max(cur_depth, tree->leaf_depth(left_leaf));
  }
  Log::Debug("Trained a tree with leaves = %d and max_depth = %d", tree->num_leaves(), cur_depth);
  return tree.release();
}

bool SerialTreeLearner::BeforeFindBestSplit(const Tree* tree, int left_leaf, int right_leaf) {
  if (config_->max_depth > 0 && tree->leaf_depth(left_leaf) >= config_->max_depth) {
    best_split_per_leaf_[left_leaf].gain = kMinScore;
    if (right_leaf >= 0) best_split_per_leaf_[right_leaf].gain = kMinScore;
    return false;
  }
  const data_size_t nl = GetGlobalDataCountInLeaf(left_leaf);
  const data_size_t nr = GetGlobalDataCountInLeaf(right_leaf);
  if (nr < static_cast<data_size_t>(config_->min_data_in_leaf * 2) &&
      nl < static_cast<data_size_t>(config_->min_data_in_leaf * 2)) {
    best_split_per_leaf_[left_leaf].gain = kMinScore;
    if (right_leaf >= 0) best_split_per_leaf_[right_leaf].gain = kMinScore;
    return false;
  }
  has_parent_hist_ = false;
  if (right_leaf < 0) {
    smaller_slot_ = left_leaf;
    larger_slot_ = -1;
    PoolAssign(left_leaf, -1);
    return true;
  }
  // the parent's histogram (held by the left leaf id) moves to the larger child; the smaller
  // child takes a new slot.  A parent evicted from a bounded pool: both children from rows.
  const bool parent_cached = leaf_slot_[left_leaf] >= 0;
  if (nl < nr) {
    std::swap(splittable_[left_leaf], splittable_[right_leaf]);
    larger_slot_ = right_leaf;
    smaller_slot_ = left_leaf;
    PoolMove(left_leaf, right_leaf);
  } else {
    larger_slot_ = left_leaf;
    smaller_slot_ = right_leaf;
    PoolTouch(left_leaf);
  }
  has_parent_hist_ = parent_cached;
  PoolAssign(larger_slot_, -1);
  PoolAssign(smaller_slot_, larger_slot_);
  return true;
}

std::vector<int8_t> SerialTreeLearner::GroupsUsed(const std::vector<int8_t>& feature_used) const {
  std::vector<int8_t> g(data_->num_groups(), 0);
  for (int f = 0; f < num_features_; ++f) {
    if (feature_used[f]) g[data_->Feature2Group(f)] = 1;
  }
  return g;
}

void SerialTreeLearner::FindBestSplits(const Tree* tree) {
  std::vector<int8_t> used(num_features_, 0);
  const auto& bytree = col_sampler_.is_feature_used_bytree();
  for (int f = 0; f < num_features_; ++f) {
    if (!bytree[f]) continue;
    if (!feature_mask_.empty() && !feature_mask_[f]) continue;
    if (has_parent_hist_ && !splittable_[larger_slot_][f]) {
      splittable_[smaller_slot_][f] = 0;
      continue;
    }
    used[f] = 1;
  }
  ConstructHistograms(used, has_parent_hist_);
  FindBestSplitsFromHistograms(used, has_parent_hist_, tree);
}

void SerialTreeLearner::ConstructHistograms(const std::vector<int8_t>& feature_used, bool use_subtract) {
  common::ScopedTimer timer("SerialTreeLearner::ConstructHistograms");
  auto groups = GroupsUsed(feature_used);
  data_size_t cnt = 0;
  const data_size_t* idx = LeafIndices(smaller_.leaf, &cnt);
  const bool all_rows = !use_bag_ && cnt == num_data_;
  bool built = false;
  if (hist_mode_ == 0) {
    // deterministic: col-wise (the two modes sum in different orders, a timing choice would
    // make models differ between runs); else the timing test, whose winning build is kept
    if (config_->deterministic) {
      SetHistMode(1);
    } else {
      SetHistMode(ChooseHistogramThreading(groups, all_rows ? nullptr : idx, cnt));
      built = true;
    }
  }
  const bool row_wise = hist_mode_ == 2;
  if (!built) {
    data_->ConstructHistograms(groups, all_rows ? nullptr : idx, cnt, gradients_, hessians_,
                               LeafHist(smaller_slot_).data(), row_wise, &row_scratch_);
  }
  if (larger_slot_ >= 0 && !use_subtract) {
    const data_size_t* idx2 = LeafIndices(larger_.leaf, &cnt);
    data_->ConstructHistograms(groups, idx2, cnt, gradients_, hessians_, LeafHist(larger_slot_).data(), row_wise,
                               &row_scratch_);
  }
}

// auto threading (reference Dataset::TestMultiThreadingMethod, dataset.cpp:589-684): the
// first histogram is built both ways and the faster one is kept for the rest of training
// (the leaf's histogram is left built by the faster mode)
int SerialTreeLearner::ChooseHistogramThreading(const std::vector<int8_t>& groups, const data_size_t* idx,
                                                data_size_t cnt) {
  std::vector<hist_t>& leaf = LeafHist(smaller_slot_);
  std::vector<hist_t> other(leaf.size());
  // (held for the test; SetHistMode(2) below keeps it if row-wise wins)
  data_->RetainRowMajor();
  struct Hold {
    const Dataset* d;
    ~Hold() { d->ReleaseRowMajor(); }
  } hold{data_};
  const double t0 = common::NowSeconds();
  data_->ConstructHistograms(groups, idx, cnt, gradients_, hessians_, leaf.data(), false);
  const double t1 = common::NowSeconds();
  data_->ConstructHistograms(groups, idx, cnt, gradients_, hessians_, other.data(), true, &row_scratch_);
  const double t2 = common::NowSeconds();
  const bool row = (t2 - t1) < (t1 - t0);
  if (row) leaf.swap(other);
  // col-wise won: this learner's per-thread buffers go, and the Dataset's row-major copy with
  // the test's hold unless another learner holds it
  if (!row) Dataset::RowWiseScratch().bufs.swap(row_scratch_.bufs);
  if (row) SetHistMode(2);  // (taken before the test's hold is released)
  Log::Info("Auto-choosing %s-wise multi-threading, the overhead of testing was %f seconds.\n"
            "You can set `force_%s_wise=true` to remove the overhead.",
            row ? "row" : "col", t2 - t0, row ? "row" : "col");
  return row ? 2 : 1;
}

void SerialTreeLearner::ComputeBestSplitForFeature(int slot, int inner, const std::vector<int8_t>& node_used,
                                                   const LeafState& ls, int depth, SplitInfo* best) {
  if (!node_used[inner]) return;
  splittable_[slot][inner] = EvalFeature(FeatureHist(slot, inner), inner, params_, ls, depth, best) ? 1 : 0;
}

bool SerialTreeLearner::EvalFeature(hist_t* hist, int inner, const SplitParams& p, const LeafState& ls, int depth,
                                    SplitInfo* best, const FeatureMeta* meta) {
  const ConstraintRange& c = constraints_.entries[ls.leaf];
  double parent_output;
  if (ls.leaf == 0) {
    SplitParams rp = p;
    rp.use_l1 = 1;
    rp.use_max_output = 1;
    rp.use_smoothing = 0;
    rp.use_mc = 1;
    parent_output = LeafOutputConstrained(ls.sum_g, ls.sum_h, p.lambda_l2, rp, c, ls.num_data, 0);
  } else {
    parent_output = ls.output;
  }
  SplitInfo ns;
  bool splittable = false;
  FindBestThreshold(meta != nullptr ? *meta : meta_[inner], p, config_->extra_trees, hist, ls.sum_g, ls.sum_h,
                    ls.num_data, c, parent_output, &ns, &splittable);
  ns.feature = data_->RealFeatureIndex(inner);
  ns.inner_feature = inner;
  if (cegb_) ns.gain -= cegb_->DeltaGain(inner, ns.feature, ls.leaf, ls.num_data, ns);
  if (ns.monotone_type != 0) {
    // reference: penalty by the leaf's depth in the tree being grown
    ns.gain *= MonotoneSplitPenalty(depth, config_->monotone_penalty);
  }
  if (ns > *best) *best = ns;
  return splittable;
}

void SerialTreeLearner::FindBestSplitsFromHistograms(const std::vector<int8_t>& used, bool use_subtract,
                                                     const Tree* tree) {
  common::ScopedTimer timer("SerialTreeLearner::FindBestSplitsFromHistograms");
  PrepareCegbLeaves();
  auto small_node = col_sampler_.GetByNode(tree, smaller_.leaf);
  std::vector<int8_t> large_node;
  if (larger_.leaf >= 0) large_node = col_sampler_.GetByNode(tree, larger_.leaf);
  const int nt = omp_get_max_threads();
  std::vector<SplitInfo> sb(nt), lb(nt);
  const int small_depth = tree->leaf_depth(smaller_.leaf);
  const int large_depth = larger_.leaf >= 0 ? tree->leaf_depth(larger_.leaf) : 0;
#pragma omp parallel for schedule(static)
  for (int f = 0; f < num_features_; ++f) {
    if (!used[f]) continue;
    const int tid = omp_get_thread_num();
    data_->FixHistogram(f, smaller_.sum_g, smaller_.sum_h, FeatureHist(smaller_slot_, f));
    ComputeBestSplitForFeature(smaller_slot_, f, small_node, smaller_, small_depth, &sb[tid]);
    if (larger_.leaf < 0) continue;
    hist_t* lh = FeatureHist(larger_slot_, f);
    if (use_subtract) {
      const hist_t* sh = FeatureHist(smaller_slot_, f);
      const int n = 2 * data_->FeatureHistSize(f);
      for (int i = 0; i < n; ++i) lh[i] -= sh[i];
    } else {
      data_->FixHistogram(f, larger_.sum_g, larger_.sum_h, lh);
    }
    ComputeBestSplitForFeature(larger_slot_, f, large_node, larger_, large_depth, &lb[tid]);
  }
  SplitInfo best_s, best_l;
  for (int t = 0; t < nt; ++t) {
    if (sb[t] > best_s) best_s = sb[t];
    if (lb[t] > best_l) best_l = lb[t];
  }
  best_split_per_leaf_[smaller_.leaf] = best_s;
  if (larger_.leaf >= 0) best_split_per_leaf_[larger_.leaf] = best_l;
}

data_size_t SerialTreeLearner::PartitionLeaf(int leaf, int inner, const SplitInfo& s, int new_leaf) {
  const data_size_t begin = leaf_begin_[leaf];
  const data_size_t cnt = leaf_count_[leaf];
  data_size_t* idx = indices_.data() + begin;
  const BinMapper* m = data_->FeatureBinMapper(inner);
  const bool is_cat = m->bin_type() == BinType::Categorical;
  const uint32_t default_bin = m->GetDefaultBin();
  const uint32_t nan_bin = static_cast<uint32_t>(m->num_bin() - 1);
  const MissingType mt = m->missing_type();
  std::vector<uint32_t> bits;
  if (is_cat) bits = common::ConstructBitset(s.cat_threshold.data(), s.num_cat_threshold);
  auto goes_left = [&](Dataset::BinReader& rd, data_size_t row) -> bool {
    const uint32_t b = rd.Get(row);
    if (is_cat) return common::FindInBitset(bits.data(), static_cast<int>(bits.size()), b);
    if ((mt == MissingType::Zero && b == default_bin) || (mt == MissingType::NaN && b == nan_bin)) return s.default_left;
    return b <= s.threshold;
  };
  // blocked parallel stable partition
  const int nb = std::max(1, std::min(omp_get_max_threads() * 4, static_cast<int>((cnt + 4095) / 4096)));
  const data_size_t bs = (cnt + nb - 1) / nb;
  std::vector<data_size_t> lc(nb, 0), rc(nb, 0);
#pragma omp parallel for schedule(static)
  for (int b = 0; b < nb; ++b) {
    const data_size_t s0 = b * bs, e0 = std::min(cnt, s0 + bs);
    data_size_t l = 0, r = 0;
    Dataset::BinReader rd = data_->FeatureBinReader(inner);  // (a leaf's rows are ascending)
    for (data_size_t i = s0; i < e0; ++i) {
      if (goes_left(rd, idx[i])) tmp_left_[begin + s0 + l++] = idx[i];
      else tmp_right_[begin + s0 + r++] = idx[i];
    }
    lc[b] = l;
    rc[b] = r;
  }
  std::vector<data_size_t> lo(nb + 1, 0), ro(nb + 1, 0);
  for (int b = 0; b < nb; ++b) {
    lo[b + 1] = lo[b] + lc[b];
    ro[b + 1] = ro[b] + rc[b];
  }
  const data_size_t left_total = lo[nb];
#pragma omp parallel for schedule(static)
  for (int b = 0; b < nb; ++b) {
    const data_size_t s0 = b * bs;
    std::copy(tmp_left_.begin() + begin + s0, tmp_left_.begin() + begin + s0 + lc[b], idx + lo[b]);
    std::copy(tmp_right_.begin() + begin + s0, tmp_right_.begin() + begin + s0 + rc[b], idx + left_total + ro[b]);
  }
  leaf_count_[leaf] = left_total;
  leaf_begin_[new_leaf] = begin + left_total;
  leaf_count_[new_leaf] = cnt - left_total;
  return left_total;
}

void SerialTreeLearner::Split(Tree* tree, int best_leaf, int* left_leaf, int* right_leaf) {
  SplitInner(tree, best_leaf, left_leaf, right_leaf, true);
}

void SerialTreeLearner::SplitInner(Tree* tree, int best_leaf, int* left_leaf, int* right_leaf, bool update_cnt) {
  common::ScopedTimer timer("SerialTreeLearner::SplitInner");
  SplitInfo& s = best_split_per_leaf_[best_leaf];
  const int inner = data_->InnerFeatureIndex(s.feature);
  if (cegb_) {
    data_size_t cnt = 0;
    const data_size_t* rows = config_->cegb_penalty_feature_lazy.empty() ? nullptr : HostLeafRows(best_leaf, &cnt);
    cegb_->OnSplit(tree, best_leaf, s, rows, cnt, &best_split_per_leaf_);
  }
  *left_leaf = best_leaf;
  const int next = tree->NextLeafId();
  const BinMapper* m = data_->FeatureBinMapper(inner);
  const bool is_num = m->bin_type() == BinType::Numerical;
  constraints_.BeforeSplit(tree, best_leaf, next, s.monotone_type);
  PartitionLeaf(best_leaf, inner, s, next);
  if (update_cnt) {
    s.left_count = leaf_count_[best_leaf];
    s.right_count = leaf_count_[next];
  }
  const float gain = static_cast<float>(s.gain + config_->min_gain_to_split);
  if (is_num) {
    *right_leaf = tree->Split(best_leaf, inner, s.feature, s.threshold, data_->RealThreshold(inner, s.threshold),
                              s.left_output, s.right_output, s.left_count, s.right_count, s.left_sum_hessian,
                              s.right_sum_hessian, gain, m->missing_type(), s.default_left);
  } else {
    auto bits_inner = common::ConstructBitset(s.cat_threshold.data(), s.num_cat_threshold);
    std::vector<int> cats(s.num_cat_threshold);
    for (int i = 0; i < s.num_cat_threshold; ++i) cats[i] = static_cast<int>(data_->RealThreshold(inner, s.cat_threshold[i]));
    auto bits = common::ConstructBitset(cats.data(), s.num_cat_threshold);
    *right_leaf = tree->SplitCategorical(best_leaf, inner, s.feature, bits_inner.data(),
                                         static_cast<int>(bits_inner.size()), bits.data(), static_cast<int>(bits.size()),
                                         s.left_output, s.right_output, s.left_count, s.right_count,
                                         s.left_sum_hessian, s.right_sum_hessian, gain, m->missing_type());
  }
  if (s.left_count < s.right_count) {
    LGBM_CHECK_GT(s.left_count, 0);
    smaller_ = LeafState{*left_leaf, leaf_count_[*left_leaf], s.left_sum_gradient, s.left_sum_hessian, s.left_output};
    larger_ = LeafState{*right_leaf, leaf_count_[*right_leaf], s.right_sum_gradient, s.right_sum_hessian, s.right_output};
  } else {
    LGBM_CHECK_GT(s.right_count, 0);
    smaller_ = LeafState{*right_leaf, leaf_count_[*right_leaf], s.right_sum_gradient, s.right_sum_hessian, s.right_output};
    larger_ = LeafState{*left_leaf, leaf_count_[*left_leaf], s.left_sum_gradient, s.left_sum_hessian, s.left_output};
  }
  if (!update_cnt) {
    // data-parallel: leaf sizes are global counts from the split info
    smaller_.num_data = smaller_.leaf == *left_leaf ? s.left_count : s.right_count;
    larger_.num_data = larger_.leaf == *left_leaf ? s.left_count : s.right_count;
  }
  const auto stale = constraints_.Update(tree, is_num, *left_leaf, *right_leaf, s.monotone_type, s.right_output,
                                         s.left_output, inner, s, best_split_per_leaf_);
  for (int leaf : stale) RecomputeBestSplitForLeaf(tree, leaf);
}

void SerialTreeLearner::RecomputeBestSplitForLeaf(const Tree* tree, int leaf) {
  SplitInfo& cur = best_split_per_leaf_[leaf];
  const int slot = leaf;  // (FeatureHist maps the leaf to its pool slot)
  if (leaf_slot_[leaf] < 0) {  // evicted from a bounded pool (reference: skipped with a warning)
    Log::Warning("Get historical Histogram for leaf %d failed, will skip the ``RecomputeBestSplitForLeaf``", leaf);
    return;
  }
  // the leaf's statistics as its current best split saw them (reference: a fresh LeafSplits,
  // whose output -- the smoothing parent -- is 0)
  LeafState ls{leaf, cur.left_count + cur.right_count, cur.left_sum_gradient + cur.right_sum_gradient,
               cur.left_sum_hessian + cur.right_sum_hessian, 0.0};
  const auto& bytree = col_sampler_.is_feature_used_bytree();
  const int depth = tree->leaf_depth(leaf);
  std::vector<SplitInfo> bests(num_features_);
#pragma omp parallel for schedule(static)
  for (int f = 0; f < num_features_; ++f) {
    if (!bytree[f] || !splittable_[slot][f]) continue;
    EvalFeature(FeatureHist(slot, f), f, params_, ls, depth, &bests[f]);
  }
  SplitInfo best;
  for (const auto& b : bests) {
    if (b > best) best = b;
  }
  cur = best;
}

int SerialTreeLearner::ForceSplits(Tree* tree, int* left_leaf, int* right_leaf, int* cur_depth) {
  if (!has_forced_split_) return 0;
  bool abort_last = false;
  int count = 0;
  *left_leaf = 0;
  std::queue<std::pair<Json, int>> q;
  Json left = forced_split_, right;
  bool left_smaller = true;
  std::unordered_map<int, SplitInfo> forced;
  q.push({left, *left_leaf});
  auto gather = [&](const Json& node, bool use_smaller, SplitInfo* out) {
    const int feat = node["feature"].int_value();
    const int inner = data_->InnerFeatureIndex(feat);
    if (inner < 0) {
      out->gain = kMinScore;
      return;
    }
    const uint32_t thr = data_->BinThreshold(inner, node["threshold"].number_value());
    const LeafState& ls = use_smaller ? smaller_ : larger_;
    const int slot = use_smaller ? smaller_slot_ : larger_slot_;
    GatherInfoForThreshold(meta_[inner], params_, FeatureHist(slot, inner), ls.sum_g, ls.sum_h, thr, ls.num_data,
                           ls.output, out);
    out->feature = feat;
    out->inner_feature = inner;
  };
  while (!q.empty()) {
    if (BeforeFindBestSplit(tree, *left_leaf, *right_leaf)) FindBestSplits(tree);
    if (!left.is_null()) {
      SplitInfo ls;
      gather(left, left_smaller, &ls);
      forced[*left_leaf] = ls;
      if (ls.gain < 0) forced.erase(*left_leaf);
    }
    if (!right.is_null()) {
      SplitInfo rs;
      gather(right, !left_smaller, &rs);
      forced[*right_leaf] = rs;
      if (rs.gain < 0) forced.erase(*right_leaf);
    }
    auto pr = q.front();
    q.pop();
    const int cur = pr.second;
    if (!forced.count(cur)) {
      abort_last = true;
      break;
    }
    best_split_per_leaf_[cur] = forced[cur];
    Split(tree, cur, left_leaf, right_leaf);
    left_smaller = best_split_per_leaf_[cur].left_count < best_split_per_leaf_[cur].right_count;
    left = Json();
    right = Json();
    const Json& node = pr.first;
    if (node.has("left")) {
      left = node["left"];
      if (left.has("feature") && left.has("threshold")) q.push({left, *left_leaf});
    }
    if (node.has("right")) {
      right = node["right"];
      if (right.has("feature") && right.has("threshold")) q.push({right, *right_leaf});
    }
    ++count;
    *cur_depth = std::max(*cur_depth, tree->leaf_depth(*left_leaf));
  }
  if (abort_last) {
    int best = 0;
    for (int i = 1; i < static_cast<int>(best_split_per_leaf_.size()); ++i) {
      if (best_split_per_leaf_[i] > best_split_per_leaf_[best]) best = i;
    }
    if (best_split_per_leaf_[best].gain <= 0.0) {
      Log::Warning("No further splits with positive gain, best gain: %f", best_split_per_leaf_[best].gain);
      return config_->num_leaves;
    }
    Split(tree, best, left_leaf, right_leaf);
    *cur_depth = std::max(*cur_depth, tree->leaf_depth(*left_leaf));
    ++count;
  }
  return count;
}

void SerialTreeLearner::AddPredictionToScore(const Tree* tree, double* out) const {
  if (tree->num_leaves() <= 1) return;
#pragma omp parallel for schedule(static, 1)
  for (int i = 0; i < tree->num_leaves(); ++i) {
    const double v = tree->LeafOutput(i);
    data_size_t cnt;
    const data_size_t* idx = LeafIndices(i, &cnt);
    for (data_size_t j = 0; j < cnt; ++j) out[idx[j]] += v;
  }
}

void SerialTreeLearner::RenewTreeOutput(Tree* tree, const ObjectiveFunction* obj,
                                        const std::function<double(const label_t*, int)>& residual,
                                        data_size_t, const data_size_t*, data_size_t) const {
  if (obj == nullptr || !obj->IsRenewTreeOutput()) return;
  const int nm = Network::num_machines();
  std::vector<int> nonzero(tree->num_leaves(), 1);
#pragma omp parallel for schedule(static)
  for (int i = 0; i < tree->num_leaves(); ++i) {
    data_size_t cnt;
    const data_size_t* idx = LeafIndices(i, &cnt);
    if (cnt > 0) {
      tree->SetLeafOutput(i, obj->RenewTreeOutput(tree->LeafOutput(i), residual, idx, nullptr, cnt));
    } else {
      tree->SetLeafOutput(i, 0.0);
      nonzero[i] = 0;
    }
  }
  if (nm > 1) {
    std::vector<double> outs(tree->num_leaves());
    for (int i = 0; i < tree->num_leaves(); ++i) outs[i] = tree->LeafOutput(i);
    outs = Network::GlobalSum(outs);
    nonzero = Network::GlobalSum(nonzero);
    for (int i = 0; i < tree->num_leaves(); ++i) tree->SetLeafOutput(i, outs[i] / nonzero[i]);
  }
}

Tree* SerialTreeLearner::FitByExistingTree(const Tree* old_tree, const score_t* g, const score_t* h) const {
  std::unique_ptr<Tree> tree(new Tree(*old_tree));
  const bool smooth = config_->path_smooth > kEpsilon;
#pragma omp parallel for schedule(static)
  for (int i = 0; i < tree->num_leaves(); ++i) {
    data_size_t cnt;
    const data_size_t* idx = LeafIndices(i, &cnt);
    double sg = 0, sh = kEpsilon;
    for (data_size_t j = 0; j < cnt; ++j) {
      sg += g[idx[j]];
      sh += h[idx[j]];
    }
    double out;
    if (smooth && i > 0) {
      out = LeafOutputRaw(sg, sh, config_->lambda_l1, config_->lambda_l2, config_->max_delta_step,
                          config_->path_smooth, cnt, tree->leaf_parent(i), 1, 1, 1);
    } else {
      out = LeafOutputRaw(sg, sh, config_->lambda_l1, config_->lambda_l2, config_->max_delta_step,
                          config_->path_smooth, cnt, 0, 1, 1, 0);
    }
    const double old = tree->LeafOutput(i);
    const double nw = out * tree->shrinkage();
    tree->SetLeafOutput(i, config_->refit_decay_rate * old + (1.0 - config_->refit_decay_rate) * nw);
  }
  return tree.release();
}

Tree* SerialTreeLearner::FitByExistingTree(const Tree* old_tree, const std::vector<int>& leaf_pred,
                                           const score_t* g, const score_t* h) {
  const int nl = old_tree->num_leaves();
  LGBM_CHECK_LE(nl, config_->num_leaves);
  std::vector<data_size_t> cnt(nl, 0);
  for (data_size_t i = 0; i < num_data_; ++i) ++cnt[leaf_pred[i]];
  data_size_t off = 0;
  for (int l = 0; l < nl; ++l) {
    leaf_begin_[l] = off;
    leaf_count_[l] = 0;
    off += cnt[l];
  }
  for (data_size_t i = 0; i < num_data_; ++i) {
    const int l = leaf_pred[i];
    indices_[leaf_begin_[l] + leaf_count_[l]++] = i;
  }
  return FitByExistingTree(old_tree, g, h);
}

SerialTreeLearner::LeafState SerialTreeLearner::LocalLeafSums(int leaf) const {
  data_size_t cnt = 0;
  const data_size_t* idx = LeafIndices(leaf, &cnt);
  double sg = 0, sh = 0;
#pragma omp parallel for schedule(static) reduction(+ : sg, sh)
  for (data_size_t i = 0; i < cnt; ++i) {
    sg += gradients_[idx[i]];
    sh += hessians_[idx[i]];
  }
  return LeafState{leaf, cnt, sg, sh, 0.0};
}

}  // namespace lgbm_amd
