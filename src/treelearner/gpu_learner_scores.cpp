// MI355X tree learner: validation sets, device-resident training scores, gradients and
// row sampling.
#include "gpu_learner_internal.h"
#include "lgbm_amd/tuning.h"

namespace lgbm_amd {

// ---------------------------------------------------------------- validation sets
int GPUTreeLearner::AddValidData(const Dataset* valid, int ntpi, const double* scores) {
  if (valid->num_groups() != num_groups_ || valid->num_total_bin() != data_->num_total_bin()) return -1;
  for (int g = 0; g < num_groups_; ++g) {
    if (valid->group_bin_boundary(g) != data_->group_bin_boundary(g) ||
        valid->group(g).num_total_bin != data_->group(g).num_total_bin) {
      return -1;
    }
  }
  HIPCHECK(hipSetDevice(device_id_));
  ValidSet vs;
  vs.num_data = valid->num_data();
  vs.ntpi = ntpi;
  std::vector<uint8_t> host = RowMajorBins(valid, args_.words_per_row);
  HIPCHECK(hipMalloc(&vs.bins, std::max<size_t>(1, host.size())));
  valid_allocs_.push_back(vs.bins);
  HIPCHECK(hipMemcpy(vs.bins, host.data(), host.size(), hipMemcpyHostToDevice));
  const size_t ns = static_cast<size_t>(vs.num_data) * ntpi;
  HIPCHECK(hipMalloc(reinterpret_cast<void**>(&vs.score), std::max<size_t>(1, ns) * sizeof(double)));
  valid_allocs_.push_back(vs.score);
  HIPCHECK(hipMemcpy(vs.score, scores, ns * sizeof(double), hipMemcpyHostToDevice));
  valid_.push_back(vs);
  return static_cast<int>(valid_.size()) - 1;
}

void GPUTreeLearner::ValidAddConst(int slot, double v, int k) {
  const ValidSet& vs = valid_[slot];
  dev::AddConst(vs.score + static_cast<size_t>(k) * vs.num_data, vs.num_data, v, stream_);
}

void GPUTreeLearner::ValidMultiply(int slot, double v, int k) {
  const ValidSet& vs = valid_[slot];
  dev::MulConst(vs.score + static_cast<size_t>(k) * vs.num_data, vs.num_data, v, stream_);
}

void GPUTreeLearner::ValidAddTree(int slot, const Tree* tree, int k) {
  const ValidSet& vs = valid_[slot];
  double* score = vs.score + static_cast<size_t>(k) * vs.num_data;
  if (tree->num_leaves() <= 1) {
    dev::AddConst(score, vs.num_data, tree->LeafOutput(0), stream_);
    return;
  }
  dev::DevTree t = StageTree(tree);
  dev::KArgs a = args_;
  a.bins = vs.bins;
  a.row_words = a.words_per_row;  // (validation rows carry no (g, h))
  dev::AddTreeScore(a, t, nullptr, vs.num_data, score, stream_);
}

bool GPUTreeLearner::ValidEval(int slot, const DeviceMetricSpec& spec, std::vector<double>* sums) {
  ValidSet& vs = valid_[slot];
  if (spec.kind == 0 || spec.label == nullptr || vs.num_data <= 0) return false;
  const bool aucmu = spec.kind == dev::kMetricAucMu;
  const bool multi = spec.kind == dev::kMetricMultiLogloss || spec.kind == dev::kMetricMultiError || aucmu;
  const bool query = spec.kind == dev::kMetricNDCG || spec.kind == dev::kMetricMAP;
  if (vs.ntpi != (multi ? spec.num_class : 1)) return false;
  if (query && (spec.qb == nullptr || spec.nq <= 0 || spec.eval_at.empty())) return false;
  // a query's device ranking is O(cnt^2) on one workgroup; very long queries are sorted on the
  // host in O(cnt log cnt) instead (reference rank_metric.hpp)
  if (query && spec.max_query_docs > tuning::kQueryMetricDeviceMaxDocs) return false;
  HIPCHECK(hipSetDevice(device_id_));
  const size_t n = static_cast<size_t>(vs.num_data);
  auto dev_alloc = [&](size_t bytes) {
    void* p = nullptr;
    HIPCHECK(hipMalloc(&p, std::max<size_t>(1, bytes)));
    valid_allocs_.push_back(p);
    return p;
  };
  auto upload = [&](const void* src, size_t bytes) {
    void* d = dev_alloc(bytes);
    if (bytes > 0) HIPCHECK(hipMemcpy(d, src, bytes, hipMemcpyHostToDevice));
    return d;
  };
  if (vs.label == nullptr || vs.label_src != spec.label || vs.weights_src != spec.weights) {
    if (vs.label != nullptr) ReleaseValidInputs(&vs);  // (the set's fields were replaced)
    vs.label = static_cast<float*>(upload(spec.label, sizeof(float) * n));
    if (spec.weights != nullptr) vs.weights = static_cast<float*>(upload(spec.weights, sizeof(float) * n));
    vs.label_src = spec.label;
    vs.weights_src = spec.weights;
    vs.negative_weights = false;
    if (spec.weights != nullptr) {
      for (size_t i = 0; i < n && !vs.negative_weights; ++i) vs.negative_weights = spec.weights[i] < 0.0f;
    }
    vs.metric_out = static_cast<double*>(dev_alloc(sizeof(double) * 64));
  }
  if (spec.nout > 64) return false;
  // the device AUC sorts each row's weight with its class in the sign: a negative weight would
  // flip the class (the reference binary_metric.hpp:240-241 adds it to the row's own class)
  if (spec.kind == dev::kMetricAUC && vs.negative_weights) return false;
  dev::MetricArgs m{};
  if (query) {
    // the metric's query inputs, uploaded on its first evaluation
    auto it = vs.queries.find(spec.key);
    if (it == vs.queries.end()) {
      ValidSet::QueryInputs qi;
      std::vector<int32_t> qb(spec.qb, spec.qb + spec.nq + 1);
      qi.qb = static_cast<int32_t*>(upload(qb.data(), sizeof(int32_t) * qb.size()));
      if (spec.qw != nullptr) qi.qw = static_cast<float*>(upload(spec.qw, sizeof(float) * spec.nq));
      std::vector<int32_t> at(spec.eval_at.begin(), spec.eval_at.end());
      qi.eval_at = static_cast<int32_t*>(upload(at.data(), sizeof(int32_t) * at.size()));
      qi.qconst = static_cast<double*>(upload(spec.qconst.data(), sizeof(double) * spec.qconst.size()));
      qi.label_gain = static_cast<double*>(upload(spec.label_gain.data(), sizeof(double) * spec.label_gain.size()));
      qi.discount = static_cast<double*>(upload(spec.discount.data(), sizeof(double) * spec.discount.size()));
      qi.big = spec.max_query_docs > dev::kRankMaxDocs;
      qi.scratch = dev_alloc(dev::MetricScratchBytes(qi.big ? vs.num_data : 0,
                                                     static_cast<int64_t>(spec.nq) * spec.eval_at.size()));
      it = vs.queries.emplace(spec.key, qi).first;
    }
    const ValidSet::QueryInputs& qi = it->second;
    m.nq = spec.nq;
    m.nk = static_cast<int32_t>(spec.eval_at.size());
    m.qb = qi.qb;
    m.qw = qi.qw;
    m.eval_at = qi.eval_at;
    m.qconst = qi.qconst;
    m.label_gain = qi.label_gain;
    m.discount = qi.discount;
    m.scratch = qi.scratch;
    m.big = qi.big ? 1 : 0;
  } else {
    if (aucmu) {  // the class weight matrix, uploaded on the metric's first evaluation
      auto it = vs.queries.find(spec.key);
      if (it == vs.queries.end()) {
        ValidSet::QueryInputs qi;
        qi.qconst = static_cast<double*>(upload(spec.qconst.data(), sizeof(double) * spec.qconst.size()));
        it = vs.queries.emplace(spec.key, qi).first;
      }
      m.qconst = it->second.qconst;
    }
    if ((spec.kind == dev::kMetricAUC || aucmu) && vs.metric_scratch_rows < vs.num_data) {
      vs.metric_scratch = dev_alloc(dev::MetricScratchBytes(vs.num_data));
      vs.metric_scratch_rows = vs.num_data;
    } else if (vs.metric_scratch == nullptr) {
      vs.metric_scratch = dev_alloc(dev::MetricScratchBytes(0));
    }
    m.scratch = vs.metric_scratch;
  }
  m.kind = spec.kind;
  m.convert = spec.convert;
  m.sigmoid = spec.sigmoid;
  m.param = spec.param;
  m.n = vs.num_data;
  m.score = vs.score;
  m.label = vs.label;
  m.weights = vs.weights;
  m.num_class = spec.num_class;
  m.top_k = spec.top_k;
  m.out = vs.metric_out;
  dev::EvalMetric(m, stream_);
  if (vs.logged_kinds.insert(spec.kind).second) {
    if (slot == train_eval_slot_) Log::Debug("device metric (kind %d) on the training set", spec.kind);
    else Log::Debug("device metric (kind %d) on validation set %d", spec.kind, slot);
  }
  sums->assign(std::max(2, spec.nout), 0.0);
  HIPCHECK(hipMemcpyAsync(sums->data(), vs.metric_out, sizeof(double) * sums->size(), hipMemcpyDeviceToHost,
                          stream_));
  HIPCHECK(hipStreamSynchronize(stream_));
  return true;
}

// training metrics (reference gbdt.cpp:484-542 evaluates them every metric_freq iterations):
// the device metric kernels of the validation sets over the resident training scores, so
// valid_sets=[train] costs one reduction instead of an 8 N-byte download and a host pass
bool GPUTreeLearner::TrainEval(const DeviceMetricSpec& spec, std::vector<double>* sums) {
  if (d_score_ == nullptr || num_data_ <= 0) return false;
  if (train_eval_slot_ < 0) {
    valid_.emplace_back();
    train_eval_slot_ = static_cast<int>(valid_.size()) - 1;
  }
  ValidSet& vs = valid_[train_eval_slot_];
  if (vs.score != d_score_ || vs.num_data != num_data_ || vs.ntpi != num_tree_per_iteration_) {
    // the training data was reset (ResetTrainingData re-allocates the scores): the slot's
    // inputs describe the old rows
    ReleaseValidInputs(&vs);
    vs.num_data = num_data_;
    vs.ntpi = num_tree_per_iteration_;
    vs.score = d_score_;  // (not owned: valid_allocs_ holds only the metric inputs)
  }
  return ValidEval(train_eval_slot_, spec, sums);
}

void GPUTreeLearner::ReleaseValidInputs(ValidSet* vs) {
  std::vector<void*> dead = {vs->label, vs->weights, vs->metric_scratch, vs->metric_out};
  for (const auto& kv : vs->queries) {
    const ValidSet::QueryInputs& q = kv.second;
    for (void* p : {static_cast<void*>(q.qb), static_cast<void*>(q.qw), static_cast<void*>(q.eval_at),
                    static_cast<void*>(q.qconst), static_cast<void*>(q.label_gain), static_cast<void*>(q.discount),
                    q.scratch}) {
      dead.push_back(p);
    }
  }
  HIPCHECK(hipStreamSynchronize(stream_));
  for (void* p : dead) {
    if (p == nullptr) continue;
    auto it = std::find(valid_allocs_.begin(), valid_allocs_.end(), p);
    if (it != valid_allocs_.end()) valid_allocs_.erase(it);
    HIPCHECK(hipFree(p));
  }
  vs->label = vs->weights = nullptr;
  vs->label_src = vs->weights_src = nullptr;
  vs->negative_weights = false;
  vs->metric_scratch = nullptr;
  vs->metric_scratch_rows = 0;
  vs->metric_out = nullptr;
  vs->queries.clear();
}

void GPUTreeLearner::ValidScoreToHost(int slot, double* host) {
  const ValidSet& vs = valid_[slot];
  HIPCHECK(hipMemcpyAsync(host, vs.score, sizeof(double) * vs.num_data * vs.ntpi, hipMemcpyDeviceToHost, stream_));
  HIPCHECK(hipStreamSynchronize(stream_));
}

// ---------------------------------------------------------------- scores & gradients
void GPUTreeLearner::InitScores(int ntpi, const double* init_score) {
  HIPCHECK(hipSetDevice(device_id_));
  grad_prefetched_ = false;
  num_tree_per_iteration_ = ntpi;
  const size_t n = static_cast<size_t>(num_data_) * ntpi;
  if (d_score_ == nullptr) {
    d_score_ = Alloc<double>(n);
    d_grad_ = Alloc<float>(n);
    d_hess_ = Alloc<float>(n);
  }
  if (init_score != nullptr) {
    HIPCHECK(hipMemcpy(d_score_, init_score, sizeof(double) * n, hipMemcpyHostToDevice));
  } else {
    HIPCHECK(hipMemset(d_score_, 0, sizeof(double) * n));
  }
}

void GPUTreeLearner::SyncScoreToHost(double* host, int k) {
  HIPCHECK(hipMemcpyAsync(host, d_score_ + static_cast<size_t>(k) * num_data_, sizeof(double) * num_data_,
                          hipMemcpyDeviceToHost, stream_));
  HIPCHECK(hipStreamSynchronize(stream_));
}

void GPUTreeLearner::SyncScoreFromHost(const double* host, int k) {
  grad_prefetched_ = false;
  HIPCHECK(hipMemcpyAsync(d_score_ + static_cast<size_t>(k) * num_data_, host, sizeof(double) * num_data_,
                          hipMemcpyHostToDevice, stream_));
  HIPCHECK(hipStreamSynchronize(stream_));
}

void GPUTreeLearner::AddConstToScore(double v, int k) {
  grad_prefetched_ = false;
  dev::AddConst(d_score_ + static_cast<size_t>(k) * num_data_, num_data_, v, stream_);
}

void GPUTreeLearner::MultiplyScore(double v, int k) {
  grad_prefetched_ = false;
  dev::MulConst(d_score_ + static_cast<size_t>(k) * num_data_, num_data_, v, stream_);
}

bool GPUTreeLearner::FusedScoreWalk(int num_leaves, int k) const {
  return dev::TreeBitmapsApply(args_, num_leaves) && last_grad_fusable_ && k == 0 && num_tree_per_iteration_ == 1 &&
         dev::AddTreeScoreGradKind(last_grad_.kind) && FuseNextGradients();
}

// The tree the device just grew goes into the training scores (with the next gradients) from
// its split records, before the host has built the Tree object: the score walk overlaps the
// host's tree building and its return through GBDT::TrainOneIter.  AddTrainedTreeToScore then
// only takes note.  The same DevTree and kernels as that call's fused path: the same scores.
void GPUTreeLearner::EarlyScoreUpdate(int nsplit, double shrinkage) {
  const int L = config_->num_leaves;
  if (d_early_blob_ == nullptr) d_early_blob_ = Alloc<char>(dev::TreeFromRecordsBytes(L));
  const int nbm = std::max(1, L - 1);
  if (tree_bm_cap_ < nbm) {
    tree_bm_cap_ = nbm;
    d_tree_bm_ = Alloc<unsigned long long>(4 * static_cast<size_t>(nbm));
    d_tree_bm_meta_ = Alloc<int32_t>(3 * static_cast<size_t>(nbm));
  }
  dev::DevTree t = dev::TreeFromRecords(args_, nsplit, L, shrinkage, d_early_blob_, stream_, d_tree_bm_, d_tree_bm_meta_);
  t.bm_work = d_tree_bm_;
  t.bm_meta = d_tree_bm_meta_;
  dev::AddTreeScoreGrad(args_, t, num_data_, d_score_, last_grad_, stream_);
  early_scored_leaves_ = nsplit + 1;
}

void GPUTreeLearner::AddTrainedTreeToScore(const Tree* tree, int k) {
  const int nl = tree->num_leaves();
  double* score = d_score_ + static_cast<size_t>(k) * num_data_;
  if (early_scored_leaves_ > 0) {  // (added by EarlyScoreUpdate during Train)
    if (nl != early_scored_leaves_ || k != 0) {
      Log::Fatal("device learner: the tree added to the training scores early has %d leaves, this one %d (class %d)",
                 early_scored_leaves_, nl, k);
    }
    early_scored_leaves_ = 0;
    grad_parts_ = dev::AddTreeScoreGradParts(num_data_);
    grad_prefetched_ = true;
    gh_fresh_ = false;    // (d_gh_ now holds the next iteration's gradients ...
    split_stale_ = true;  //  ... and d_grad_ / d_hess_ are behind it until unpacked)
    return;
  }
  if (nl <= 1) {
    AddConstToScore(tree->LeafOutput(0), k);
    return;
  }
  if (dev::TreeBitmapsApply(args_, nl)) {
    // the bitmap walk of every row (coalesced row reads and score updates) beats the
    // partition-ordered scatter of leaf values; it also covers out-of-bag rows.  Wider or
    // row-sparse storage scatters instead (the generic walk took 5 ms per tree on 100M rows)
    if (FusedScoreWalk(nl, k)) {
      // ... and computes the next iteration's gradients from the scores it writes
      dev::DevTree t = StageTree(tree);
      dev::AddTreeScoreGrad(args_, t, num_data_, score, last_grad_, stream_);
      grad_parts_ = dev::AddTreeScoreGradParts(num_data_);
      grad_prefetched_ = true;
      gh_fresh_ = false;    // (d_gh_ now holds the next iteration's gradients ...
      split_stale_ = true;  //  ... and d_grad_ / d_hess_ are behind it until unpacked)
      return;
    }
    AddTreeToScore(tree, k);
    return;
  }
  if (!device_mode_) {
    // host-assisted growth keeps the leaves' row ranges on the host (the device leaf records
    // are the last device-resident tree's): walk the tree for every row instead
    AddTreeToScore(tree, k);
    return;
  }
  std::vector<double> vals(nl);
  for (int i = 0; i < nl; ++i) vals[i] = tree->LeafOutput(i);
  HIPCHECK(hipMemcpyAsync(d_leaf_values_, vals.data(), sizeof(double) * nl, hipMemcpyHostToDevice, stream_));
  dev::KArgs a = args_;
  a.num_rows = root_rows_;
  dev::AddLeafScore(a, d_leaf_values_, nl, score, stream_);
  if (oob_cnt_ > 0) {
    in_trained_update_ = true;  // AddTreeToScore restricts the traversal to out-of-bag rows
    AddTreeToScore(tree, k);
    in_trained_update_ = false;
  }
  HIPCHECK(hipStreamSynchronize(stream_));
}

dev::DevTree GPUTreeLearner::StageTree(const Tree* tree) {
  const int nl = tree->num_leaves();
  const int ni = nl - 1;
  const auto& cb = tree->cat_boundaries_inner();
  const auto& ct = tree->cat_threshold_inner();
  // blob: [i32: split feature, left, right, category boundaries][u32: thresholds, category
  // words][f64: leaf values][i8: decision types], 8-byte aligned sections
  auto up8 = [](size_t x) { return (x + 7) & ~static_cast<size_t>(7); };
  const size_t n_i32 = 3 * static_cast<size_t>(ni) + cb.size() + 1;
  const size_t n_u32 = static_cast<size_t>(ni) + ct.size() + 1;
  const size_t o_u32 = up8(4 * n_i32), o_f64 = o_u32 + up8(4 * n_u32), o_i8 = o_f64 + 8 * static_cast<size_t>(nl);
  const size_t bytes = up8(o_i8 + std::max(1, ni));
  if (tree_blob_cap_ < bytes) {
    tree_blob_cap_ = std::max(bytes, 64 * static_cast<size_t>(config_->num_leaves) + 4096);
    d_tree_blob_ = Alloc<char>(tree_blob_cap_);
  }
  const int nbm = std::max(ni, config_->num_leaves);
  if (tree_bm_cap_ < nbm) {
    tree_bm_cap_ = nbm;
    d_tree_bm_ = Alloc<unsigned long long>(4 * static_cast<size_t>(nbm));
    d_tree_bm_meta_ = Alloc<int32_t>(3 * static_cast<size_t>(nbm));
  }
  StageSlot& sl = stage_slots_[stage_next_];
  stage_next_ = (stage_next_ + 1) % kStageSlots;
  if (sl.done != nullptr) HIPCHECK(hipEventSynchronize(sl.done));  // (its previous copy: long done)
  if (sl.cap < bytes) {
    if (sl.host != nullptr) HIPCHECK(hipHostFree(sl.host));
    sl.cap = std::max(bytes, tree_blob_cap_);
    HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&sl.host), sl.cap, hipHostMallocDefault));
  }
  if (sl.done == nullptr) HIPCHECK(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
  int32_t* hi = reinterpret_cast<int32_t*>(sl.host);
  uint32_t* hu = reinterpret_cast<uint32_t*>(sl.host + o_u32);
  double* hf = reinterpret_cast<double*>(sl.host + o_f64);
  int8_t* hb = reinterpret_cast<int8_t*>(sl.host + o_i8);
  for (int j = 0; j < ni; ++j) {
    hi[j] = tree->split_feature_inner(j);
    hi[ni + j] = tree->left_child(j);
    hi[2 * ni + j] = tree->right_child(j);
    hu[j] = tree->threshold_in_bin(j);
    hb[j] = tree->decision_type(j);
  }
  for (size_t j = 0; j < cb.size(); ++j) hi[3 * ni + j] = cb[j];
  for (size_t j = 0; j < ct.size(); ++j) hu[ni + j] = ct[j];
  for (int j = 0; j < nl; ++j) hf[j] = tree->LeafOutput(j);
  HIPCHECK(hipMemcpyAsync(d_tree_blob_, sl.host, bytes, hipMemcpyHostToDevice, stream_));
  HIPCHECK(hipEventRecord(sl.done, stream_));
  const int32_t* di = reinterpret_cast<const int32_t*>(d_tree_blob_);
  dev::DevTree t{};
  t.num_leaves = nl;
  t.split_feature_inner = di;
  t.left_child = di + ni;
  t.right_child = di + 2 * ni;
  t.cat_boundaries_inner = di + 3 * ni;
  t.threshold_in_bin = reinterpret_cast<const uint32_t*>(d_tree_blob_ + o_u32);
  t.cat_threshold_inner = t.threshold_in_bin + ni;
  t.decision_type = reinterpret_cast<const int8_t*>(d_tree_blob_ + o_i8);
  t.leaf_value = reinterpret_cast<const double*>(d_tree_blob_ + o_f64);
  t.bm_work = d_tree_bm_;
  t.bm_meta = d_tree_bm_meta_;
  return t;
}

void GPUTreeLearner::AddTreeToScore(const Tree* tree, int k) {
  grad_prefetched_ = false;
  // NOTE: called from AddTrainedTreeToScore for out-of-bag rows only (oob_cnt_ > 0 and the
  // tree just trained), otherwise for every row
  double* score = d_score_ + static_cast<size_t>(k) * num_data_;
  if (tree->num_leaves() <= 1) {
    AddConstToScore(tree->LeafOutput(0), k);
    return;
  }
  dev::DevTree t = StageTree(tree);
  const bool oob_only = oob_cnt_ > 0 && in_trained_update_;
  if (oob_only) {
    dev::AddTreeScore(args_, t, d_oob_, oob_cnt_, score, stream_);
  } else {
    dev::AddTreeScore(args_, t, nullptr, num_data_, score, stream_);
  }
}

// LGBM_AMD_FUSE_GRAD=0: the score walk does not compute the next gradients
bool GPUTreeLearner::FuseNextGradients() {
  const char* e = tuning::Get(tuning::Knob::FuseGrad);
  return !(e != nullptr && e[0] == '0');
}

bool GPUTreeLearner::SameGradArgs(const dev::GradArgs& x, const dev::GradArgs& y) {
  return x.kind == y.kind && x.num_class == y.num_class && x.num_data == y.num_data && x.p0 == y.p0 && x.p1 == y.p1 &&
         x.p2 == y.p2 && x.lw0 == y.lw0 && x.lw1 == y.lw1 && x.label == y.label && x.weights == y.weights &&
         x.label_weight == y.label_weight && x.score == y.score && x.gh == y.gh && x.gh_stride == y.gh_stride &&
         x.max_parts == y.max_parts && x.root_parts == y.root_parts;
}

bool GPUTreeLearner::ComputeGradients(const DeviceGradSpec& spec, int ntpi) {
  if (spec.kind == DeviceGradKind::None || spec.kind == DeviceGradKind::MulticlassOVA) return false;
  if (spec.kind != DeviceGradKind::MulticlassSoftmax && ntpi != 1) return false;
  if (spec.label == nullptr) return false;
  const bool listwise = spec.kind == DeviceGradKind::Lambdarank || spec.kind == DeviceGradKind::RankXendcg;
  if (listwise && spec.rank.query_boundaries == nullptr) return false;
  const size_t n = static_cast<size_t>(num_data_);
  const bool prefetched = grad_prefetched_;
  grad_prefetched_ = false;
  grad_from_prefetch_ = false;
  bool uploaded = false;
  if (uploaded_label_src_ != spec.label) {
    if (d_label_ == nullptr) d_label_ = Alloc<float>(n);
    HIPCHECK(hipMemcpy(d_label_, spec.label, sizeof(float) * n, hipMemcpyHostToDevice));
    uploaded_label_src_ = spec.label;
    uploaded = true;
  }
  if (spec.weights != nullptr && uploaded_weight_src_ != spec.weights) {
    if (d_weights_ == nullptr) d_weights_ = Alloc<float>(n);
    HIPCHECK(hipMemcpy(d_weights_, spec.weights, sizeof(float) * n, hipMemcpyHostToDevice));
    uploaded_weight_src_ = spec.weights;
    uploaded = true;
  }
  if (spec.label_weight_arr != nullptr && uploaded_lw_src_ != spec.label_weight_arr) {
    if (d_label_weight_ == nullptr) d_label_weight_ = Alloc<float>(n);
    HIPCHECK(hipMemcpy(d_label_weight_, spec.label_weight_arr, sizeof(float) * n, hipMemcpyHostToDevice));
    uploaded_lw_src_ = spec.label_weight_arr;
    uploaded = true;
  }
  last_grad_fusable_ = false;
  if (listwise) {
    UploadRankTables(spec.rank, spec.kind);
    dev::RankArgs ra{};
    ra.kind = spec.kind == DeviceGradKind::Lambdarank ? dev::kRankKindLambdarank : dev::kRankKindXendcg;
    ra.num_queries = spec.rank.num_queries;
    ra.qb = d_qb_;
    ra.label = d_label_;
    ra.weights = spec.weights != nullptr ? d_weights_ : nullptr;
    ra.score = d_score_;
    ra.grad = d_grad_;
    ra.hess = d_hess_;
    ra.inv_max_dcg = d_inv_max_dcg_;
    ra.label_gain = d_label_gain_;
    ra.discount = d_discount_;
    ra.sigmoid = spec.rank.sigmoid;
    ra.sig_min = spec.rank.sig_min;
    ra.sig_max = spec.rank.sig_max;
    ra.sig_factor = spec.rank.sig_factor;
    ra.sig_table = d_sig_table_;
    ra.big_q = d_rank_big_q_;
    ra.num_big = rank_num_big_;
    ra.big_d0 = d_rank_big_d0_;
    ra.big_d1 = d_rank_big_d1_;
    ra.big_dh = d_rank_big_dh_;
    ra.max_docs = rank_max_docs_;
    ra.pair_buf = d_rank_pairs_;
    ra.pair_off = d_rank_pair_off_;
    ra.big_f = d_rank_big_f_;
    ra.big_i0 = d_rank_big_i0_;
    ra.big_i1 = d_rank_big_i1_;
    ra.big_i2 = d_rank_big_i2_;
    ra.norm = spec.rank.norm ? 1 : 0;
    ra.rng = d_rank_rng_;
    dev::RankGradients(ra, stream_);
    HIPCHECK(hipGetLastError());  // (a failed launch would leave last iteration's gradients)
    gh_fresh_ = false;
    split_stale_ = false;
    last_grad_fusable_ = false;
    return true;
  }
  dev::GradArgs g{};
  tuning::PoisonArgs(&g);  // (every field set below)
  g.kind = static_cast<int32_t>(spec.kind);
  g.num_class = spec.kind == DeviceGradKind::MulticlassSoftmax ? ntpi : 1;
  g.num_data = num_data_;
  g.p0 = spec.p0;
  g.p1 = spec.p1;
  g.p2 = spec.p2;
  g.lw0 = spec.label_weight[0];
  g.lw1 = spec.label_weight[1];
  g.label = d_label_;
  g.weights = spec.weights != nullptr ? d_weights_ : nullptr;
  g.label_weight = spec.label_weight_arr != nullptr ? d_label_weight_ : nullptr;
  g.score = d_score_;
  g.grad = d_grad_;
  g.hess = d_hess_;
  g.write_split = 1;
  g.gh = nullptr;
  g.gh_stride = args_.gh_stride;
  g.max_parts = nullptr;
  g.root_parts = nullptr;
  const bool fuse = ntpi == 1 && spec.kind != DeviceGradKind::MulticlassSoftmax;
  if (fuse) {
    g.gh = d_gh_;
    g.max_parts = d_max_parts_;
    g.root_parts = d_root_parts_;
    g.write_split = 0;
    // the last score walk already computed these gradients from the current scores
    // (AddTrainedTreeToScore), unless anything changed the scores or inputs since
    if (prefetched && !uploaded && SameGradArgs(g, last_grad_)) {
      gh_fresh_ = true;
      split_stale_ = true;
      last_grad_fusable_ = true;
      grad_from_prefetch_ = true;
      return true;
    }
  }
  grad_from_prefetch_ = false;
  dev::Gradients(g, stream_);
  gh_fresh_ = fuse;
  split_stale_ = fuse;
  grad_parts_ = dev::GradientBlocks(num_data_);
  if (fuse) {
    last_grad_ = g;
    last_grad_fusable_ = true;
  }
  return true;
}

// query boundaries, 1 / max DCG, label gains and position discounts (lambdarank) or the
// per-query generators (xendcg; from here on they advance on the device)
void GPUTreeLearner::UploadRankTables(const DeviceRankSpec& r, DeviceGradKind kind) {
  if (uploaded_qb_src_ == r.query_boundaries) return;
  const size_t nq = static_cast<size_t>(r.num_queries);
  d_qb_ = Alloc<int32_t>(nq + 1);
  HIPCHECK(hipMemcpy(d_qb_, r.query_boundaries, sizeof(int32_t) * (nq + 1), hipMemcpyHostToDevice));
  if (kind == DeviceGradKind::Lambdarank) {
    d_inv_max_dcg_ = Alloc<double>(nq);
    HIPCHECK(hipMemcpy(d_inv_max_dcg_, r.inv_max_dcg, sizeof(double) * nq, hipMemcpyHostToDevice));
    d_label_gain_ = Alloc<double>(r.num_label_gain);
    HIPCHECK(hipMemcpy(d_label_gain_, r.label_gain, sizeof(double) * r.num_label_gain, hipMemcpyHostToDevice));
    std::vector<double> disc(std::max<data_size_t>(1, r.max_query_docs));
    for (size_t i = 0; i < disc.size(); ++i) disc[i] = DCG::Discount(static_cast<data_size_t>(i));
    d_discount_ = Alloc<double>(disc.size());
    HIPCHECK(hipMemcpy(d_discount_, disc.data(), sizeof(double) * disc.size(), hipMemcpyHostToDevice));
    if (r.sig_table == nullptr || r.sig_bins != dev::kRankSigmoidBins) {
      Log::Fatal("device lambdarank: the objective's sigmoid table (%lld entries) is not the device's (%d)",
                 static_cast<long long>(r.sig_bins), dev::kRankSigmoidBins);
    }
    d_sig_table_ = Alloc<double>(static_cast<size_t>(r.sig_bins));
    HIPCHECK(hipMemcpy(d_sig_table_, r.sig_table, sizeof(double) * r.sig_bins, hipMemcpyHostToDevice));
  } else {
    d_rank_rng_ = Alloc<uint32_t>(nq);
    HIPCHECK(hipMemcpy(d_rank_rng_, r.rng_states, sizeof(uint32_t) * nq, hipMemcpyHostToDevice));
  }
  // queries longer than the LDS staging: one 1024-thread workgroup each over a global scratch;
  // the others' LDS is sized to the longest of them.  Lambdarank: the pair scratch of every
  // LDS-staged query (cnt^2 float pairs each), within a memory budget
  std::vector<int32_t> big;
  std::vector<int64_t> pair_off(nq, 0);
  int64_t pair_total = 0;
  rank_max_docs_ = 1;
  for (size_t q = 0; q < nq; ++q) {
    const int64_t cnt = r.query_boundaries[q + 1] - r.query_boundaries[q];
    if (cnt > dev::kRankMaxDocs) {
      big.push_back(static_cast<int32_t>(q));
      continue;
    }
    rank_max_docs_ = std::max<int32_t>(rank_max_docs_, static_cast<int32_t>(cnt));
    pair_off[q] = pair_total;
    pair_total += cnt * cnt;
  }
  d_rank_pairs_ = nullptr;
  d_rank_pair_off_ = nullptr;
  // budget: a share of the free memory (the histograms and round buffers are already resident),
  // capped; LGBM_AMD_RANK_PAIR_MB overrides it
  int64_t pair_budget = int64_t{tuning::kRankPairCapMb} << 20;
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
    pair_budget = std::min<int64_t>(pair_budget, static_cast<int64_t>(tuning::kRankPairFreeShare * free_b));
  } else {
    (void)hipGetLastError();
  }
  pair_budget = static_cast<int64_t>(tuning::Int(tuning::Knob::RankPairMb, static_cast<int>(pair_budget >> 20))) << 20;
  const int64_t pair_bytes = pair_total * static_cast<int64_t>(sizeof(float2));
  if (kind == DeviceGradKind::Lambdarank && pair_total > 0 && pair_bytes > pair_budget) {
    Log::Info("device lambdarank: pair scratch of %.1f MiB is over its %.1f MiB budget; each pair is evaluated "
              "from both of its documents", pair_bytes / 1048576.0, pair_budget / 1048576.0);
  }
  if (kind == DeviceGradKind::Lambdarank && pair_total > 0 && pair_bytes <= pair_budget) {
    d_rank_pairs_ = Alloc<float2>(static_cast<size_t>(pair_total));
    d_rank_pair_off_ = Alloc<int64_t>(nq);
    HIPCHECK(hipMemcpy(d_rank_pair_off_, pair_off.data(), sizeof(int64_t) * nq, hipMemcpyHostToDevice));
  }
  rank_num_big_ = static_cast<int32_t>(big.size());
  d_rank_big_q_ = nullptr;
  d_rank_big_d0_ = d_rank_big_d1_ = d_rank_big_dh_ = nullptr;
  d_rank_big_f_ = nullptr;
  d_rank_big_i0_ = d_rank_big_i1_ = d_rank_big_i2_ = nullptr;
  if (!big.empty()) {
    const size_t n = static_cast<size_t>(num_data_);
    d_rank_big_q_ = Alloc<int32_t>(big.size());
    HIPCHECK(hipMemcpy(d_rank_big_q_, big.data(), sizeof(int32_t) * big.size(), hipMemcpyHostToDevice));
    d_rank_big_d0_ = Alloc<double>(n);
    d_rank_big_d1_ = Alloc<double>(n);
    d_rank_big_dh_ = Alloc<double>(n);
    d_rank_big_f_ = Alloc<float>(n);
    d_rank_big_i0_ = Alloc<int32_t>(n);
    d_rank_big_i1_ = Alloc<int32_t>(n);
    d_rank_big_i2_ = Alloc<int32_t>(n);
    Log::Debug("device %s: %d queries of more than %d documents in global scratch",
               kind == DeviceGradKind::Lambdarank ? "lambdarank" : "rank_xendcg", rank_num_big_, dev::kRankMaxDocs);
  }
  uploaded_qb_src_ = r.query_boundaries;
}

data_size_t GPUTreeLearner::DeviceSample(const DeviceSampleSpec& sp) {
  HIPCHECK(hipSetDevice(device_id_));
  const int64_t nb = dev::SampleBlocks(num_data_);
  if (d_sample_rng_ == nullptr) {
    d_sample_rng_ = Alloc<uint32_t>(nb);
    d_sample_codes_ = Alloc<uint8_t>(num_data_);
    d_sample_cnt_ = Alloc<int32_t>(nb);
    d_sample_off_ = Alloc<int32_t>(nb);
  }
  if (sp.reset || !sample_seeded_) {
    // generator of block b: Random(seed + b) (reference bagging_rands_)
    std::vector<uint32_t> st(nb);
    for (int64_t b = 0; b < nb; ++b) st[b] = static_cast<uint32_t>(sp.seed + static_cast<int>(b));
    HIPCHECK(hipMemcpy(d_sample_rng_, st.data(), sizeof(uint32_t) * nb, hipMemcpyHostToDevice));
    sample_seeded_ = true;
  }
  if (sp.balanced && uploaded_label_src_ != sp.label) {
    if (d_label_ == nullptr) d_label_ = Alloc<float>(num_data_);
    HIPCHECK(hipMemcpy(d_label_, sp.label, sizeof(float) * num_data_, hipMemcpyHostToDevice));
    uploaded_label_src_ = sp.label;
  }
  if (sp.goss) MaterializeSplitGradients();  // (GOSS reads and rescales grad / hess)
  dev::SampleArgs s{};
  tuning::PoisonArgs(&s);
  s.num_data = num_data_;
  s.num_blocks = nb;
  s.goss = sp.goss ? 1 : 0;
  s.balanced = sp.balanced ? 1 : 0;
  s.num_class = sp.num_tree_per_iteration;
  s.fraction = sp.fraction;
  s.pos_fraction = sp.pos_fraction;
  s.neg_fraction = sp.neg_fraction;
  s.top_rate = sp.top_rate;
  s.other_rate = sp.other_rate;
  s.label = d_label_;
  s.grad = d_grad_;
  s.hess = d_hess_;
  s.rng = d_sample_rng_;
  s.codes = d_sample_codes_;
  s.block_cnt = d_sample_cnt_;
  s.block_off = d_sample_off_;
  s.bag = d_bag_;
  s.oob = d_oob_;
  s.bag_count = d_bag_count_;
  dev::SampleRows(s, stream_);
  int32_t cnt = 0;
  HIPCHECK(hipMemcpyAsync(&cnt, d_bag_count_, sizeof(int32_t), hipMemcpyDeviceToHost, stream_));
  HIPCHECK(hipStreamSynchronize(stream_));
  if (sp.goss) gh_fresh_ = false;  // the sampled rows' gradients were rescaled in place
  // SerialTreeLearner::SetBaggingData state; the rows themselves stay on the device
  bag_indices_ = nullptr;
  bag_cnt_ = cnt;
  use_bag_ = cnt < num_data_;
  oob_cnt_ = num_data_ - cnt;
  if (sp.host_indices != nullptr) {
    sp.host_indices->resize(num_data_);
    HIPCHECK(hipMemcpy(sp.host_indices->data(), d_bag_, sizeof(int32_t) * cnt, hipMemcpyDeviceToHost));
    if (oob_cnt_ > 0) {
      HIPCHECK(hipMemcpy(sp.host_indices->data() + cnt, d_oob_, sizeof(int32_t) * oob_cnt_, hipMemcpyDeviceToHost));
    }
    bag_indices_ = sp.host_indices->data();
  }
  return cnt;
}

void GPUTreeLearner::UploadGradients(const score_t* g, const score_t* h, int64_t n) {
  gh_fresh_ = false;
  split_stale_ = false;
  last_grad_fusable_ = false;
  grad_prefetched_ = false;
  HIPCHECK(hipMemcpyAsync(d_grad_, g, sizeof(float) * n, hipMemcpyHostToDevice, stream_));
  HIPCHECK(hipMemcpyAsync(d_hess_, h, sizeof(float) * n, hipMemcpyHostToDevice, stream_));
  HIPCHECK(hipStreamSynchronize(stream_));
}

void GPUTreeLearner::DownloadGradients(score_t* g, score_t* h, int64_t n) {
  MaterializeSplitGradients();
  HIPCHECK(hipMemcpyAsync(g, d_grad_, sizeof(float) * n, hipMemcpyDeviceToHost, stream_));
  HIPCHECK(hipMemcpyAsync(h, d_hess_, sizeof(float) * n, hipMemcpyDeviceToHost, stream_));
  HIPCHECK(hipStreamSynchronize(stream_));
}

void GPUTreeLearner::Synchronize() { HIPCHECK(hipStreamSynchronize(stream_)); }

}  // namespace lgbm_amd
