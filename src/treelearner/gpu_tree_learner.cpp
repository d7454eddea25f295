// MI355X tree learner host orchestration (see gpu_tree_learner.h).
#include "gpu_learner_internal.h"
#include "lgbm_amd/tuning.h"

namespace lgbm_amd {

namespace {

int PickDevice(const Config* cfg) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
    Log::Fatal("device_type=gpu requested but no HIP device is visible");
  }
  if (cfg->gpu_device_id >= 0) return cfg->gpu_device_id % count;
  const char* lr = std::getenv("LOCAL_RANK");
  if (lr != nullptr) return std::atoi(lr) % count;
  return 0;
}

}  // namespace

TreeLearner* CreateDeviceTreeLearner(const std::string& learner_type, const Config* config) {
  if (learner_type == "serial") return new GPUTreeLearner(config, GPUTreeLearner::Mode::kSerial);
  if (learner_type == "data") return new GPUTreeLearner(config, GPUTreeLearner::Mode::kData);
  if (learner_type == "feature") return new GPUTreeLearner(config, GPUTreeLearner::Mode::kFeature);
  if (learner_type == "voting") return new VotingParallelTreeLearner<GPUTreeLearner>(config);
  Log::Fatal("Unknown tree learner type %s", learner_type.c_str());
  return nullptr;
}

// fx64 (two int64 words per bin, 31-bit rows) or fx32 (one packed word, ~16 bits below max |g|
// per row): gpu_use_dp or gpu_hist_precision=fx64 force fx64; auto picks it for the listwise
// objectives, whose gradients span orders of magnitude across queries (the fx32 quantum of one
// query's max |g| erases another's small lambdas: config #4 NDCG@10 0.7911 fx32, 0.7927 fx64,
// CPU learner 0.7955, profiles/r03_v6_ltr_ndcg_parity.md)
bool GPUTreeLearner::WideHistograms(const Config& c) {
  if (c.gpu_use_dp || c.gpu_hist_precision == "fx64") return true;
  if (c.gpu_hist_precision == "fx32") return false;
  if (c.gpu_hist_precision != "auto") Log::Fatal("gpu_hist_precision must be auto, fx32 or fx64, got %s", c.gpu_hist_precision.c_str());
  return c.objective == "lambdarank" || c.objective == "rank_xendcg";
}

GPUTreeLearner::GPUTreeLearner(const Config* config, Mode mode) : SerialTreeLearner(config), mode_(mode) {}

GPUTreeLearner::~GPUTreeLearner() {
  if (spec_live_ && stream_ != nullptr) (void)hipStreamSynchronize(stream_);  // (a launched next tree)
  spec_live_ = false;
  FreeAll();
  for (void* p : valid_allocs_) (void)hipFree(p);
}

void GPUTreeLearner::FreeBuffers() {
  DestroyGraph();
  for (void* p : allocs_) (void)hipFree(p);
  allocs_.clear();
  for (void** hp : {reinterpret_cast<void**>(&h_mask_), reinterpret_cast<void**>(&h_rec_),
                    reinterpret_cast<void**>(&h_step_), reinterpret_cast<void**>(&h_root_),
                    reinterpret_cast<void**>(&h_absmax_), reinterpret_cast<void**>(&h_scales_),
                    reinterpret_cast<void**>(&h_round_), reinterpret_cast<void**>(&h_tree_out_)}) {
    if (*hp) (void)hipHostFree(*hp);
    *hp = nullptr;
  }
  d_score_ = nullptr;
  d_grad_ = d_hess_ = nullptr;
  d_label_ = d_weights_ = d_label_weight_ = nullptr;
  uploaded_label_src_ = uploaded_weight_src_ = uploaded_lw_src_ = nullptr;
  d_qb_ = nullptr;
  d_inv_max_dcg_ = d_label_gain_ = d_discount_ = d_sig_table_ = nullptr;
  d_rank_big_q_ = nullptr;
  rank_num_big_ = 0;
  d_rank_big_d0_ = d_rank_big_d1_ = d_rank_big_dh_ = nullptr;
  d_rank_pairs_ = nullptr;
  d_rank_pair_off_ = nullptr;
  rank_max_docs_ = 0;
  d_rank_big_f_ = nullptr;
  d_rank_big_i0_ = d_rank_big_i1_ = d_rank_big_i2_ = nullptr;
  d_rank_rng_ = nullptr;
  uploaded_qb_src_ = nullptr;
  d_sample_rng_ = nullptr;
  d_sample_codes_ = nullptr;
  d_sample_cnt_ = d_sample_off_ = d_bag_count_ = nullptr;
  sample_seeded_ = false;
  d_tree_blob_ = nullptr;
  tree_blob_cap_ = 0;
  d_early_blob_ = nullptr;
  early_scored_leaves_ = 0;
  d_tree_bm_ = nullptr;
  d_tree_bm_meta_ = nullptr;
  tree_bm_cap_ = 0;
  for (StageSlot& sl : stage_slots_) {
    if (sl.done != nullptr) {
      (void)hipEventSynchronize(sl.done);
      (void)hipEventDestroy(sl.done);
    }
    if (sl.host != nullptr) (void)hipHostFree(sl.host);
    sl = StageSlot();
  }
}

void GPUTreeLearner::FreeAll() {
  FreeBuffers();
  if (rec_event_ != nullptr) (void)hipEventDestroy(rec_event_);
  rec_event_ = nullptr;
  if (stream_) (void)hipStreamDestroy(stream_);
  stream_ = nullptr;
}

void GPUTreeLearner::Init(const Dataset* train_data, bool is_constant_hessian) {
  SerialTreeLearner::Init(train_data, is_constant_hessian);
  if (config_->num_leaves > dev::kMaxLeaves) {
    Log::Fatal("device learner supports num_leaves <= %d", dev::kMaxLeaves);
  }
  device_id_ = PickDevice(config_);
  world_ = Network::num_machines();
  rank_ = Network::rank();
  distributed_ = mode_ != Mode::kSerial && world_ > 1;
  data_parallel_ = mode_ == Mode::kData && world_ > 1;
  voting_ = mode_ == Mode::kVoting && world_ > 1;
  // device-side waits of the collectives are bounded like the reference's socket linker: by
  // time_out minutes (rank skew between trees -- evaluation, checkpoints, logging on one rank
  // -- is not an error)
  if (distributed_ && Network::device_comm() != nullptr) {
    Network::device_comm()->SetWaitLimit(60.0 * std::max(1, config_->time_out));
  }
  HIPCHECK(hipSetDevice(device_id_));
  int cus = 0;
  HIPCHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device_id_));
  dev::SetNumCUs(cus);
  dev::PrepareKernels();
  HIPCHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  UploadData();
  global_count_.assign(config_->num_leaves, 0);
  const char* layout = sparse_rows_ ? "row-sparse"
                       : nibbles_ ? "4-bit" : (args_.bin_bytes == 1 ? "8-bit" : (args_.bin_bytes == 2 ? "16-bit" : "8/16-bit"));
  Log::Info("MI355X learner on device %d (%d CUs): %d rows, %d groups, %d histogram bins, %s rows, %d hist tiles",
            device_id_, cus, num_data_, num_groups_, total_bins_, layout, args_.hist_tiles);
}

void GPUTreeLearner::UploadData() {
  num_groups_ = data_->num_groups();
  total_bins_ = static_cast<int>(data_->num_total_bin());
  int max_group_bins = 0;
  for (int g = 0; g < num_groups_; ++g) max_group_bins = std::max(max_group_bins, data_->group(g).num_total_bin);
  if (max_group_bins > 65536) Log::Fatal("device learner: a feature group has more than 65536 bins");
  // row layout: groups in order, 8-bit groups four to a 32-bit word, 16-bit groups (more than
  // 256 bins) two to a word; a group of the other width starts a new word.  One wide group no
  // longer widens every column (LGBM_AMD_UNIFORM_BINS=1: the uniform layout, for A/B runs)
  const bool uniform = tuning::Get(tuning::Knob::UniformBins) != nullptr && tuning::Get(tuning::Knob::UniformBins)[0] == '1';
  h_gwide_.assign(num_groups_, 0);
  h_gbyte_.assign(num_groups_, 0);
  h_word_of_group_.assign(num_groups_, 0);
  h_word_g0_.clear();
  h_word_wide_.clear();
  int n_wide = 0;
  for (int g = 0; g < num_groups_; ++g) {
    h_gwide_[g] = (data_->group(g).num_total_bin > 256 || (uniform && max_group_bins > 256)) ? 1 : 0;
    n_wide += h_gwide_[g];
  }
  // 4-bit storage (the reference's DenseBin<uint8_t, true>, dense_bin.hpp IS_4BIT): when every
  // group has at most 16 bins, eight groups share a word -- half the bytes of the matrix and
  // of each gathered row.  The histogram gather is bound by its LDS atomics (one per row and
  // group either way), so bytes are as fast or faster (Higgs 10M x 28, max_bin 15: 2.06 vs
  // 2.02 ms/iter, profiles/r03_v5_four_bit_ab.md): 4-bit rows are chosen when the 8-bit matrix
  // would take more than 32 GiB of HBM, or by LGBM_AMD_NIBBLE_BINS=1 (=0: never).
  const bool can_nib = n_wide == 0 && max_group_bins <= 16 && !uniform;
  const size_t byte_matrix = static_cast<size_t>(num_data_) * 4 * static_cast<size_t>((num_groups_ + 3) / 4);
  nibbles_ = can_nib && byte_matrix > (size_t(32) << 30);
  if (const char* e = tuning::Get(tuning::Knob::NibbleBins)) nibbles_ = can_nib && e[0] == '1';
  h_gnib_.assign(num_groups_, 0);
  int slot = 0;
  for (int g = 0; g < num_groups_; ++g) {
    const int wide = h_gwide_[g], per = nibbles_ ? 8 : (wide ? 2 : 4);
    if (h_word_g0_.empty() || h_word_wide_.back() != wide || slot == per) {
      h_word_g0_.push_back(g);
      h_word_wide_.push_back(static_cast<int8_t>(wide));
      slot = 0;
    }
    const int w = static_cast<int>(h_word_g0_.size()) - 1;
    h_word_of_group_[g] = w;
    h_gbyte_[g] = nibbles_ ? 4 * w + slot / 2 : 4 * w + slot * (wide ? 2 : 1);
    if (nibbles_) h_gnib_[g] = static_cast<int8_t>(2 + (slot & 1));
    ++slot;
  }
  if (h_word_g0_.empty()) {
    h_word_g0_.push_back(0);
    h_word_wide_.push_back(0);
  }
  const int wpr = static_cast<int>(h_word_g0_.size());
  h_word_g0_.push_back(num_groups_);  // sentinel
  const int bin_bytes = n_wide == 0 ? 1 : (n_wide == num_groups_ ? 2 : 0);
  const size_t row_bytes = static_cast<size_t>(wpr) * 4;
  d_word_g0_ = Alloc<int32_t>(h_word_g0_.size());
  HIPCHECK(hipMemcpy(d_word_g0_, h_word_g0_.data(), sizeof(int32_t) * h_word_g0_.size(), hipMemcpyHostToDevice));
  d_word_wide_ = Alloc<int8_t>(h_word_wide_.size());
  HIPCHECK(hipMemcpy(d_word_wide_, h_word_wide_.data(), h_word_wide_.size(), hipMemcpyHostToDevice));
  args_.bin_bytes = bin_bytes;
  args_.nibbles = nibbles_ ? 1 : 0;
  args_.words_per_row = wpr;
  args_.row_words = wpr;
  args_.gh_stride = 1;
  // training rows: the row-major word matrix, or row-sparse lists of stored bins (validation
  // sets always use the word layout)
  sparse_rows_ = UseSparseRows(wpr);
  d_sp_ptr_ = nullptr;
  d_sp_bin_ = nullptr;
  d_bins_ = nullptr;
  d_gh_ = nullptr;
  if (sparse_rows_) {
    UploadSparseRows();
  } else {
    // (g, h) interleaved at the end of each row, rows padded to 64 / 128 B (or 32-B multiples
    // when wider): a gathered row of the histogrammed child is then one cache line, where a
    // 28-B bins row straddling lines plus a separate 8-B (g, h) line took ~2.2 lines
    // (LGBM_AMD_GH_IN_ROWS=0: separate compact (g, h) array)
    int row_words = wpr + 2;
    row_words = row_words <= 16 ? 16 : (row_words <= 32 ? 32 : (row_words + 7) / 8 * 8);
    // A/B on the headline 10M x 28 (7 bin words -> 64-B rows): 2.52 ms/iter separate, 2.71
    // interleaved -- off by default
    bool gh_rows = false;
    if (const char* e = tuning::Get(tuning::Knob::GhInRows)) gh_rows = e[0] == '1';
    if (gh_rows) {
      args_.row_words = row_words;
      args_.gh_stride = row_words / 2;
    }
    // LGBM_AMD_ROW_ALIGN_WORDS=n: row stride rounded up to n words (A/B: 8 -> 32-B rows that
    // never straddle a 64-B line, at 8/7 of the matrix bytes on the headline shape)
    if (const char* e = tuning::Get(tuning::Knob::RowAlignWords)) {
      const int al = std::max(1, std::atoi(e));
      if (!gh_rows) args_.row_words = (wpr + al - 1) / al * al;
    }
    std::vector<uint8_t> host = RowMajorBins(data_, args_.row_words);
    d_bins_ = Alloc<uint8_t>(host.size());
    HIPCHECK(hipMemcpy(d_bins_, host.data(), host.size(), hipMemcpyHostToDevice));
    if (gh_rows) d_gh_ = reinterpret_cast<dev::GH*>(static_cast<uint8_t*>(d_bins_) + 4 * static_cast<size_t>(row_words - 2));
  }
  // column-major copy for the partition kernels (one byte / short per row of the split column):
  // ~3% faster trees on the headline shape (profiles/r02_column_copy_ab.txt), at the price of a
  // second copy of the matrix -- kept when that copy is under 8 GiB (LGBM_AMD_COLUMN_COPY=0/1
  // forces it off / on); without it the partition reads the row-major matrix
  d_bins_col_ = nullptr;
  std::vector<int64_t> col_off(num_groups_ + 1, 0);
  for (int g = 0; g < num_groups_; ++g) col_off[g + 1] = col_off[g] + static_cast<int64_t>(num_data_) * (h_gwide_[g] ? 2 : 1);
  const size_t col_bytes = static_cast<size_t>(col_off[num_groups_]);
  bool col_copy = col_bytes <= (size_t(8) << 30);
  if (const char* cc = tuning::Get(tuning::Knob::ColumnCopy)) col_copy = cc[0] == '1';
  col_copy = col_copy || sparse_rows_;  // (the partition's only source of the split column)
  if (col_copy) {
    std::vector<uint8_t> col(std::max<size_t>(1, col_bytes));
#pragma omp parallel for schedule(static)
    for (int g = 0; g < num_groups_; ++g) {
      const FeatureGroup& grp = data_->group(g);
      uint8_t* dst = col.data() + col_off[g];
      if (grp.sparse) {  // (zero-filled column: the stored rows only)
        grp.ForEachStored(num_data_, [&](data_size_t r, uint32_t v) {
          if (!h_gwide_[g]) dst[r] = static_cast<uint8_t>(v);
          else reinterpret_cast<uint16_t*>(dst)[r] = static_cast<uint16_t>(v);
        });
      } else if (!h_gwide_[g] && grp.bin_bytes == 1) {
        std::memcpy(dst, grp.data.data(), static_cast<size_t>(num_data_));
      } else {
        for (data_size_t r = 0; r < num_data_; ++r) {
          const uint32_t v = grp.Get(r);
          if (!h_gwide_[g]) dst[r] = static_cast<uint8_t>(v);
          else reinterpret_cast<uint16_t*>(dst)[r] = static_cast<uint16_t>(v);
        }
      }
    }
    d_bins_col_ = Alloc<uint8_t>(col.size());
    HIPCHECK(hipMemcpy(d_bins_col_, col.data(), col.size(), hipMemcpyHostToDevice));
  }
  // features
  std::vector<dev::Feature> feats(num_features_);
  for (int f = 0; f < num_features_; ++f) {
    const BinMapper* m = data_->FeatureBinMapper(f);
    const int g = data_->Feature2Group(f), sub = data_->Feature2SubFeature(f);
    dev::Feature& F = feats[f];
    F.group = g;
    F.hist_offset = static_cast<int32_t>(data_->FeatureHistOffset(f));
    F.num_bin = m->num_bin();
    F.offset = m->GetMostFreqBin() == 0 ? 1 : 0;
    F.default_bin = static_cast<int32_t>(m->GetDefaultBin());
    F.mfb = static_cast<int32_t>(m->GetMostFreqBin());
    F.missing_type = m->missing_type() == MissingType::None ? 0 : (m->missing_type() == MissingType::Zero ? 1 : 2);
    F.is_cat = m->bin_type() == BinType::Categorical ? 1 : 0;
    F.sub_lo = static_cast<int32_t>(data_->group(g).bin_offsets[sub]);
    F.sub_hi = static_cast<int32_t>(data_->group(g).bin_offsets[sub + 1]);
    F.real_index = data_->RealFeatureIndex(f);
    F.monotone = meta_[f].monotone_type;
    F.gbyte = h_gbyte_[g];
    F.gwide = h_gnib_[g] != 0 ? h_gnib_[g] : h_gwide_[g];
    F.col_off = col_off[g];
    F.penalty = meta_[f].penalty;
  }
  d_feat_ = Alloc<dev::Feature>(num_features_);
  HIPCHECK(hipMemcpy(d_feat_, feats.data(), sizeof(dev::Feature) * num_features_, hipMemcpyHostToDevice));
  h_feats_ = feats;
  std::vector<int32_t> goff(std::max(1, num_groups_), 0);
  for (int g = 0; g < num_groups_; ++g) goff[g] = static_cast<int32_t>(data_->group_bin_boundary(g));
  d_group_off_ = Alloc<int32_t>(goff.size());
  HIPCHECK(hipMemcpy(d_group_off_, goff.data(), sizeof(int32_t) * goff.size(), hipMemcpyHostToDevice));
  // histogram column tiles: the split kernel's LDS is the tile histogram (8 or 16 bytes per
  // bin) plus its 16 KiB row list; <= 80 KiB keeps two 1024-thread workgroups per CU
  hist_units_ = WideHistograms(*config_) ? 2 : 1;
  auto tile_bins_for = [&](int tw) {
    int mx = 0;
    for (int w0 = 0; w0 < wpr; w0 += tw) {
      const int g0 = h_word_g0_[w0], g1 = h_word_g0_[std::min(wpr, w0 + tw)];
      if (g0 >= num_groups_) break;
      const int lo = goff[g0], hi = g1 < num_groups_ ? goff[g1] : total_bins_;
      mx = std::max(mx, hi - lo);
    }
    return mx;
  };
  // widest tile that fits: a workgroup reads whole rows (one cache line per gathered row,
  // and the row's (g, h) once) -- 1-word tiles re-gather (g, h) per tile and measured
  // ~40% slower on small leaves (profiles/r01_v2_*)
  int max_tw = 1 << 20;
  if (const char* e = tuning::Get(tuning::Knob::HistTileWords)) max_tw = std::max(1, std::atoi(e));
  int tile_words = sparse_rows_ ? 1 : 0;  // (row-sparse tiles are bin ranges, below)
  const std::vector<int> limits = hist_units_ == 1 ? std::vector<int>{8192, 16384} : std::vector<int>{8192};
  for (int limit : limits) {
    if (sparse_rows_) break;
    for (int tw = std::min({wpr, dev::kHistThreads, max_tw}); tw >= 1; --tw) {
      if (tile_bins_for(tw) <= limit) {
        tile_words = tw;
        break;
      }
    }
    if (tile_words > 0) break;
  }
  if (tile_words == 0) Log::Fatal("device learner: feature groups too wide for LDS histograms; reduce max_bin");
  num_cat_total_ = 0;
  for (const auto& F : feats) num_cat_total_ += F.is_cat ? 1 : 0;
  args_.tile_words = tile_words;
  SetupOwnership();
  const int n_leaves = config_->num_leaves;
  // round growth: up to round_k_ leaves expanded per round (LGBM_AMD_ROUND_K, 1 = one split per
  // step; distributed learners run rounds with a device communicator)
  // Without LGBM_AMD_ROUND_K the width adapts per tree (RunRounds): 8 while the last tree's
  // speculation was accepted (expansions <= splits + 2: early trees), else 6 (A/B at 300
  // iterations of the headline, profiles/r04_round_width.md: K=8 saves 2 rounds on the first
  // trees for 2 more expansions, later it adds 8-10 unaccepted ones; fixed K 6 / 8 / 10 =
  // 2.040 / 2.072 / 2.132 ms, window of 20 after 5: 2.148 / 2.075)
  // Below 4M rows per rank the width stays 8: a round there is latency-bound and the extra
  // speculation is nearly free (r04_round_width.md: 1.25M / 2.5M rows 0.929 / 1.106 ms fixed
  // vs 0.943 / 1.120 adaptive; Epsilon 8.28 vs 8.44 ms, Bosch / LTR shapes equal)
  // (the rows per rank are averaged over the ranks at the first tree, RunRounds: every rank
  // must plan with the same width)
  // Trees of 90 leaves or more run num_leaves / 10 expansions per round (at most 16), fixed:
  // at 255 leaves width 16 halves the rounds per tree (41 -> 23) and saves 11-22% per
  // iteration on every 255-leaf shape measured (config #2 at 255 / 63 / 15 bins, the five
  // config #3 workloads; the same trees); at 127 leaves width 12 beats 8 and 16 (2.73 vs 2.88
  // / 2.80 ms: profiles/r06_round_width_255.md)
  round_k_ = tuning::kRoundWidth;
  k_adapt_ = true;
  k_adapt_checked_ = false;
  if (n_leaves / tuning::kRoundLeavesPerWidth > tuning::kRoundWidth) {
    round_k_ = n_leaves / tuning::kRoundLeavesPerWidth;
    k_adapt_ = false;
  }
  if (const char* e = tuning::Get(tuning::Knob::RoundK)) {
    round_k_ = std::atoi(e);
    k_adapt_ = false;
  }
  round_k_ = std::max(1, std::min(dev::kMaxRoundExp, round_k_));
  // speculation below the leaves (LGBM_AMD_ROUND_VMAX levels, 0: leaves only): one index
  // buffer per level + 2 (device_types.h), bounded to 32 GiB of row indices
  round_vmax_ = dev::kMaxRoundVmax;
  if (const char* e = tuning::Get(tuning::Knob::RoundVmax)) round_vmax_ = std::atoi(e);
  round_vmax_ = std::max(0, std::min(dev::kMaxRoundVmax, round_vmax_));
  while (round_vmax_ > 0 && static_cast<double>(num_data_) * 4.0 * (round_vmax_ + 1) > 32.0 * (1ull << 30)) --round_vmax_;
  if (round_k_ <= 1) round_vmax_ = 0;
  SizeRoundPools(n_leaves);
  d_tree_mask_ = Alloc<int8_t>(num_features_);
  d_node_mask_ = Alloc<int8_t>(static_cast<size_t>(2 * n_leaves) * std::max(1, num_features_));
  h_node_mask_.clear();
  d_bynode_pool_ = Alloc<int32_t>(std::max(1, num_features_));
  d_bynode_scratch_ = Alloc<int32_t>(std::max(1, num_features_));
  d_bynode_rng_ = Alloc<uint32_t>(1);
  d_xt_base_ = Alloc<uint32_t>(std::max(1, num_features_));
  d_xt_cum_ = Alloc<int32_t>(static_cast<size_t>(n_leaves) * std::max(1, num_features_));
  AllocVoteXt(n_leaves);
  if (d_gh_ == nullptr) d_gh_ = Alloc<dev::GH>(num_data_);
  d_idx_ = Alloc<int32_t>(num_data_);
  d_tmp_ = Alloc<int32_t>(static_cast<size_t>(num_data_) * (round_vmax_ + 1));
  d_bag_ = Alloc<int32_t>(num_data_);
  d_oob_ = Alloc<int32_t>(num_data_);
  d_bag_count_ = Alloc<int32_t>(1);
  d_leaves_ = Alloc<dev::Leaf>(n_leaves);
  d_step_ = Alloc<dev::Step>(1);
  d_find_sub_ = Alloc<uint32_t>(static_cast<size_t>(dev::kFindSub) * dev::kFindSubStride);
  HIPCHECK(hipMemset(d_find_sub_, 0, sizeof(uint32_t) * dev::kFindSub * dev::kFindSubStride));
  d_rec_ = Alloc<dev::SplitRecord>(std::max(1, n_leaves - 1));
  d_best_ = Alloc<DeviceSplit>(n_leaves);
  d_hist_ = Alloc<long long>(static_cast<size_t>(hist_slots_) * 2 * total_bins_);
  // two step buffers (data-parallel: owner-major blocks padded to equal size); round growth:
  // two parities of round_k_ expansion buffers
  const int64_t scratch_stride =
      std::max<int64_t>(2 * static_cast<int64_t>(total_bins_), 2 * static_cast<int64_t>(world_) * rs_block_);
  d_scratch_ = Alloc<long long>(std::max<size_t>(2 * static_cast<size_t>(scratch_stride),
                                                 round_k_ > 1 ? 4 * static_cast<size_t>(round_k_) * total_bins_ : 0));
  d_scales_ = Alloc<double>(4);
  d_absmax_ = Alloc<uint32_t>(4);
  // per-feature results: [2][num_features], or rank-major [world][2][max_owned] (gathered)
  const size_t fb_slots = std::max<size_t>(2 * static_cast<size_t>(round_k_) * std::max(1, num_features_),
                                           2 * static_cast<size_t>(world_) * round_k_ * std::max(1, max_owned_));
  d_feat_best_ = Alloc<dev::FeatureBest>(fb_slots);
  d_feat_cat_ = Alloc<uint32_t>(fb_slots * kMaxCatWords);
  fb_slots_ = fb_slots;
  // row blocks: the root histogram runs on two workgroups per CU, a split step on one; a
  // packed (hist_units 1) row block holds at most kHistRowsCap rows, so the fixed-point
  // scale does not depend on the number of rows; wide blocks are unbounded
  root_grid_ = dev::HistGridBlocks();
  // a split step launches split_grid x hist_tiles workgroups of 1024 threads: about one per
  // CU in all, since the smaller leaves' blocks exit at once and their launches alone cost
  // tens of microseconds (Epsilon, 8 column tiles: 37.4 ms/iter at 256 x 8, 28.7 at 32 x 8;
  // Yahoo, 3 tiles: 20.8 at 256 x 3, 20.6 at 64 x 3 -- profiles/r02_v10_split_grid_wide.txt)
  // column tiles of the histogram kernels (row-sparse: bin ranges of 16384 packed / 8192 wide bins)
  const int sparse_tile_bins = hist_units_ == 1 ? 16384 : 8192;
  const int col_tiles = sparse_rows_ ? (total_bins_ + sparse_tile_bins - 1) / sparse_tile_bins
                                     : (wpr + tile_words - 1) / tile_words;
  split_grid_ = std::max(std::min(8, dev::HistGridBlocks() / 2), dev::HistGridBlocks() / 2 / std::max(1, col_tiles));
  if (const char* e = tuning::Get(tuning::Knob::SplitGrid)) split_grid_ = std::max(1, std::atoi(e));
  rows_cap_ = hist_units_ == 1 ? dev::kHistRowsCap : (1 << 30);
  if (const char* e = tuning::Get(tuning::Knob::HistRowsCap)) {
    if (hist_units_ == 1) rows_cap_ = std::max(dev::kHistMinRows, std::min(dev::kHistRowsCap, std::atoi(e)));
  }
  // rows per split row block, lower bound: 4096 for one column tile (headline 10M x 28), 2048
  // for 2-5 tiles (Bosch 16.7 -> 16.0), 1024 from 6 (the split kernel's grid shrinks with the tiles, so smaller
  // blocks keep its workgroups busy: Epsilon, 8 tiles, 4096/2048/1024 = 23.0/21.7/20.8 ms/iter;
  // profiles/r02_v11_blk_min_rows_wide.txt)
  blk_min_rows_ = col_tiles >= 6 ? 1024 : col_tiles > 1 ? 2048 : 4096;
  if (const char* e = tuning::Get(tuning::Knob::BlkMinRows)) blk_min_rows_ = std::max(256, std::atoi(e));
  int hist_blocks = std::max({1, dev::HistBlocksFor(num_data_, root_grid_, rows_cap_, dev::kHistMinRows),
                              dev::HistBlocksFor(num_data_, split_grid_, rows_cap_, blk_min_rows_)});
  if (round_k_ > 1) {
    // a round's blocks share one size: at most split_grid (or the rows at the headroom cap)
    // plus one partial block per expansion
    const int64_t capped = (static_cast<int64_t>(num_data_) + rows_cap_ - 1) / rows_cap_;
    int rg = 2 * split_grid_;
    if (const char* e = tuning::Get(tuning::Knob::RoundGrid)) rg = std::max(rg, std::atoi(e));
    // (k_round_plan: blocks <= rows / rows_cap + expansions + grid)
    hist_blocks = std::max<int>(hist_blocks, static_cast<int>(capped + rg + dev::kMaxRoundExp + 1));
  }
  d_partials_ = Alloc<unsigned long long>(static_cast<size_t>(hist_blocks) * total_bins_ * hist_units_);
  d_root_ = Alloc<double>(4);
  d_leaf_sums_ = Alloc<double>(4);
  d_root_blk_ = Alloc<double>(2 * static_cast<size_t>(dev::RootSumBlocks()));
  // (per-workgroup partials of the gradient kernel, the packing kernel or the score walk that
  // computes the next gradients)
  const int parts = std::max({dev::GradientBlocks(num_data_), dev::PackBlocks(num_data_),
                              dev::AddTreeScoreGradParts(num_data_)});
  d_root_parts_ = Alloc<double>(2 * static_cast<size_t>(parts));
  d_max_parts_ = Alloc<float>(2 * static_cast<size_t>(parts));
  d_leaf_values_ = Alloc<double>(n_leaves);
  // (fine-grained: k_tree_begin reads the mask the host wrote before each tree's launch)
  HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&h_mask_), std::max(1, num_features_), hipHostMallocCoherent));
  HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&h_rec_), sizeof(dev::SplitRecord) * std::max(1, n_leaves - 1),
                         hipHostMallocDefault));
  HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&h_step_), sizeof(dev::Step), hipHostMallocDefault));
  HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&h_root_), sizeof(double) * 4, hipHostMallocDefault));
  HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&h_absmax_), sizeof(uint32_t) * 4, hipHostMallocDefault));
  HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&h_scales_), sizeof(double) * 4, hipHostMallocDefault));

  dev::KArgs& a = args_;
  a.p.sp = params_;
  a.p.num_leaves = n_leaves;
  a.p.max_depth = config_->max_depth;
  a.p.num_features = num_features_;
  a.p.num_groups = num_groups_;
  a.p.row_stride = static_cast<int32_t>(row_bytes);
  a.p.total_bins = total_bins_;
  a.p.monotone_penalty = config_->monotone_penalty;
  a.p.data_parallel = (data_parallel_ || voting_) ? 1 : 0;  // global counts from the split estimates
  a.p.vote_phase = 0;
  a.p.vote_k = 0;
  a.p.cegb = 0;
  a.p.cegb_split = 0.0;
  a.cegb_coupled = nullptr;
  a.cegb_used = nullptr;
  a.cegb_mem = nullptr;
  a.cegb_mem_cat = nullptr;
  a.p.mono_inter = 0;
  a.mt_leaf_parent = nullptr;
  a.mt_node = nullptr;
  a.mt_in_sub = nullptr;
  a.mt_upd = nullptr;
  a.cegb_lazy = nullptr;
  a.cegb_paid = nullptr;
  a.cegb_paid_words = 0;
  a.cegb_cnt = nullptr;
  a.cegb_scratch = nullptr;
  a.cegb_snap = nullptr;
  a.p.world = world_;
  a.root_local = nullptr;
  a.vote_buf = nullptr;
  a.vote_rank = rank_;
  a.vote_list = nullptr;
  a.vote_hist = nullptr;
  a.bins = d_bins_;
  a.feat = d_feat_;
  a.group_off = d_group_off_;
  a.tree_mask = d_tree_mask_;
  a.node_mask = nullptr;
  a.bynode_pool = d_bynode_pool_;
  a.bynode_pool_n = 0;
  a.bynode_cnt = 0;
  a.bynode_rng = nullptr;
  a.bynode_scratch = d_bynode_scratch_;
  a.gh = d_gh_;
  a.idx = d_idx_;
  a.tmp = d_tmp_;
  a.buf_stride = num_data_;
  a.leaves = d_leaves_;
  a.st = d_step_;
  a.find_sub = d_find_sub_;
  a.rec = d_rec_;
  a.host_out = nullptr;
  a.best = d_best_;
  a.hist = d_hist_;
  a.scratch = d_scratch_;
  a.scratch_stride = scratch_stride;
  a.partials = d_partials_;
  a.hist_max_blocks = hist_blocks;
  a.hist_units = hist_units_;
  a.root_grid = root_grid_;
  a.split_grid = split_grid_;
  a.blk_min_rows = blk_min_rows_;
  a.hist_rows_cap = rows_cap_;
  a.pick_in_find = distributed_ ? 0 : 1;  // distributed: k_pick after the gather
  a.host_mode = 0;
  a.ktrace = nullptr;
  if (const char* kt = tuning::Get(tuning::Knob::Ktrace)) {  // (before the rest of the arguments)
    if (kt[0] == '1') {
      d_ktrace_ = Alloc<long long>(static_cast<size_t>(n_leaves) * dev::kTraceSlots);
      a.ktrace = d_ktrace_;
    }
  }
  a.root = d_root_;
  a.root_blk = d_root_blk_;
  a.num_rows = num_data_;
  a.num_rows_dev = nullptr;
  a.root_identity = 1;
  a.bin_bytes = bin_bytes;
  a.nibbles = nibbles_ ? 1 : 0;
  a.words_per_row = wpr;
  a.word_g0 = d_word_g0_;
  a.word_wide = d_word_wide_;
  a.tile_words = tile_words;
  a.hist_tiles = col_tiles;
  a.tile_w0 = 0;
  a.tile_w1 = wpr;
  a.feat_list = nullptr;
  a.num_scan = num_features_;
  a.fb_index = nullptr;
  a.fb_side = num_features_;
  a.rs_pos = nullptr;
  a.owned_hist = nullptr;
  a.owned_off = nullptr;
  a.owned_bin_lo = 0;
  a.tile_bins = tile_bins_for(tile_words);
  a.sp_ptr = d_sp_ptr_;
  a.sp_bin = d_sp_bin_;
  a.sp_team = sp_team_;
  if (sparse_rows_) {  // column tiles = bin ranges of at most 16384 (packed) / 8192 (wide) bins
    a.tile_bins = (total_bins_ + a.hist_tiles - 1) / a.hist_tiles;
    a.tile_w0 = 0;
    a.tile_w1 = a.hist_tiles;
  }
  a.range_begin = 0;
  a.scales = d_scales_;
  a.bins_col = d_bins_col_;
  a.num_data = num_data_;
  a.feat_best = d_feat_best_;
  a.feat_cat = d_feat_cat_;
  int max_fb = 1;
  for (const auto& F : feats) max_fb = std::max(max_fb, F.num_bin - F.offset);
  a.p.max_feature_bins = max_fb;
  // from this split on the tree's graph has no reduce kernel: smaller children are small
  // enough for the split scan to sum their partial histograms (LGBM_AMD_DIRECT_FROM_SPLIT)
  a.p.direct_from_split = 100;  // a reduce kernel for every step with > kReduceChunk blocks (r02 sweep)
  a.p.trace_repeat = tuning::Get(tuning::Knob::KtraceRepeat) != nullptr ? 1 : 0;
  if (const char* e = tuning::Get(tuning::Knob::DirectFromSplit)) a.p.direct_from_split = std::atoi(e);
  std::vector<int32_t> cats;
  for (int f = 0; f < num_features_; ++f) {
    if (feats[f].is_cat) cats.push_back(f);
  }
  a.p.has_cat = static_cast<int32_t>(cats.size());
  a.p.wide_cat = 0;
  for (int f : cats) a.p.wide_cat |= feats[f].num_bin > dev::kFindCatNarrow ? 1 : 0;
  d_cat_list_ = Alloc<int32_t>(std::max<size_t>(1, cats.size()));
  if (!cats.empty()) {
    HIPCHECK(hipMemcpy(d_cat_list_, cats.data(), sizeof(int32_t) * cats.size(), hipMemcpyHostToDevice));
  }
  a.cat_list = d_cat_list_;
  if (voting_) {
    // every rank scans every feature locally (phase 1), then the elected ones globally (phase 2,
    // the arguments of VoteExchange); the per-leaf election buffers
    vote_k_ = std::max(1, std::min(config_->top_k, num_features_));
    if (vote_k_ > 64 || world_ * vote_k_ > 1024) {
      Log::Fatal("device voting-parallel supports top_k <= 64 and num_machines * top_k <= 1024");
    }
    a.p.vote_phase = 1;
    a.p.vote_k = vote_k_;
    a.p.skip_min_data = config_->min_data_in_leaf + 1;  // (encoded + 1: 0 is unset)
    a.p.sp = [&] {
      Config local = *config_;
      local.min_data_in_leaf /= world_;
      local.min_sum_hessian_in_leaf /= world_;
      return MakeSplitParams(local);
    }();
    d_root_local_ = Alloc<double>(3);
    // (round growth: one election per child of the round's expansions, 2 * round_k_ at once)
    const size_t sides = 2 * static_cast<size_t>(std::max(1, round_k_));
    d_vote_buf_ = Alloc<dev::VoteEntry>(static_cast<size_t>(world_) * sides * vote_k_);
    d_vote_list_ = Alloc<int32_t>(sides * vote_k_);
    d_vote_hist_ = Alloc<long long>(sides * vote_k_ * 2 * max_fb);
    a.root_local = d_root_local_;
    a.vote_buf = d_vote_buf_;
    a.vote_list = d_vote_list_;
    a.vote_hist = d_vote_hist_;
    split_collective_bytes_ = static_cast<double>(sizeof(dev::VoteEntry) * 2 * vote_k_ * world_) +
                              sizeof(long long) * 4.0 * vote_k_ * max_fb;
    root_collective_bytes_ = split_collective_bytes_ + 3 * sizeof(double) + 3 * sizeof(uint32_t);
    Log::Info("voting-parallel device learner, rank %d of %d: top_k %d; per split: proposal allgather %zu bytes "
              "per rank, elected-histogram all-reduce %zu bytes", rank_, world_, vote_k_,
              sizeof(dev::VoteEntry) * 2 * vote_k_, sizeof(long long) * 4 * static_cast<size_t>(vote_k_) * max_fb);
  } else if (distributed_) {
    // this rank scans its own features; the per-feature results are gathered rank-major
    a.feat_list = d_feat_list_;
    // (per-tree owners: every capacity slot has a workgroup, the unused ones exit)
    a.num_scan = dyn_owner_ ? max_owned_ : static_cast<int32_t>(owned_feats_.size());
    a.fb_index = d_fb_index_;
    a.fb_side = max_owned_;
    int owned_cats = 0;
    for (int f : owned_feats_) owned_cats += feats[f].is_cat ? 1 : 0;
    a.p.has_cat = dyn_owner_ ? (cats.empty() ? 0 : cat_cap_) : owned_cats;
    a.cat_list = d_owned_cats_;
    if (mode_ == Mode::kData) {
      a.rs_pos = d_rs_pos_;
      a.owned_hist = d_owned_hist_;
      a.owned_off = d_owned_off_;
      a.owned_bin_lo = owned_bin_lo_;
    } else {
      // feature-parallel: every rank has every row; histograms only over this rank's words
      int g_lo = num_groups_, g_hi = 0;
      for (int f : owned_feats_) {
        g_lo = std::min(g_lo, feats[f].group);
        g_hi = std::max(g_hi, feats[f].group + 1);
      }
      if (g_lo < g_hi) {
        a.tile_w0 = h_word_of_group_[g_lo];
        a.tile_w1 = h_word_of_group_[g_hi - 1] + 1;
      } else {  // no features: one tile of redundant work keeps the partition's launch shape
        a.tile_w0 = 0;
        a.tile_w1 = std::min(wpr, tile_words);
      }
      a.hist_tiles = (a.tile_w1 - a.tile_w0 + tile_words - 1) / tile_words;
    }
  }
  a.rd = nullptr;
  a.round_k = round_k_;
  a.round_dist = distributed_ ? 1 : 0;
  a.round_vote = (voting_ && round_k_ > 1) ? 1 : 0;
  a.rnode_lsum = nullptr;
  a.max_owned = max_owned_;
  a.rs_block = rs_block_;
  a.round_send = nullptr;
  a.round_owned = nullptr;
  if (round_k_ > 1 && data_parallel_) {
    d_round_send_ = Alloc<long long>(static_cast<size_t>(world_) * round_k_ * rs_block_ * 2);
    d_round_owned_ = Alloc<long long>(static_cast<size_t>(round_k_) * rs_block_ * 2);
    a.round_send = d_round_send_;
    a.round_owned = d_round_owned_;
  }
  // one workgroup per CU: the split kernel's registers (101-128 VGPRs) allow one 1024-thread
  // workgroup per CU, so a second one per CU ran as a second wave with its tail (A/B at HEAD,
  // 60 iterations: 256 / 384 / 512 / 768 workgroups = 2.11 / 2.30 / 2.18 / 2.21 ms at 10M,
  // 0.888 / 0.92 / 0.918 / 0.92 at 1.25M; round 3's 512 was chosen with fewer registers).
  // Wide int64 histograms (gpu_use_dp: two words per bin, LDS-bound at one workgroup per CU
  // either way) balance better over two waves of workgroups: 512 / 256 = 2.78 / 2.84 ms
  a.round_grid = a.hist_units == 2 ? 2 * split_grid_ : split_grid_;
  a.round_gr = 0;
  a.round_fused = 1;
  // the plan in the split scan's last workgroup while its tables fit the scan's LDS budget
  a.plan_in_find = (!distributed_ && dev::RoundPlanLds(n_leaves, split_rows_) <= 16384) ? 1 : 0;
  if (const char* e = tuning::Get(tuning::Knob::PlanInFind)) a.plan_in_find = e[0] == '1' ? 1 : 0;
  // (voting: the local sums are accumulated by k_round_split)
  if (const char* e = tuning::Get(tuning::Knob::RoundFused)) a.round_fused = (e[0] == '1' || a.round_vote) ? 1 : 0;
  if (const char* e = tuning::Get(tuning::Knob::RoundGrid)) a.round_grid = std::max(1, std::atoi(e));
  if (const char* e = tuning::Get(tuning::Knob::RoundGr)) a.round_gr = std::atoi(e);
  a.round_need_div = 0;
  if (const char* e = tuning::Get(tuning::Knob::RoundNeedDiv)) a.round_need_div = std::max(0, std::atoi(e));
  a.round_predict = 1;
  if (const char* e = tuning::Get(tuning::Knob::RoundPredict)) a.round_predict = e[0] == '0' ? 0 : 1;
  AllocRoundState();
  UploadInteractionMasks();
  AllocSplittable();
}

// interaction constraints as per-feature constraint bitmasks (device-resident growth
// supports up to dev::kMaxIcConstraints = 256 constraints, see DecideMode); rebuilt when the config changes
void GPUTreeLearner::UploadInteractionMasks() {
  const auto& ic = config_->interaction_constraints_vector;
  args_.feat_icmask = nullptr;
  if (ic.empty() || ic.size() > static_cast<size_t>(dev::kMaxIcConstraints)) return;
  std::vector<dev::IcMask> icm(std::max(1, num_features_), dev::IcMask{});
  for (int f = 0; f < num_features_; ++f) {
    const int real = data_->RealFeatureIndex(f);
    for (size_t k = 0; k < ic.size(); ++k) {
      if (std::find(ic[k].begin(), ic[k].end(), real) != ic[k].end()) icm[f].Set(static_cast<int>(k));
    }
  }
  if (d_feat_icmask_ == nullptr) d_feat_icmask_ = Alloc<dev::IcMask>(icm.size());
  HIPCHECK(hipMemcpy(d_feat_icmask_, icm.data(), sizeof(dev::IcMask) * icm.size(), hipMemcpyHostToDevice));
  args_.feat_icmask = d_feat_icmask_;
}

void GPUTreeLearner::AllocSplittable() {
  const int n_leaves = config_->num_leaves, nf = std::max(1, num_features_);
  d_splittable_ = Alloc<int8_t>(static_cast<size_t>(std::max(n_leaves, split_rows_)) * nf);
  d_parent_flags_ = Alloc<int8_t>(nf);
  std::vector<dev::Leaf> leaves(n_leaves);
  for (int l = 0; l < n_leaves; ++l) {
    std::memset(&leaves[l], 0, sizeof(dev::Leaf));
    leaves[l].frow = l;
  }
  HIPCHECK(hipMemsetAsync(d_splittable_, 1, static_cast<size_t>(std::max(n_leaves, split_rows_)) * nf, stream_));
  HIPCHECK(hipMemcpyAsync(d_leaves_, leaves.data(), sizeof(dev::Leaf) * n_leaves, hipMemcpyHostToDevice, stream_));
  HIPCHECK(hipStreamSynchronize(stream_));
  args_.splittable = d_splittable_;
  args_.parent_flags = d_parent_flags_;
}

void GPUTreeLearner::ResetTrainingData(const Dataset* train_data, bool is_constant_hessian) {
  DropSpeculation();
  ++state_epoch_;
  SerialTreeLearner::ResetTrainingData(train_data, is_constant_hessian);
  HIPCHECK(hipSetDevice(device_id_));
  // rebuild the device data for the new rows (bin mappers are aligned)
  HIPCHECK(hipStreamSynchronize(stream_));
  FreeBuffers();
  UploadData();  // (re-decides the round width for the new rows per rank)
  oob_cnt_ = 0;
  // the growth-mode timing and the width history belong to the old rows (every rank resets
  // here, so the distributed ranks re-decide at the same tree)
  auto_state_ = kAutoUnset;
  auto_tree_ = 0;
  auto_rounds_ms_ = 1e300;
  prev_splits_ = prev_expansions_ = 0;
}

void GPUTreeLearner::ResetConfig(const Config* config) {
  DropSpeculation();
  ++state_epoch_;
  const int old_leaves = config_->num_leaves;
  SerialTreeLearner::ResetConfig(config);
  ResetVoteXt();  // (both generator sets reseeded, as the reference's ResetConfig)
  DestroyGraph();  // kernel arguments are baked into the captured graph
  args_.p.sp = params_;
  args_.p.cegb = 0;  // re-derived from the new penalties by the next DecideMode
  args_.p.mono_inter = 0;
  args_.p.max_depth = config_->max_depth;
  args_.p.monotone_penalty = config_->monotone_penalty;
  if (config_->num_leaves != old_leaves) {
    if (config_->num_leaves > dev::kMaxLeaves) Log::Fatal("device learner supports num_leaves <= %d", dev::kMaxLeaves);
    HIPCHECK(hipSetDevice(device_id_));
    const int n_leaves = config_->num_leaves;
    d_leaves_ = Alloc<dev::Leaf>(n_leaves);
    d_node_mask_ = Alloc<int8_t>(static_cast<size_t>(2 * n_leaves) * std::max(1, num_features_));
    d_xt_cum_ = Alloc<int32_t>(static_cast<size_t>(n_leaves) * std::max(1, num_features_));
    AllocVoteXt(n_leaves);
    d_rec_ = Alloc<dev::SplitRecord>(std::max(1, n_leaves - 1));
    d_best_ = Alloc<DeviceSplit>(n_leaves);
    SizeRoundPools(n_leaves);
    d_hist_ = Alloc<long long>(static_cast<size_t>(hist_slots_) * 2 * total_bins_);
    d_leaf_values_ = Alloc<double>(n_leaves);
    if (h_rec_) (void)hipHostFree(h_rec_);
    HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&h_rec_), sizeof(dev::SplitRecord) * std::max(1, n_leaves - 1),
                           hipHostMallocDefault));
    args_.p.num_leaves = n_leaves;
    args_.leaves = d_leaves_;
    args_.rec = d_rec_;
    args_.best = d_best_;
    args_.hist = d_hist_;
    AllocRoundState();
    AllocSplittable();
    global_count_.assign(n_leaves, 0);
  }
  if (WideHistograms(*config_) != (hist_units_ == 2)) {
    Log::Warning("device learner: gpu_use_dp cannot change after training started; keeping %s histograms",
                 hist_units_ == 2 ? "wide" : "packed");
  }
  UploadInteractionMasks();
  // monotone / penalty metadata may have changed
  std::vector<dev::Feature> feats(num_features_);
  HIPCHECK(hipMemcpy(feats.data(), d_feat_, sizeof(dev::Feature) * num_features_, hipMemcpyDeviceToHost));
  for (int f = 0; f < num_features_; ++f) {
    feats[f].monotone = meta_[f].monotone_type;
    feats[f].penalty = meta_[f].penalty;
  }
  HIPCHECK(hipMemcpy(d_feat_, feats.data(), sizeof(dev::Feature) * num_features_, hipMemcpyHostToDevice));
  h_feats_ = feats;
}

void GPUTreeLearner::DecideMode() {
  bool dm = true;
  const char* force = tuning::Get(tuning::Knob::HostAssist);
  if ((force != nullptr && force[0] == '1') || force_host_mode_) dm = false;
  bool any_cat = false;
  for (int f = 0; f < num_features_ && dm; ++f) {
    // categorical splits are scanned on the device up to kFindMaxCatBins categories
    const BinMapper* m = data_->FeatureBinMapper(f);
    if (m->bin_type() == BinType::Categorical) any_cat = true;
    if (m->bin_type() == BinType::Categorical && m->num_bin() > dev::kFindMaxCatBins) dm = false;
  }
  // extra_trees: random thresholds are drawn on the device (categorical ones by the workgroup
  // that scans both children of the feature in order); the distributed learners keep
  // categorical draws host-assisted
  if (config_->extra_trees && any_cat && distributed_) dm = false;
  // interaction constraints: on the device up to 256 constraints; with per-node sampling the
  // children's masks are drawn on the device after each partition (k_bynode_step) -- under the
  // distributed learners too: every rank picks the same split, so every rank's generator draws
  // the same masks
  const auto& ic = config_->interaction_constraints_vector;
  if (!ic.empty() && ic.size() > static_cast<size_t>(dev::kMaxIcConstraints)) dm = false;
  // intermediate monotone constraints re-bound leaves all over the tree after a split: the pick
  // walks the tree and the next split scan re-scans the re-bounded leaves (one process, one
  // split per step; with extra_trees draws, forced splits or more than kMonoInterMaxLeaves
  // leaves the host loop does it between the device histogram builds)
  const bool mono_inter = config_->monotone_constraints_method == "intermediate" &&
                          std::any_of(config_->monotone_constraints.begin(), config_->monotone_constraints.end(),
                                      [](int8_t m) { return m != 0; });
  if (mono_inter && (distributed_ || config_->extra_trees || has_forced_split_ ||
                     config_->num_leaves > dev::kMonoInterMaxLeaves)) {
    dm = false;
  }
  // voting: extra_trees draws stay with the host voting loop -- its local scans skip the
  // features their parent's local scan could not split and draw from the feature generators,
  // its global scans draw from a second generator set on the rank that owns each elected
  // histogram (reference feature_metas_); per-node sampling runs on the device (the global
  // scan's masks)
  if (voting_ && config_->extra_trees && any_cat) dm = false;
  // CEGB: split and coupled feature penalties are applied by the device scans (single rank);
  // lazy penalties (per-row usage bitsets) and distributed CEGB run host-assisted
  const bool cegb = CostEffectiveGB::Enabled(*config_);
  // forced splits: applied by the pick (the static BFS schedule of the JSON tree); under the
  // feature-parallel learner the owner of a forced node's feature computes its record and every
  // rank picks it from the gathered records (the data-parallel learner rejects forced splits, as
  // the reference does; voting keeps them host-assisted).  Per-node sampling and CEGB split / coupled penalties run
  // device-resident under the distributed learners too: every rank draws the same node samples
  // and holds the same CEGB state, the owners' scans apply them (LGBM_AMD_DIST_HOST_ASSIST=1:
  // the host-assisted fallback, for A/B)
  const char* dha = tuning::Get(tuning::Knob::DistHostAssist);
  const bool dist_fallback = distributed_ && dha != nullptr && dha[0] == '1';
  if (has_forced_split_ && ((distributed_ && !ForcedGathered()) || !SetupForcedSplits())) dm = false;
  if (!has_forced_split_ && args_.forced_n > 0) SetupForcedSplits();  // (cleared)
  if ((config_->feature_fraction_bynode < 1.0 && dist_fallback) ||
      (cegb && ((!config_->cegb_penalty_feature_lazy.empty() && (distributed_ || num_features_ > 8192)) ||
                dist_fallback))) {
    dm = false;
  }
  if (cegb && dm && !args_.p.cegb) SetupCegb();
  if (mono_inter && dm && !args_.p.mono_inter) SetupMonoInter();
  if (!(mono_inter && dm) && args_.p.mono_inter) {
    args_.p.mono_inter = 0;
    DestroyGraph();
  }
  if (dm != device_mode_ || !mode_decided_) {
    mode_decided_ = true;
    Log::Debug("device learner: %s growth", dm ? "device-resident" : "host-assisted");
  }
  device_mode_ = dm;
}

void GPUTreeLearner::SetBaggingData(const Dataset* subset, const data_size_t* used_indices, data_size_t n) {
  DropSpeculation();
  SerialTreeLearner::SetBaggingData(subset, used_indices, n);
  HIPCHECK(hipSetDevice(device_id_));
  oob_cnt_ = 0;
  if (use_bag_) {
    HIPCHECK(hipMemcpyAsync(d_bag_, used_indices, sizeof(int32_t) * n, hipMemcpyHostToDevice, stream_));
    // GBDT keeps the out-of-bag rows after the in-bag ones (bag_data_indices_ has num_data entries)
    oob_cnt_ = num_data_ - n;
    if (oob_cnt_ > 0) {
      HIPCHECK(hipMemcpyAsync(d_oob_, used_indices + n, sizeof(int32_t) * oob_cnt_, hipMemcpyHostToDevice, stream_));
    }
    const int32_t cnt = n;
    HIPCHECK(hipMemcpyAsync(d_bag_count_, &cnt, sizeof(int32_t), hipMemcpyHostToDevice, stream_));
    HIPCHECK(hipStreamSynchronize(stream_));
  }
}

// ---------------------------------------------------------------- tree growth
// the fused gradient kernel writes only the interleaved (g, h): grad / hess are unpacked
// when something reads them (GOSS, a download, a host-assisted tree, a repack)
void GPUTreeLearner::MaterializeSplitGradients() {
  if (!split_stale_) return;
  dev::UnpackGH(d_gh_, args_.gh_stride, num_data_, d_grad_, d_hess_, stream_);
  split_stale_ = false;
}

Tree* GPUTreeLearner::Train(const score_t* gradients, const score_t* hessians) {
  common::ScopedTimer timer("GPUTreeLearner::Train");
  HIPCHECK(hipSetDevice(device_id_));
  train_shrink_ = expect_shrinkage_;  // (the promise covers this tree only)
  expect_shrinkage_ = 0.0;
  early_scored_leaves_ = 0;
  if (distributed_ && Network::device_comm() != nullptr) Network::device_comm()->HostBarrier();
  // fixed-point scales of this tree: max |g|, max h over all rows (and ranks)
  // the gradient kernel already interleaved (g, h) and found max|g| / max h when it wrote
  // exactly these buffers (one model per iteration, not modified on the host since)
  root_from_parts_ = gh_fresh_ && gradients == d_grad_ && hessians == d_hess_;
  gh_fresh_ = false;
  if (spec_live_) {
    // the tree launched when the last one ended: its scales came from the score walk's
    // partials, so it is this tree when these are the walk's gradients and nothing was reset
    if (root_from_parts_ && grad_from_prefetch_ && spec_epoch_ == state_epoch_ && !use_bag_) {
      spec_live_ = false;
      spec_sampler_.reset();
      host_partition_fresh_ = false;
      DecideMode();
      if (device_mode_) return TrainDeviceMode(true);
      DropSpeculation();  // (unreachable: the mode depends on the configuration only)
    } else {
      Log::Debug("device learner: the launched tree is regrown (walk parts %d, prefetched gradients %d, epoch %d, bag %d)",
                 root_from_parts_ ? 1 : 0, grad_from_prefetch_ ? 1 : 0, spec_epoch_ == state_epoch_ ? 1 : 0,
                 use_bag_ ? 1 : 0);
      DropSpeculation();
    }
  }
  // (the reduction writes the whole absmax record: no reset copy; without an all-reduce of it
  // the same launch computes the scales)
  const bool absmax_global = (data_parallel_ || voting_) && Network::num_machines() > 1;
  double* fused_scales = absmax_global ? nullptr : d_scales_;
  if (root_from_parts_) {
    dev::ReduceParts(d_max_parts_, d_root_parts_, grad_parts_, num_data_, rows_cap_, d_absmax_, d_root_, stream_,
                     hist_units_, fused_scales);
  } else {
    MaterializeSplitGradients();
    dev::PackGH(gradients, hessians, d_gh_, args_.gh_stride, num_data_, d_max_parts_, stream_);
    dev::ReduceParts(d_max_parts_, nullptr, dev::PackBlocks(num_data_), num_data_, rows_cap_, d_absmax_, nullptr,
                     stream_, hist_units_, fused_scales);
  }
  if (absmax_global) {
    AllreduceAbsMax();
    dev::ComputeScales(d_absmax_, rows_cap_, hist_units_, d_scales_, stream_);
  }
  host_partition_fresh_ = false;
  DecideMode();
  if (device_mode_) return TrainDeviceMode();
  MaterializeSplitGradients();
  last_stats_ = TreeStats();
  Tree* t = SerialTreeLearner::Train(gradients, hessians);
  last_stats_.splits = t->num_leaves() - 1;
  return t;
}

// wait for the tree; with device collectives, poll the communicator for asynchronous
// errors and bound the wait by time_out minutes (the reference's socket timeout): a failed
// or vanished peer aborts the communicator and raises instead of hanging every rank
void GPUTreeLearner::WatchdogSync() {
  DeviceComm* dc = distributed_ ? Network::device_comm() : nullptr;
  if (dc == nullptr) {
    HIPCHECK(hipStreamSynchronize(stream_));
    return;
  }
  const double limit_s = 60.0 * std::max(1, config_->time_out);
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t q = hipStreamQuery(stream_);
    if (q == hipSuccess) return;
    if (q != hipErrorNotReady) HIPCHECK(q);
    std::string err;
    if (dc->AsyncError(&err)) {
      dc->Abort();
      Log::Fatal("device collective failed during tree growth: %s", err.c_str());
    }
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (el > limit_s) {
      dc->Abort();
      Log::Fatal("device collectives timed out after %.0f s (time_out=%d min): a peer rank stopped", el,
                 config_->time_out);
    }
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

// diagnostics (LGBM_AMD_KERNEL_PROBE=1): the tree is finished (Step::done), so every step
// kernel exits after reading the Step record; time N back-to-back launches of each
void GPUTreeLearner::KernelFloorProbe(const dev::KArgs& a) {
  hipEvent_t e0, e1;
  HIPCHECK(hipEventCreate(&e0));
  HIPCHECK(hipEventCreate(&e1));
  const int n = 500;
  struct P {
    const char* name;
    void (*fn)(const dev::KArgs&, hipStream_t);
  };
  const P probes[] = {{"split+reduce", [](const dev::KArgs& k, hipStream_t st) { dev::SplitStep(k, st, true); }},
                      {"find", dev::FindStep}};
  for (const P& p : probes) {
    for (int i = 0; i < 20; ++i) p.fn(a, stream_);
    HIPCHECK(hipEventRecord(e0, stream_));
    for (int i = 0; i < n; ++i) p.fn(a, stream_);
    HIPCHECK(hipEventRecord(e1, stream_));
    HIPCHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
    std::fprintf(stderr, "kernel probe %-12s %.2f us per launch (tree done: early exit)\n", p.name, 1000.f * ms / n);
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
}

// LGBM_AMD_KTRACE=1: in-kernel timestamps of the first workgroup of every step kernel (and
// of the picking workgroup), 100 MHz clock, averaged over the splits of each tree and printed
// to stderr as the time between consecutive stamps (a stamp a split did not take -- no
// reduce kernel, no split scan -- is skipped)
void GPUTreeLearner::ReportKernelTrace(int num_splits) {
  const int L = config_->num_leaves;
  std::vector<long long> t(static_cast<size_t>(L) * dev::kTraceSlots);
  HIPCHECK(hipMemcpy(t.data(), d_ktrace_, sizeof(long long) * t.size(), hipMemcpyDeviceToHost));
  static const int order[] = {dev::kTrSplitEntry, dev::kTrSplitRows,   dev::kTrSplitSide,   dev::kTrSplitResv,
                              dev::kTrSplitGather, dev::kTrSplitAccum, dev::kTrSplitExit,   dev::kTrRedEntry,
                              dev::kTrRedExit,     dev::kTrFindEntry,  dev::kTrFindHdr,     dev::kTrFindLoaded,
                              dev::kTrFindScanned, dev::kTrFindExit,   dev::kTrPickEntry,   dev::kTrPick1,
                              dev::kTrPW1,         dev::kTrPW2,        dev::kTrPick2,       dev::kTrPickRep,
                              dev::kTrPick3,
                              dev::kTrPick4,       dev::kTrPickExit};
  static const char* names[] = {"split.entry", "split.rows",  "split.side", "split.resv", "split.gather",
                                "split.accum", "split.exit",  "red.entry",  "red.exit",   "find.entry",
                                "find.hdr",    "find.loaded", "find.scanned", "find.exit", "pick.entry",
                                "pick.book",   "pick.fsides", "pick.leaves", "pick.wave",  "pick.again",
                                "pick.copy",
                                "pick.conv",   "pick.exit"};
  const int n = static_cast<int>(sizeof(order) / sizeof(order[0]));
  std::vector<double> sum(n + 1, 0.0);
  std::vector<int> cnt(n + 1, 0);
  const int s0 = std::min(num_splits, 8);
  double total = 0.0;
  int total_n = 0;
  for (int s = s0; s + 1 < num_splits; ++s) {
    const long long* row = &t[static_cast<size_t>(s) * dev::kTraceSlots];
    long long prev = 0;
    for (int k = 0; k <= n; ++k) {
      const long long v = k < n ? row[order[k]] : t[static_cast<size_t>(s + 1) * dev::kTraceSlots + dev::kTrSplitEntry];
      if (v <= 0) continue;
      if (prev > 0 && v >= prev) {
        sum[k] += static_cast<double>(v - prev) / 100.0;
        ++cnt[k];
      }
      prev = v;
    }
    const long long b = row[dev::kTrSplitEntry];
    const long long e = t[static_cast<size_t>(s + 1) * dev::kTraceSlots + dev::kTrSplitEntry];
    if (b > 0 && e > b) {
      total += static_cast<double>(e - b) / 100.0;
      ++total_n;
    }
  }
  std::string line = "ktrace (us to each stamp, avg over splits " + std::to_string(s0) + ".." +
                     std::to_string(num_splits - 2) + "):";
  for (int k = 0; k <= n; ++k) {
    if (cnt[k] == 0) continue;
    char buf[64];
    std::snprintf(buf, sizeof(buf), " %s=%.2f", k < n ? names[k] : "next.split", sum[k] / cnt[k]);
    line += buf;
  }
  char buf[64];
  std::snprintf(buf, sizeof(buf), " | per split %.2f", total_n ? total / total_n : -1.0);
  line += buf;
  // shader clock over the picks (s_memtime cycles per 100 MHz wall tick)
  double cyc = 0.0, wall = 0.0;
  for (int s = s0; s + 1 < num_splits; ++s) {
    const long long* row = &t[static_cast<size_t>(s) * dev::kTraceSlots];
    if (row[dev::kTrClk1] > row[dev::kTrClk0] && row[dev::kTrPickExit] > row[dev::kTrPick1]) {
      cyc += static_cast<double>(row[dev::kTrClk1] - row[dev::kTrClk0]);
      wall += static_cast<double>(row[dev::kTrPickExit] - row[dev::kTrPick1]);
    }
  }
  if (wall > 0) {
    std::snprintf(buf, sizeof(buf), " | shader clock %.0f MHz", 100.0 * cyc / wall);
    line += buf;
  }
  std::fprintf(stderr, "%s\n", line.c_str());
}

void GPUTreeLearner::DestroyGraph() {
  DestroyStepGraph();
  DestroyRoundGraphs();
}

void GPUTreeLearner::DestroyStepGraph() {
  if (graph_exec_ != nullptr) (void)hipGraphExecDestroy(graph_exec_);
  graph_exec_ = nullptr;
}

void GPUTreeLearner::DestroyRoundGraphs() {
  for (hipGraphExec_t& e : round_root_execs_) {
    if (e != nullptr) (void)hipGraphExecDestroy(e);
  }
  round_root_execs_.clear();
  if (round_seg_exec_ != nullptr) (void)hipGraphExecDestroy(round_seg_exec_);
  round_seg_exec_ = nullptr;
}

// the whole tree as a stream-ordered kernel sequence (no host synchronisation inside)
void GPUTreeLearner::EnqueueTree(const dev::KArgs& a) {
  EnqueueRoot(a);
  // voting: the global scan of the elected features picks (pick_in_find); the local scan does not
  const dev::KArgs glob = voting_ ? VoteGlobalArgs(a, 1) : a;
  if (voting_) {
    VoteExchange(glob, true);
    dev::FindRoot(glob, stream_);
  } else if (distributed_) {
    GatherFeatureBests();
    dev::PickStep(a, stream_, true);
  }
  const size_t stride_bytes = sizeof(long long) * static_cast<size_t>(a.scratch_stride);
  // one split per step: the picked split applied to the leaf's rows with one child's
  // histogram (+ reduction, + reduce-scatter to the feature owners) -> split scans of both
  // children (+ the next pick; distributed: after gathering every rank's results).  The
  // sequence is fixed; kernels of a finished tree exit at once.
  for (int s = 0; s < config_->num_leaves - 1; ++s) {
    if (data_parallel_) {
      HIPCHECK(hipMemsetAsync(d_scratch_ + static_cast<size_t>((s + 1) & 1) * a.scratch_stride, 0, stride_bytes,
                              stream_));
    }
    // (a reduce kernel for every step of the learners with global counts -- data- and
    // voting-parallel: DirectPartials never lets their split scans sum the partials)
    dev::SplitStep(a, stream_, s < a.p.direct_from_split || a.p.data_parallel != 0);
    if (a.cegb_lazy != nullptr) dev::CegbStep(a, stream_);
    if (a.bynode_rng != nullptr) dev::ByNodeStep(a, stream_);
    ReduceScatterStep(s + 1);
    dev::FindStep(a, stream_);
    if (voting_) {
      VoteExchange(glob, false);
      dev::FindStep(glob, stream_);
    } else if (distributed_) {
      GatherFeatureBests();
      dev::PickStep(a, stream_, false);
    }
  }
}

// the tree's root: row set, sums, histogram and split scan (+ the first pick / plan)
void GPUTreeLearner::EnqueueRoot(const dev::KArgs& a) {
  if (a.forced_n > 0) {
    // every forced record starts the tree as zero words: a node whose leaf was not scanned this
    // tree reads as invalid (no rows) instead of as the last tree's record
    const size_t blocks = a.forced_world > 1 ? a.forced_world : 1;
    HIPCHECK(hipMemsetAsync(d_forced_best_, 0, sizeof(dev::FeatureBest) * a.forced_n * blocks, stream_));
    HIPCHECK(hipMemsetAsync(d_forced_cat_, 0, sizeof(uint32_t) * kMaxCatWords * a.forced_n * blocks, stream_));
  }
  if (use_bag_) {
    // the whole buffer: the copy (like the tree's graph) does not depend on the bag size
    HIPCHECK(hipMemcpyAsync(d_idx_, d_bag_, sizeof(int32_t) * num_data_, hipMemcpyDeviceToDevice, stream_));
  }
  // both step buffers start at zero; afterwards each split-scan zeroes the next one
  // (data-parallel: the owner-major buffer is cleared before every reduction)
  // both step buffers start at zero (round growth: every expansion buffer of both parities)
  const size_t stride_bytes = sizeof(long long) * static_cast<size_t>(a.scratch_stride);
  const size_t zero_bytes = a.rd != nullptr ? sizeof(long long) * 4 * static_cast<size_t>(a.round_k) * total_bins_
                                            : 2 * stride_bytes;
  if (a.ktrace != nullptr) {
    HIPCHECK(hipMemsetAsync(a.ktrace, 0, sizeof(long long) * dev::kTraceSlots * config_->num_leaves, stream_));
  }
  // (the scratch zeroing and the feature mask's upload happen in the tree's first kernel)
  const bool copy_nodes = tuning::On(tuning::Knob::GraphCopyNodes);
  if (copy_nodes) {
    HIPCHECK(hipMemcpyAsync(d_tree_mask_, h_mask_, num_features_, hipMemcpyHostToDevice, stream_));
    HIPCHECK(hipMemsetAsync(d_scratch_, 0, zero_bytes, stream_));
    dev::TreeBegin(a, stream_);
  } else {
    dev::TreeBegin(a, stream_, d_scratch_, zero_bytes, h_mask_, num_features_);
  }
  if (a.p.mono_inter) {  // (intermediate monotone: the root leaf has no parent, nothing is re-bounded yet)
    const int L = config_->num_leaves;
    HIPCHECK(hipMemsetAsync(a.mt_leaf_parent, 0xff, sizeof(int32_t) * L, stream_));
    HIPCHECK(hipMemsetAsync(a.mt_in_sub, 0, L, stream_));
    HIPCHECK(hipMemsetAsync(a.mt_upd, 0, sizeof(int32_t), stream_));
  }
  if (a.xt_cum != nullptr) {
    HIPCHECK(hipMemsetAsync(a.xt_cum, 0, sizeof(int32_t) * config_->num_leaves * num_features_, stream_));
  }
  if (a.xt_cum_glob != nullptr) {
    HIPCHECK(hipMemsetAsync(a.xt_cum_glob, 0, sizeof(int32_t) * config_->num_leaves * world_ * num_features_, stream_));
  }
  if (!(root_from_parts_ && !use_bag_)) dev::RootSum(a, stream_);  // else: set by ReduceParts
  AllreduceRoot();
  if (a.rd != nullptr && data_parallel_ && d_round_send_ != nullptr) {  // (the first round's send buffer)
    HIPCHECK(hipMemsetAsync(d_round_send_, 0, sizeof(long long) * world_ * round_k_ * rs_block_ * 2, stream_));
  }
  dev::HistRoot(a, stream_);
  ReduceScatterStep(0);
  if (a.cegb_lazy != nullptr) {
    HIPCHECK(hipMemsetAsync(a.cegb_cnt, 0, sizeof(int32_t) * num_features_, stream_));
    HIPCHECK(hipMemsetAsync(a.cegb_scratch, 0, sizeof(int32_t) * 2 * num_features_, stream_));
    dev::CegbRoot(a, stream_);
  }
  dev::FindRoot(a, stream_);
  if (a.rd != nullptr && voting_) {
    // the root's vote and global scan (publish only), then the first plan from its results
    const dev::KArgs glob = VoteGlobalArgs(a, 0);
    VoteExchange(glob, true);
    dev::FindRoot(glob, stream_);
    dev::RoundRootPlan(glob, stream_);
  } else if (a.rd != nullptr) {
    if (distributed_) GatherFeatureBests();  // (the root's results, side-0 layout)
    dev::RoundRootPlan(a, stream_);
  }
}

Tree* GPUTreeLearner::TrainDeviceMode(bool speculated) {
  if (!speculated) {  // (a speculated tree drew its sample when it was launched)
    col_sampler_.ResetByTree();
    const auto& mask = col_sampler_.is_feature_used_bytree();
    for (int f = 0; f < num_features_; ++f) h_mask_[f] = mask[f];
  }
  OwnershipForTree();
  dev::KArgs a = args_;
  const bool bynode = config_->feature_fraction_bynode < 1.0;
  const bool bynode_ic = bynode && col_sampler_.has_interaction_constraints();
  if (bynode_ic) {
    // the root's mask (no branch: every constraint's features) from a copy of the generator;
    // the children's masks are drawn on the device from the state after it (k_bynode_step)
    const Tree empty(2, true);
    ColSampler copy(col_sampler_);
    h_node_mask_ = copy.GetByNode(&empty, 0);
    h_bynode_rng_ = copy.rng_state();
    h_bynode_pool_ = col_sampler_.NodePoolInner();
    HIPCHECK(hipMemcpyAsync(d_node_mask_, h_node_mask_.data(), h_node_mask_.size(), hipMemcpyHostToDevice, stream_));
    HIPCHECK(hipMemcpyAsync(d_bynode_pool_, h_bynode_pool_.data(), sizeof(int32_t) * h_bynode_pool_.size(),
                            hipMemcpyHostToDevice, stream_));
    HIPCHECK(hipMemcpyAsync(d_bynode_rng_, &h_bynode_rng_, sizeof(uint32_t), hipMemcpyHostToDevice, stream_));
    a.node_mask = d_node_mask_;
    a.bynode_pool_n = static_cast<int32_t>(h_bynode_pool_.size());
    a.bynode_cnt = col_sampler_.NodeSampleCount();
    a.bynode_rng = d_bynode_rng_;
  } else if (bynode) {
    // every GetByNode draw the tree can make (root + two per split), from a copy of the
    // generator; the draws actually made are replayed after the tree
    h_node_mask_ = col_sampler_.PeekByNodeMasks(2 * (config_->num_leaves - 1) + 1);
    HIPCHECK(hipMemcpyAsync(d_node_mask_, h_node_mask_.data(), h_node_mask_.size(), hipMemcpyHostToDevice, stream_));
    a.node_mask = d_node_mask_;
  }
  const bool xt = config_->extra_trees;
  a.xt_base = nullptr;
  a.xt_cum = nullptr;
  a.xt_base_glob = nullptr;
  a.xt_cum_glob = nullptr;
  if (xt && voting_) {
    // voting: every rank's global generator set at the tree's start (every rank replays every
    // owner's draws; VoteXtAdvance catches the host states up after the tree)
    if (xt_glob_rand_.size() != static_cast<size_t>(world_) * num_features_) ResetVoteXt();
    h_xt_base_glob_.resize(xt_glob_rand_.size());
    for (size_t i = 0; i < xt_glob_rand_.size(); ++i) h_xt_base_glob_[i] = xt_glob_rand_[i].state();
    HIPCHECK(hipMemcpyAsync(d_xt_base_glob_, h_xt_base_glob_.data(), sizeof(uint32_t) * h_xt_base_glob_.size(),
                            hipMemcpyHostToDevice, stream_));
    a.xt_base_glob = d_xt_base_glob_;
    a.xt_cum_glob = d_xt_cum_glob_;
  }
  if (xt) {
    // each feature's generator state at the tree's start: the split scans derive their draws
    // from it and the step rows of xt_cum; the host generators catch up after the tree
    h_xt_base_.resize(num_features_);
    for (int f = 0; f < num_features_; ++f) h_xt_base_[f] = meta_[f].rand.state();
    HIPCHECK(hipMemcpyAsync(d_xt_base_, h_xt_base_.data(), sizeof(uint32_t) * num_features_, hipMemcpyHostToDevice,
                            stream_));
    a.xt_base = d_xt_base_;
    a.xt_cum = d_xt_cum_;
  }
  if (use_bag_) {
    // bag size read on the device: one captured graph serves every bag
    a.num_rows = num_data_;
    a.num_rows_dev = d_bag_count_;
    a.root_identity = 0;
    root_rows_ = bag_cnt_;
  } else {
    a.num_rows = num_data_;
    a.root_identity = 1;
    root_rows_ = num_data_;
  }
  last_stats_.rounds = 0;
  last_stats_.expansions = 0;
  last_stats_.graph = false;
  last_stats_.speculated = speculated;
  const bool can_round = RoundGrowth(a);
  const bool rounds = can_round && AutoGrowthRounds();
  const auto t_grow = std::chrono::steady_clock::now();
  if (!rounds && last_tree_rounds_) {
    // one split per step after round trees: splittable rows follow the leaf ids again
    std::vector<dev::Leaf> lv(config_->num_leaves);
    HIPCHECK(hipMemcpyAsync(lv.data(), d_leaves_, sizeof(dev::Leaf) * lv.size(), hipMemcpyDeviceToHost, stream_));
    HIPCHECK(hipStreamSynchronize(stream_));
    for (int l = 0; l < config_->num_leaves; ++l) lv[l].frow = l;
    HIPCHECK(hipMemcpy(d_leaves_, lv.data(), sizeof(dev::Leaf) * lv.size(), hipMemcpyHostToDevice));
  }
  if (speculated && !rounds) Log::Fatal("device learner: the launched next tree is not a round tree");
  last_tree_rounds_ = rounds;
  int num_splits = 0;
  if (rounds) {
    if (a.p.cegb && a.cegb_coupled != nullptr) {  // (the model-wide used flags: all of the tree's sample)
      h_cegb_used_ = cegb_->used_in_split();
      h_cegb_used_.resize(std::max(1, num_features_), 0);
      HIPCHECK(hipMemcpyAsync(d_cegb_used_, h_cegb_used_.data(), h_cegb_used_.size(), hipMemcpyHostToDevice, stream_));
    }
    if (speculated) {
      num_splits = WaitRounds(&spec_);
    } else if (spec_live_) {
      Log::Fatal("device learner: a launched next tree was not consumed");
    } else {
      num_splits = RunRounds(a);
    }
    if (a.round_cegb && a.cegb_coupled != nullptr && cegb_) {  // (the features the tree used first)
      HIPCHECK(hipStreamSynchronize(stream_));
      HIPCHECK(hipMemcpy(h_cegb_used_.data(), d_cegb_used_, h_cegb_used_.size(), hipMemcpyDeviceToHost));
      cegb_->set_used_in_split(std::vector<char>(h_cegb_used_.begin(), h_cegb_used_.begin() + num_features_));
    }
  } else {
    // the tree's fixed kernel sequence (~4 launches per split) is replayed from a hipGraph:
    // eager launches are host-bound at ~4 us each, longer than most of these kernels.  With
    // data-parallel training the per-split RCCL all-reduces are captured into the same graph
    // (they are stream-ordered; every rank enqueues the same collectives either way); with
    // host collectives (no device communicator) the tree is launched eagerly.
    const bool distributed = distributed_;
    DeviceComm* dcomm = distributed ? Network::device_comm() : nullptr;
    const bool dev_comm = dcomm != nullptr && dcomm->CaptureSafe();
    const char* ng = tuning::Get(tuning::Knob::NoGraph);
    const char* gc = tuning::Get(tuning::Knob::GraphCollectives);
    const bool graph_collectives = dev_comm && !(gc != nullptr && gc[0] == '0') && !graph_capture_failed_;
    const bool use_graph = (!distributed || graph_collectives) && !(ng != nullptr && ng[0] == '1');
    bool launched = false;
    if (a.p.cegb && cegb_) {  // the model-wide used-feature flags of the host CEGB state
      h_cegb_used_ = cegb_->used_in_split();
      h_cegb_used_.resize(std::max(1, num_features_), 0);
      HIPCHECK(hipMemcpyAsync(d_cegb_used_, h_cegb_used_.data(), h_cegb_used_.size(), hipMemcpyHostToDevice, stream_));
    }
    if (use_graph) {
      const int root_mode = (root_from_parts_ && !use_bag_) ? 1 : 0;
      if (graph_exec_ == nullptr || graph_rows_ != a.num_rows || graph_identity_ != a.root_identity ||
          graph_root_mode_ != root_mode || graph_xt_ != (xt ? 1 : 0) + (bynode_ic ? 2 : 0)) {
        if (dcomm != nullptr) dcomm->HostBarrier();
        DestroyStepGraph();  // (the round graphs stay: the growth mode may switch per tree)
        hipGraph_t g = nullptr;
        HIPCHECK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
        std::string why;
        try {
          EnqueueTree(a);
        } catch (const std::exception& e) {
          why = e.what();
        }
        hipError_t ec = hipStreamEndCapture(stream_, &g);
        if (why.empty() && ec == hipSuccess) ec = hipGraphInstantiate(&graph_exec_, g, nullptr, nullptr, 0);
        if (g != nullptr) (void)hipGraphDestroy(g);
        if (!why.empty() || ec != hipSuccess) {
          if (why.empty()) why = hipGetErrorString(ec);
          (void)hipGetLastError();
          graph_exec_ = nullptr;
          if (!distributed) Log::Fatal("device learner: capturing the tree graph failed: %s", why.c_str());
          Log::Warning("device learner: capturing the RCCL collectives into the tree graph failed (%s); "
                       "launching trees eagerly", why.c_str());
          graph_capture_failed_ = true;
        } else {
          graph_rows_ = a.num_rows;
          graph_identity_ = a.root_identity;
          graph_root_mode_ = root_mode;
          graph_xt_ = (xt ? 1 : 0) + (bynode_ic ? 2 : 0);  // (the by-node kernels are part of the graph)
        }
      }
      if (graph_exec_ != nullptr) {
        HIPCHECK(hipGraphLaunch(graph_exec_, stream_));
        launched = true;
        last_stats_.graph = true;
      }
    }
    if (!launched) EnqueueTree(a);
    HIPCHECK(hipMemcpyAsync(h_step_, d_step_, sizeof(dev::Step), hipMemcpyDeviceToHost, stream_));
    HIPCHECK(hipMemcpyAsync(h_rec_, d_rec_, sizeof(dev::SplitRecord) * std::max(1, config_->num_leaves - 1),
                            hipMemcpyDeviceToHost, stream_));
    WatchdogSync();
    if (a.p.cegb && cegb_) {
      HIPCHECK(hipMemcpy(h_cegb_used_.data(), d_cegb_used_, h_cegb_used_.size(), hipMemcpyDeviceToHost));
      cegb_->set_used_in_split(std::vector<char>(h_cegb_used_.begin(), h_cegb_used_.begin() + num_features_));
    }
    num_splits = h_step_->nsplit;
  }
  if (can_round) {
    AutoGrowthRecord(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_grow).count());
  }
  last_stats_.device_mode = true;
  last_stats_.splits = num_splits;
  // every step's collectives run (exiting early once the tree is done): the sequence is fixed
  if (!rounds) {
    last_stats_.collective_bytes =
        distributed_ ? root_collective_bytes_ + split_collective_bytes_ * (config_->num_leaves - 1) : 0.0;
  }
  if (bynode && rounds) {
    // round growth: the draws the replay counted (Round::bynode_next), the root's included
    // when the root was scanned (0 otherwise: the root plan decides from the global count)
    Log::Debug("device learner: %d splits in rounds, %d by-node draws", num_splits, h_round_->bynode_next);
    col_sampler_.AdvanceByNode(h_round_->bynode_next);
  } else if (bynode) {
    // the root's draw happens only if the host learner would have scanned the root
    const bool root_scanned = h_step_->root_count >= 2 * config_->min_data_in_leaf;  // global count
    Log::Debug("device learner: %d splits, %d by-node draws, root count %d", num_splits, h_step_->bynode_next,
               h_step_->root_count);
    if (bynode_ic) {
      // the device generator went on from the root's draw: the host one takes its state
      if (root_scanned) {
        HIPCHECK(hipMemcpy(&h_bynode_rng_, d_bynode_rng_, sizeof(uint32_t), hipMemcpyDeviceToHost));
        col_sampler_.set_rng_state(h_bynode_rng_);
      }
    } else {
      col_sampler_.AdvanceByNode(root_scanned ? h_step_->bynode_next : 0);
    }
  }
  // (round growth: one process, the root's rows are this rank's; the plans keep the replay's
  // counts in row 1)
  const int xt_root_count = rounds ? static_cast<int>(root_rows_) : h_step_->root_count;
  if (xt && xt_root_count >= 2 * config_->min_data_in_leaf) {
    // replay the draws the split scans made: the rows are running counts, steps not run are 0
    const int rows = config_->num_leaves;
    h_xt_cum_.resize(static_cast<size_t>(rows) * num_features_);
    HIPCHECK(hipMemcpy(h_xt_cum_.data(), d_xt_cum_, sizeof(int32_t) * h_xt_cum_.size(), hipMemcpyDeviceToHost));
    for (int f = 0; f < num_features_; ++f) {
      int n = 0;
      for (int r = 0; r < rows; ++r) n = std::max(n, h_xt_cum_[static_cast<size_t>(r) * num_features_ + f]);
      for (int k = 0; k < n; ++k) meta_[f].rand.NextInt(0, 2);
    }
  }
  if (xt && a.xt_cum_glob != nullptr) VoteXtAdvance();
  if (a.ktrace != nullptr && !rounds) ReportKernelTrace(num_splits);
  if (const char* kp = tuning::Get(tuning::Knob::KernelProbe)) {
    if (kp[0] == '1' && !rounds) KernelFloorProbe(a);
  }
  // the promised training-score update (ExpectTrainingScoreUpdate), on the device before the
  // host builds the tree
  // round growth: the tree's last plan wrote the split records to the host (KArgs::host_out),
  // or they are copied now (one record per split) and the host waits for that copy only
  const double shrink = train_shrink_;
  const dev::SplitRecord* recs = h_rec_;
  const bool copy_recs = rounds && num_splits > 0 && !tree_out_used_;
  if (rounds && tree_out_used_) recs = reinterpret_cast<const dev::SplitRecord*>(h_tree_out_ + dev::kHostOutHeaderWords);
  if (copy_recs) {
    HIPCHECK(hipMemcpyAsync(h_rec_, d_rec_, sizeof(dev::SplitRecord) * num_splits, hipMemcpyDeviceToHost, stream_));
    if (rec_event_ == nullptr) HIPCHECK(hipEventCreateWithFlags(&rec_event_, hipEventDisableTiming));
    HIPCHECK(hipEventRecord(rec_event_, stream_));
  }
  if (shrink != 0.0 && num_splits >= 1 && FusedScoreWalk(num_splits + 1, 0) && !tuning::Off(tuning::Knob::EarlyScore)) {
    EarlyScoreUpdate(num_splits, shrink);
  }
  if (copy_recs) HIPCHECK(hipEventSynchronize(rec_event_));
  common::ScopedTimer build_timer("GPUTreeLearner::BuildTree");
  const bool track = !config_->interaction_constraints_vector.empty();
  std::unique_ptr<Tree> tree(new Tree(config_->num_leaves, track));
  for (int s = 0; s < num_splits; ++s) {
    const dev::SplitRecord& r = recs[s];
    SplitInfo si;
    si.FromDevice(r.split);
    const int inner = si.inner_feature;
    const BinMapper* m = data_->FeatureBinMapper(inner);
    const float gain = static_cast<float>(si.gain + config_->min_gain_to_split);
    if (m->bin_type() == BinType::Categorical) {
      // same tree records as SerialTreeLearner::SplitInner (bitsets over inner bins and raw values)
      auto bits_inner = common::ConstructBitset(si.cat_threshold.data(), si.num_cat_threshold);
      std::vector<int> cats(si.num_cat_threshold);
      for (int i = 0; i < si.num_cat_threshold; ++i) {
        cats[i] = static_cast<int>(data_->RealThreshold(inner, si.cat_threshold[i]));
      }
      auto bits = common::ConstructBitset(cats.data(), si.num_cat_threshold);
      tree->SplitCategorical(r.leaf, inner, si.feature, bits_inner.data(), static_cast<int>(bits_inner.size()),
                             bits.data(), static_cast<int>(bits.size()), si.left_output, si.right_output,
                             r.left_count, r.right_count, si.left_sum_hessian, si.right_sum_hessian, gain,
                             m->missing_type());
      continue;
    }
    tree->Split(r.leaf, inner, si.feature, si.threshold, data_->RealThreshold(inner, si.threshold), si.left_output,
                si.right_output, r.left_count, r.right_count, si.left_sum_hessian, si.right_sum_hessian, gain,
                m->missing_type(), si.default_left);
  }
  if (num_splits == 0) {
    Log::Warning("No further splits with positive gain, best gain: %f", -std::numeric_limits<double>::infinity());
  }
  Log::Debug("Trained a tree with leaves = %d and max_depth = %d", tree->num_leaves(), tree->max_depth());
  // the records are consumed: the next tree may be launched now (its last plan rewrites them)
  const bool spec_ok = SpeculationEligible(a, rounds) && early_scored_leaves_ == num_splits + 1 && num_splits >= 1;
  Log::Debug("device learner: next tree %s (allowed %d, rounds %d, scored early %d/%d)", spec_ok ? "launched" : "not launched",
             spec_allowed_ ? 1 : 0, rounds ? 1 : 0, early_scored_leaves_, num_splits + 1);
  if (spec_ok) LaunchSpeculative();
  return tree.release();
}

// The next tree may be launched before GBDT asks for it when nothing between the two Train()
// calls can change its inputs: GBDT allowed it (plain boosting, no bagging / renewal / custom
// gradients, one model per iteration), this tree's score walk computes the next gradients, and
// the tree grows in rounds of a single process without per-tree host state (per-node samples,
// extra_trees draws, CEGB, forced splits, intermediate monotone, the timing probe).
bool GPUTreeLearner::SpeculationEligible(const dev::KArgs& a, bool rounds) const {
  if (!spec_allowed_ || !rounds || distributed_ || use_bag_ || !device_mode_) return false;
  if (!tuning::On(tuning::Knob::Speculate)) return false;  // (opt-in: profiles/r06_speculation_ab.md)
  if (a.host_out == nullptr && !tree_out_used_) return false;
  if (config_->feature_fraction_bynode < 1.0 || config_->extra_trees || CostEffectiveGB::Enabled(*config_)) return false;
  if (a.forced_n > 0 || a.p.mono_inter || a.ktrace != nullptr) return false;
  if (auto_state_ != kAutoRounds || num_tree_per_iteration_ != 1) return false;
  return true;
}

void GPUTreeLearner::LaunchSpeculative() {
  common::ScopedTimer timer("GPUTreeLearner::LaunchSpeculative");
  // Train()'s prologue: the scales and root sums from the walk's partials (as a prefetched
  // gradient computation leaves them), the tree's feature sample
  const int parts = dev::AddTreeScoreGradParts(num_data_);
  dev::ReduceParts(d_max_parts_, d_root_parts_, parts, num_data_, rows_cap_, d_absmax_, d_root_, stream_, hist_units_,
                   d_scales_);
  spec_sampler_.reset(new ColSampler(col_sampler_));
  col_sampler_.ResetByTree();
  const auto& mask = col_sampler_.is_feature_used_bytree();
  for (int f = 0; f < num_features_; ++f) h_mask_[f] = mask[f];
  // TrainDeviceMode's arguments of a plain round tree over every row
  dev::KArgs a = args_;
  a.num_rows = num_data_;
  a.root_identity = 1;
  root_rows_ = num_data_;
  const bool keep_parts = root_from_parts_;
  root_from_parts_ = true;  // (the root graph of this mode: root sums from the partials)
  spec_ = LaunchRounds(a);
  root_from_parts_ = keep_parts;
  spec_live_ = true;
  spec_epoch_ = state_epoch_;
}

// voting extra_trees: the global scans' generator sets of every rank (each seeded like the
// feature generators, Random(extra_seed + feature): reference feature_metas_), and their
// device tables
void GPUTreeLearner::ResetVoteXt() {
  xt_glob_rand_.clear();
  if (!voting_) return;
  xt_glob_rand_.reserve(static_cast<size_t>(world_) * num_features_);
  for (int r = 0; r < world_; ++r) {
    for (int f = 0; f < num_features_; ++f) xt_glob_rand_.emplace_back(config_->extra_seed + f);
  }
}
void GPUTreeLearner::AllocVoteXt(int n_leaves) {
  if (!voting_) return;
  const size_t wf = static_cast<size_t>(world_) * std::max(1, num_features_);
  d_xt_base_glob_ = Alloc<uint32_t>(wf);
  d_xt_cum_glob_ = Alloc<int32_t>(static_cast<size_t>(n_leaves) * wf);
}
// after a voting tree: every rank's global generators advance by the draws its global scans
// made (the rows are running counts, steps not run are 0)
void GPUTreeLearner::VoteXtAdvance() {
  const size_t wf = static_cast<size_t>(world_) * num_features_;
  const int rows = config_->num_leaves;
  std::vector<int32_t> cum(static_cast<size_t>(rows) * wf);
  HIPCHECK(hipMemcpy(cum.data(), d_xt_cum_glob_, sizeof(int32_t) * cum.size(), hipMemcpyDeviceToHost));
  for (size_t e = 0; e < wf; ++e) {
    int n = 0;
    for (int r = 0; r < rows; ++r) n = std::max(n, cum[static_cast<size_t>(r) * wf + e]);
    for (int k = 0; k < n; ++k) xt_glob_rand_[e].NextInt(0, 2);
  }
}

void GPUTreeLearner::DropSpeculation() {
  if (!spec_live_) return;
  spec_live_ = false;
  HIPCHECK(hipStreamSynchronize(stream_));  // (the launched tree finishes: its rounds were provisioned or exit)
  if (spec_sampler_) col_sampler_ = *spec_sampler_;
  spec_sampler_.reset();
  ++state_epoch_;
}

// CEGB on the device (split + coupled penalties): the penalties, the model-wide used flags
// (mirrored from / back to the host CostEffectiveGB around every device tree) and the
// (leaf, feature) candidate memory
void GPUTreeLearner::SetupCegb() {
  const Config& c = *config_;
  args_.p.cegb = 1;
  args_.p.cegb_split = c.cegb_tradeoff * c.cegb_penalty_split;
  args_.cegb_coupled = nullptr;
  const int nf = std::max(1, num_features_);
  if (d_cegb_used_ == nullptr) d_cegb_used_ = Alloc<int8_t>(nf);
  args_.cegb_used = d_cegb_used_;
  if (!c.cegb_penalty_feature_coupled.empty()) {
    std::vector<double> coupled(nf, 0.0);
    for (int f = 0; f < num_features_; ++f) {
      coupled[f] = c.cegb_tradeoff * c.cegb_penalty_feature_coupled[data_->RealFeatureIndex(f)];
    }
    if (d_cegb_coupled_ == nullptr) d_cegb_coupled_ = Alloc<double>(nf);
    HIPCHECK(hipMemcpy(d_cegb_coupled_, coupled.data(), sizeof(double) * nf, hipMemcpyHostToDevice));
    args_.cegb_coupled = d_cegb_coupled_;
    const size_t cells = static_cast<size_t>(c.num_leaves) * nf;
    if (d_cegb_mem_ == nullptr) {
      d_cegb_mem_ = Alloc<dev::FeatureBest>(cells);
      d_cegb_mem_cat_ = Alloc<uint32_t>(cells * kMaxCatWords);
    }
  }
  args_.cegb_mem = d_cegb_mem_;
  args_.cegb_mem_cat = d_cegb_mem_cat_;
  // lazy penalties: the rows that paid for each feature, kept over the model (the reference's
  // per-model bitset, zeroed once), and the leaves' unpaid counts (src/device/cegb_kernels.hip)
  args_.cegb_lazy = nullptr;
  if (!c.cegb_penalty_feature_lazy.empty()) {
    std::vector<double> lazy(nf, 0.0);
    for (int f = 0; f < num_features_; ++f) {
      lazy[f] = c.cegb_tradeoff * c.cegb_penalty_feature_lazy[data_->RealFeatureIndex(f)];
    }
    const int pw = (nf + 31) / 32;
    if (d_cegb_lazy_ == nullptr) {
      d_cegb_lazy_ = Alloc<double>(nf);
      d_cegb_paid_ = Alloc<uint32_t>(static_cast<size_t>(num_data_) * pw);
      HIPCHECK(hipMemset(d_cegb_paid_, 0, sizeof(uint32_t) * static_cast<size_t>(num_data_) * pw));
      d_cegb_cnt_ = Alloc<int32_t>(static_cast<size_t>(c.num_leaves) * nf);
      d_cegb_scratch_ = Alloc<int32_t>(4 * static_cast<size_t>(nf));
    }
    HIPCHECK(hipMemcpy(d_cegb_lazy_, lazy.data(), sizeof(double) * nf, hipMemcpyHostToDevice));
    args_.cegb_lazy = d_cegb_lazy_;
    args_.cegb_paid = d_cegb_paid_;
    args_.cegb_paid_words = pw;
    args_.cegb_cnt = d_cegb_cnt_;
    args_.cegb_scratch = d_cegb_scratch_;
    args_.cegb_snap = d_cegb_scratch_ + 2 * static_cast<size_t>(nf);
  }
  DestroyGraph();
}

// intermediate monotone constraints on the device: per-feature result rows for the re-scanned
// leaves (sides 2 .. num_leaves + 1), the tree topology and the re-bounded leaf list
void GPUTreeLearner::SetupMonoInter() {
  const int L = config_->num_leaves, nf = std::max(1, num_features_);
  const size_t need = static_cast<size_t>(2 + L) * nf;
  if (fb_slots_ < need) {
    d_feat_best_ = Alloc<dev::FeatureBest>(need);
    d_feat_cat_ = Alloc<uint32_t>(need * kMaxCatWords);
    fb_slots_ = need;
    args_.feat_best = d_feat_best_;
    args_.feat_cat = d_feat_cat_;
  }
  if (mt_cap_ < L) {
    d_mt_leaf_parent_ = Alloc<int32_t>(L);
    d_mt_node_ = Alloc<int32_t>(3 * static_cast<size_t>(L));
    d_mt_in_sub_ = Alloc<int8_t>(L);
    d_mt_upd_ = Alloc<int32_t>(static_cast<size_t>(L) + 1);
    mt_cap_ = L;
  }
  args_.mt_leaf_parent = d_mt_leaf_parent_;
  args_.mt_node = d_mt_node_;
  args_.mt_in_sub = d_mt_in_sub_;
  args_.mt_upd = d_mt_upd_;
  args_.p.mono_inter = 1;
  DestroyGraph();
}

// percentile renewal on the device (reference regression_objective.hpp RenewTreeOutput): the
// leaves' rows straight from the partition, residuals from the device scores; leaf outputs
// averaged over the ranks like the host path
bool GPUTreeLearner::RenewTreeOutputOnDevice(Tree* tree, const ObjectiveFunction* obj, int tree_id) {
  if (spec_live_) Log::Fatal("device learner: leaf renewal after the next tree was launched (speculation not allowed)");
  DeviceRenewSpec spec;
  if (!device_mode_ || obj == nullptr || !obj->DeviceRenew(&spec) || spec.label == nullptr || d_score_ == nullptr) {
    return false;
  }
  const char* hr = tuning::Get(tuning::Knob::HostRenew);  // =1: the host path (A/B, tests)
  if (hr != nullptr && hr[0] == '1') return false;
  HIPCHECK(hipSetDevice(device_id_));
  const int L = tree->num_leaves();
  const size_t n = static_cast<size_t>(num_data_);
  if (uploaded_label_src_ != spec.label) {
    if (d_label_ == nullptr) d_label_ = Alloc<float>(n);
    HIPCHECK(hipMemcpy(d_label_, spec.label, sizeof(float) * n, hipMemcpyHostToDevice));
    uploaded_label_src_ = spec.label;
  }
  if (spec.weights != nullptr && renew_weight_src_ != spec.weights) {
    if (d_renew_weights_ == nullptr) d_renew_weights_ = Alloc<float>(n);
    HIPCHECK(hipMemcpy(d_renew_weights_, spec.weights, sizeof(float) * n, hipMemcpyHostToDevice));
    renew_weight_src_ = spec.weights;
  }
  if (d_renew_scratch_ == nullptr) {
    d_renew_scratch_ = Alloc<char>(dev::RenewScratchBytes(num_data_, config_->num_leaves));
    d_renew_off_ = Alloc<int64_t>(config_->num_leaves + 1);
    d_renew_out_ = Alloc<double>(config_->num_leaves);
  }
  // the leaves' row counts -> gathered offsets
  std::vector<dev::Leaf> leaves(L);
  HIPCHECK(hipMemcpyAsync(leaves.data(), d_leaves_, sizeof(dev::Leaf) * L, hipMemcpyDeviceToHost, stream_));
  HIPCHECK(hipStreamSynchronize(stream_));
  std::vector<int64_t> off(L + 1, 0);
  for (int l = 0; l < L; ++l) off[l + 1] = off[l] + leaves[l].count;
  HIPCHECK(hipMemcpyAsync(d_renew_off_, off.data(), sizeof(int64_t) * off.size(), hipMemcpyHostToDevice, stream_));
  dev::RenewArgs r{};
  r.leaves = d_leaves_;
  r.idx = d_idx_;
  r.tmp = d_tmp_;
  r.buf_stride = num_data_;
  r.label = d_label_;
  r.score = d_score_ + static_cast<size_t>(tree_id) * n;
  r.weights = spec.weights != nullptr ? d_renew_weights_ : nullptr;
  r.offsets = d_renew_off_;
  r.num_leaves = L;
  r.alpha = spec.alpha;
  r.out = d_renew_out_;
  r.scratch = d_renew_scratch_;
  dev::RenewLeafOutputs(r, off[L], stream_);
  std::vector<double> out(L);
  HIPCHECK(hipMemcpyAsync(out.data(), d_renew_out_, sizeof(double) * L, hipMemcpyDeviceToHost, stream_));
  HIPCHECK(hipStreamSynchronize(stream_));
  std::vector<int> nonzero(L, 1);
  for (int l = 0; l < L; ++l) {
    if (leaves[l].count <= 0) {
      out[l] = 0.0;
      nonzero[l] = 0;
    }
  }
  if (Network::num_machines() > 1) {
    out = Network::GlobalSum(out);
    nonzero = Network::GlobalSum(nonzero);
    for (int l = 0; l < L; ++l) out[l] /= nonzero[l];
  }
  for (int l = 0; l < L; ++l) tree->SetLeafOutput(l, out[l]);
  return true;
}

// ---------------------------------------------------------------- forced splits
// The reference's ForceSplits (serial_tree_learner.cpp) walks the forced-split JSON tree in
// BFS order before the leaf-wise loop: node k is split k, applied to the leaf that node's
// parent split created (a left child keeps its parent's leaf id, a right child of split k is
// leaf k + 1), as long as every forced split so far was valid.  That order and those leaves
// are static, so the schedule is built once: per node its inner feature, bin threshold and
// leaf, per split the node indices of its two children.
bool GPUTreeLearner::SetupForcedSplits() {
  const std::string text = has_forced_split_ ? forced_split_text_ : std::string();
  if (text == forced_text_built_ && (forced_ok_ || text.empty())) return forced_ok_;
  forced_text_built_ = text;
  forced_ok_ = false;
  if (args_.forced_n != 0) DestroyGraph();
  args_.forced_n = 0;
  if (!has_forced_split_) return false;
  std::vector<Json> nodes{forced_split_};
  std::vector<int32_t> feat, thr, leaf{0}, child;
  const int max_nodes = config_->num_leaves - 1;
  auto valid = [](const Json& n) { return n.is_object() && n.has("feature") && n.has("threshold"); };
  for (size_t i = 0; i < nodes.size() && static_cast<int>(i) < max_nodes; ++i) {
    const Json n = nodes[i];
    const int inner = data_->InnerFeatureIndex(n["feature"].int_value());
    feat.push_back(inner);
    thr.push_back(inner >= 0 ? static_cast<int32_t>(data_->BinThreshold(inner, n["threshold"].number_value())) : 0);
    int32_t lc = -1, rc = -1;
    if (n.has("left") && valid(n["left"])) {
      lc = static_cast<int32_t>(nodes.size());
      nodes.push_back(n["left"]);
      leaf.push_back(leaf[i]);
    }
    if (n.has("right") && valid(n["right"])) {
      rc = static_cast<int32_t>(nodes.size());
      nodes.push_back(n["right"]);
      leaf.push_back(static_cast<int32_t>(i) + 1);
    }
    child.push_back(lc);
    child.push_back(rc);
  }
  const int n = static_cast<int>(feat.size());
  for (auto& c : child) {
    if (c >= n) c = -1;  // beyond num_leaves - 1 splits
  }
  leaf.resize(n);
  // one int32 block: feat | thr | leaf | child[2n]
  std::vector<int32_t> blk;
  blk.insert(blk.end(), feat.begin(), feat.end());
  blk.insert(blk.end(), thr.begin(), thr.end());
  blk.insert(blk.end(), leaf.begin(), leaf.end());
  blk.insert(blk.end(), child.begin(), child.end());
  d_forced_i32_ = Alloc<int32_t>(blk.size());
  HIPCHECK(hipMemcpy(d_forced_i32_, blk.data(), sizeof(int32_t) * blk.size(), hipMemcpyHostToDevice));
  // feature-parallel: one block of records per rank (the owner of a node's feature fills its
  // own block; GatherFeatureBests gathers them)
  const int blocks = ForcedGathered() ? world_ : 1;
  d_forced_best_ = Alloc<dev::FeatureBest>(static_cast<size_t>(blocks) * n);
  d_forced_cat_ = Alloc<uint32_t>(static_cast<size_t>(blocks) * n * kMaxCatWords);
  const int mine = blocks > 1 ? rank_ : 0;
  args_.forced_feat = d_forced_i32_;
  args_.forced_thr = d_forced_i32_ + n;
  args_.forced_leaf = d_forced_i32_ + 2 * n;
  args_.forced_child = d_forced_i32_ + 3 * n;
  args_.forced_best = d_forced_best_ + static_cast<size_t>(mine) * n;
  args_.forced_cat = d_forced_cat_ + static_cast<size_t>(mine) * n * kMaxCatWords;
  args_.forced_world = blocks > 1 ? blocks : 0;
  args_.forced_all = d_forced_best_;
  args_.forced_cat_all = d_forced_cat_;
  args_.forced_n = n;
  forced_ok_ = true;
  DestroyGraph();  // (the captured tree holds the kernel arguments)
  return true;
}

// ---------------------------------------------------------------- binned rows
// Row-sparse training storage (reference MultiValSparseBin, src/io/multi_val_sparse_bin.hpp,
// chosen by Dataset::GetMultiBinFromSparseFeatures for sparse data): a histogram gather then
// reads a row's ~2-byte stored bins instead of its whole word row.  Chosen when a sample of
// rows stores at most a quarter of the bytes that way; needs <= 65535 histogram bins (16-bit entries)
// and a full histogram range per rank (not feature-parallel).  LGBM_AMD_SPARSE_ROWS=0/1
// forces the word matrix / the sparse lists (when allowed).
bool GPUTreeLearner::UseSparseRows(int wpr) const {
  if (total_bins_ > 65535 || num_data_ <= 0 || (distributed_ && mode_ == Mode::kFeature)) return false;
  if (const char* e = tuning::Get(tuning::Knob::SparseRows)) return e[0] == '1';
  const data_size_t step = std::max<data_size_t>(1, num_data_ / 65536);
  int64_t stored = 0, rows = 0;
  for (data_size_t r = 0; r < num_data_; r += step, ++rows) {
    for (int g = 0; g < num_groups_; ++g) stored += data_->group(g).Get(r) != 0 ? 1 : 0;
  }
  const double per_row = static_cast<double>(stored) / std::max<int64_t>(1, rows);
  // a stored bin costs about as much as a whole word of a word row (scattered 2-byte reads vs
  // one line per row): measured break-even near 4x fewer bytes (Bosch 190 stored bins per row vs
  // 238 words: word rows 22.8 vs sparse 28.2 ms/iter; Expo 14 vs 176: 54.3 vs 34.7)
  return (2.0 * per_row + 8.0) * 4.0 <= 4.0 * wpr;
}

// rows' stored bins (group_bin_boundary(g) + bin, bin != 0), ascending, as CSR lists; built
// in blocks of rows so each group column is read sequentially within a block
void GPUTreeLearner::UploadSparseRows() {
  const data_size_t n = num_data_;
  constexpr data_size_t kBlk = 1 << 15;
  const int nblk = static_cast<int>((n + kBlk - 1) / kBlk);
  std::vector<int64_t> ptr(static_cast<size_t>(n) + 1, 0);
#pragma omp parallel for schedule(dynamic)
  for (int b = 0; b < nblk; ++b) {
    const data_size_t r0 = static_cast<data_size_t>(b) * kBlk, r1 = std::min(n, r0 + kBlk);
    for (int g = 0; g < num_groups_; ++g) {
      const FeatureGroup& grp = data_->group(g);
      if (grp.sparse) {  // (the block's stored rows)
        auto k = std::lower_bound(grp.sp_rows.begin(), grp.sp_rows.end(), r0);
        for (; k != grp.sp_rows.end() && *k < r1; ++k) ptr[*k + 1] += 1;
        continue;
      }
      for (data_size_t r = r0; r < r1; ++r) ptr[r + 1] += grp.Get(r) != 0 ? 1 : 0;
    }
  }
  for (data_size_t r = 0; r < n; ++r) ptr[r + 1] += ptr[r];
  std::vector<uint16_t> ent(std::max<int64_t>(1, ptr[n]));
#pragma omp parallel for schedule(dynamic)
  for (int b = 0; b < nblk; ++b) {
    const data_size_t r0 = static_cast<data_size_t>(b) * kBlk, r1 = std::min(n, r0 + kBlk);
    std::vector<int64_t> cur(ptr.begin() + r0, ptr.begin() + r1);
    for (int g = 0; g < num_groups_; ++g) {
      const FeatureGroup& grp = data_->group(g);
      const uint32_t goff = static_cast<uint32_t>(data_->group_bin_boundary(g));
      if (grp.sparse) {
        size_t k = static_cast<size_t>(std::lower_bound(grp.sp_rows.begin(), grp.sp_rows.end(), r0) - grp.sp_rows.begin());
        for (; k < grp.sp_rows.size() && grp.sp_rows[k] < r1; ++k) {
          const data_size_t r = grp.sp_rows[k];
          ent[cur[r - r0]++] = static_cast<uint16_t>(goff + grp.ValAt(k));
        }
        continue;
      }
      for (data_size_t r = r0; r < r1; ++r) {
        const uint32_t v = grp.Get(r);
        if (v != 0) ent[cur[r - r0]++] = static_cast<uint16_t>(goff + v);
      }
    }
  }
  d_sp_ptr_ = Alloc<int64_t>(ptr.size());
  HIPCHECK(hipMemcpy(d_sp_ptr_, ptr.data(), sizeof(int64_t) * ptr.size(), hipMemcpyHostToDevice));
  d_sp_bin_ = Alloc<uint16_t>(ent.size());
  HIPCHECK(hipMemcpy(d_sp_bin_, ent.data(), sizeof(uint16_t) * ent.size(), hipMemcpyHostToDevice));
  // threads per row: a row of mean length fits the kSparsePer entries each thread loads up front
  const double mean = static_cast<double>(ptr[n]) / std::max<data_size_t>(1, n);
  sp_team_ = 4;
  while (sp_team_ < 64 && sp_team_ * dev::kSparsePerThread < mean) sp_team_ *= 2;
  Log::Info("device learner: row-sparse storage, %.2f stored bins per row (%d groups), %d threads per row", mean,
            num_groups_, sp_team_);
}

// row-major copy of a dataset's storage columns in this learner's layout (each group at its
// byte of the row, 8 or 16 bits; rows padded to whole 32-bit words)
std::vector<uint8_t> GPUTreeLearner::RowMajorBins(const Dataset* d, int row_words) const {
  const size_t row_bytes = static_cast<size_t>(row_words) * 4;
  const data_size_t n = d->num_data();
  const int ng = d->num_groups();
  std::vector<uint8_t> host(static_cast<size_t>(n) * row_bytes, 0);
  auto put = [&](uint8_t* row, int g, uint32_t v) {
    if (h_gnib_[g] != 0) row[h_gbyte_[g]] |= static_cast<uint8_t>((v & 15u) << ((h_gnib_[g] & 1) * 4));
    else if (!h_gwide_[g]) row[h_gbyte_[g]] = static_cast<uint8_t>(v);
    else reinterpret_cast<uint16_t*>(row + h_gbyte_[g])[0] = static_cast<uint16_t>(v);
  };
#pragma omp parallel for schedule(static)
  for (data_size_t r = 0; r < n; ++r) {
    uint8_t* row = host.data() + static_cast<size_t>(r) * row_bytes;
    for (int g = 0; g < ng; ++g) {
      if (!d->group(g).sparse) put(row, g, d->group(g).Get(r));
    }
  }
  // sparse groups: their stored rows (one group at a time: 4-bit neighbours share a byte)
  for (int g = 0; g < ng; ++g) {
    const FeatureGroup& grp = d->group(g);
    if (!grp.sparse) continue;
#pragma omp parallel for schedule(static)
    for (size_t k = 0; k < grp.sp_rows.size(); ++k) {
      put(host.data() + static_cast<size_t>(grp.sp_rows[k]) * row_bytes, g, grp.ValAt(k));
    }
  }
  return host;
}

}  // namespace lgbm_amd
