// Binned training data (host side).
//
// Layout: features that survive the trivial-feature filter are bundled by Exclusive
// Feature Bundling (EFB, reference src/io/dataset.cpp:97-313) into groups; each group
// is one dense column of "group bins".  Group bin 0 is shared by all member features
// at their most-frequent bin; feature j of the group owns group bins
// [bin_offsets[j], bin_offsets[j+1]) (reference include/LightGBM/feature_group.h:36-48,
// 153-165).  The same encoding is uploaded to HBM row-major by the device learner, so
// a histogram over group bins IS the concatenation of per-feature histograms with the
// reference's "offset" convention (bin 0 dropped when most_freq_bin == 0).
#pragma once

#include <algorithm>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_set>
#include <utility>
#include <vector>

#include "lgbm_amd/bin.h"
#include "lgbm_amd/config.h"
#include "lgbm_amd/meta.h"

namespace lgbm_amd {

class Metadata {
 public:
  Metadata() = default;
  void Init(data_size_t num_data, bool has_weight, bool has_query);
  void InitFromFile(const std::string& data_filename);  // side files .weight/.query/.init

  void SetLabel(const label_t* label, data_size_t len);
  void SetWeights(const label_t* weights, data_size_t len);
  void SetQuery(const int32_t* query, data_size_t len);  // query sizes (group counts)
  void SetQueryBoundaries(const std::vector<data_size_t>& boundaries);
  void SetInitScore(const double* init_score, int64_t len);
  void SetLabelAt(data_size_t i, label_t v) { label_[i] = v; }
  void SetWeightAt(data_size_t i, label_t v) { weights_[i] = v; }
  void SetQueryIdAt(data_size_t i, data_size_t q) { query_ids_tmp_[i] = q; }
  void FinishQueryIds();

  // keep rows [used_indices] (row sharding / subsets)
  void Subset(const Metadata& full, const data_size_t* used_indices, data_size_t n);
  void CheckOrPartition(data_size_t num_all_data, const std::vector<data_size_t>& used_indices);

  data_size_t num_data() const { return num_data_; }
  const label_t* label() const { return label_.data(); }
  const label_t* weights() const { return weights_.empty() ? nullptr : weights_.data(); }
  const data_size_t* query_boundaries() const { return query_boundaries_.empty() ? nullptr : query_boundaries_.data(); }
  data_size_t num_queries() const { return num_queries_; }
  const label_t* query_weights() const { return query_weights_.empty() ? nullptr : query_weights_.data(); }
  const double* init_score() const { return init_score_.empty() ? nullptr : init_score_.data(); }
  int64_t num_init_score() const { return static_cast<int64_t>(init_score_.size()); }
  std::vector<label_t>& mutable_label() { return label_; }

  void SaveBinary(std::string* out) const;  // (private V2 dataset files: still read)
  const char* LoadBinary(const char* p);
  // the reference's metadata block (metadata.cpp:471-531): num_data, num_weights, num_queries
  // (int32), labels, weights, query boundaries; init scores are not part of it
  size_t ReferenceBinarySize() const;
  void SaveReferenceBinary(std::string* out) const;
  void LoadReferenceBinary(const char* p, size_t size);

 private:
  void ComputeQueryWeights();
  data_size_t num_data_ = 0;
  std::vector<label_t> label_;
  std::vector<label_t> weights_;
  std::vector<data_size_t> query_boundaries_;
  std::vector<label_t> query_weights_;
  data_size_t num_queries_ = 0;
  std::vector<double> init_score_;
  std::vector<data_size_t> query_ids_tmp_;
};

struct FeatureGroup {
  std::vector<int> inner_features;      // inner feature indices in this group
  std::vector<uint32_t> bin_offsets;    // size nf + 1, bin_offsets[0] == 1
  int num_total_bin = 1;
  int bin_bytes = 1;                    // 1, 2 or 4 bytes per row (per stored entry when sparse)
  // storage: dense -- data holds num_data * bin_bytes, one group bin per row -- or sparse (the
  // reference's SparseBin, sparse_bin.hpp): only the rows whose group bin is not 0 (every member
  // feature at its most frequent bin), ascending in sp_rows, their bins in data.  Pushes to a
  // sparse group are buffered per thread (push_buf) and merged by Dataset::FinishLoad.
  bool sparse = false;
  std::vector<uint8_t> data;
  std::vector<data_size_t> sp_rows;
  std::vector<std::vector<std::pair<data_size_t, uint32_t>>> push_buf;  // [thread]

  inline uint32_t ValAt(size_t k) const {
    switch (bin_bytes) {
      case 1: return data[k];
      case 2: return reinterpret_cast<const uint16_t*>(data.data())[k];
      default: return reinterpret_cast<const uint32_t*>(data.data())[k];
    }
  }
  inline uint32_t Get(data_size_t row) const {
    if (sparse) {
      const auto it = std::lower_bound(sp_rows.begin(), sp_rows.end(), row);
      return (it == sp_rows.end() || *it != row) ? 0u : ValAt(static_cast<size_t>(it - sp_rows.begin()));
    }
    return ValAt(static_cast<size_t>(row));
  }
  inline void Set(data_size_t row, uint32_t v) {
    if (sparse) {
      SetSparse(row, v);
      return;
    }
    switch (bin_bytes) {
      case 1: data[row] = static_cast<uint8_t>(v); break;
      case 2: reinterpret_cast<uint16_t*>(data.data())[row] = static_cast<uint16_t>(v); break;
      default: reinterpret_cast<uint32_t*>(data.data())[row] = v; break;
    }
  }
  void SetSparse(data_size_t row, uint32_t v);  // (buffered: Dataset::FinishLoad merges)
  void MergePushes();                           // sparse: sort by row, last push of a row wins, drop 0
  // f(row, bin) for every row whose bin is not 0, ascending rows (dense: a scan of the column)
  template <typename Fn>
  void ForEachStored(data_size_t num_data, Fn f) const {
    if (sparse) {
      for (size_t k = 0; k < sp_rows.size(); ++k) f(sp_rows[k], ValAt(k));
      return;
    }
    for (data_size_t r = 0; r < num_data; ++r) {
      const uint32_t v = ValAt(static_cast<size_t>(r));
      if (v != 0) f(r, v);
    }
  }
};

class Dataset {
 public:
  Dataset() = default;
  explicit Dataset(data_size_t num_data) : num_data_(num_data) {}

  // --- construction -------------------------------------------------------------
  // Build bin mappers from a column-wise sample of non-zero values (values may be NaN)
  // and allocate storage for `num_data` rows.  Mirrors DatasetLoader::ConstructFromSampleData.
  void ConstructFromSample(std::vector<std::vector<double>>* sample_values,
                           std::vector<std::vector<int>>* sample_indices, int num_col, size_t total_sample_cnt,
                           data_size_t num_data, const Config& cfg,
                           const std::unordered_set<int>& categorical, const std::unordered_set<int>& ignored,
                           const std::vector<std::vector<double>>& forced_bins);
  // Build from already-computed bin mappers (distributed exchange / binary load)
  void ConstructFromBinMappers(std::vector<std::unique_ptr<BinMapper>>* mappers, data_size_t num_data,
                               const Config& cfg, std::vector<std::vector<int>>* sample_indices,
                               std::vector<std::vector<double>>* sample_values, size_t total_sample_cnt);
  // same bins / groups as `ref`, new rows (validation data)
  void CreateValid(const Dataset& ref, data_size_t num_data);
  // rows `idx` of `full`
  void CopySubrow(const Dataset& full, const data_size_t* idx, data_size_t n);

  void PushDenseRow(data_size_t row, const double* values, int ncol);
  void PushSparseRow(data_size_t row, const std::vector<std::pair<int, double>>& values);
  void PushColumnValue(data_size_t row, int real_col, double value);
  // every push is done: sparse groups merge their per-thread push buffers
  void FinishLoad();
  // storage of the groups: sparse when a group's non-zero share is at most kSparseGroupRate
  // (estimated from its features' bin mappers; LGBM_AMD_HOST_SPARSE=0 / 1 forces dense / sparse)
  static constexpr double kSparseGroupRate = 0.2;
  int num_sparse_groups() const;

  // --- queries --------------------------------------------------------------------
  data_size_t num_data() const { return num_data_; }
  int num_total_features() const { return num_total_features_; }
  int num_features() const { return num_features_; }
  int num_groups() const { return static_cast<int>(groups_.size()); }
  int label_idx() const { return label_idx_; }
  void set_label_idx(int i) { label_idx_ = i; }
  const std::vector<std::string>& feature_names() const { return feature_names_; }
  void set_feature_names(const std::vector<std::string>& names);
  std::vector<std::string> feature_infos() const;

  int RealFeatureIndex(int inner) const { return real_feature_idx_[inner]; }
  int InnerFeatureIndex(int real) const { return real < static_cast<int>(used_feature_map_.size()) ? used_feature_map_[real] : -1; }
  int Feature2Group(int inner) const { return feature2group_[inner]; }
  int Feature2SubFeature(int inner) const { return feature2subfeature_[inner]; }
  const BinMapper* FeatureBinMapper(int inner) const { return bin_mappers_[inner].get(); }
  int FeatureNumBin(int inner) const { return bin_mappers_[inner]->num_bin(); }
  const FeatureGroup& group(int g) const { return groups_[g]; }
  FeatureGroup& mutable_group(int g) { return groups_[g]; }
  uint64_t group_bin_boundary(int g) const { return group_bin_boundaries_[g]; }
  uint64_t num_total_bin() const { return group_bin_boundaries_.back(); }
  // offset of inner feature's histogram slice inside the leaf histogram (in bins)
  uint64_t FeatureHistOffset(int inner) const {
    int g = feature2group_[inner];
    return group_bin_boundaries_[g] + groups_[g].bin_offsets[feature2subfeature_[inner]];
  }
  // number of entries in the feature's histogram slice (num_bin - offset)
  int FeatureHistSize(int inner) const {
    int g = feature2group_[inner], s = feature2subfeature_[inner];
    return static_cast<int>(groups_[g].bin_offsets[s + 1] - groups_[g].bin_offsets[s]);
  }
  // raw feature bin of `row`, decoding the group-bin encoding
  inline uint32_t FeatureBin(int inner, data_size_t row) const {
    const FeatureGroup& g = groups_[feature2group_[inner]];
    int s = feature2subfeature_[inner];
    uint32_t gb = g.Get(row);
    const BinMapper* m = bin_mappers_[inner].get();
    if (gb < g.bin_offsets[s] || gb >= g.bin_offsets[s + 1]) return m->GetMostFreqBin();
    return gb - g.bin_offsets[s] + (m->GetMostFreqBin() == 0 ? 1 : 0);
  }

  // FeatureBin for rows read in ascending order (a leaf's rows, a score walk's chunk): a sparse
  // group's stored rows are walked forward from the last hit by galloping search instead of a
  // binary search over all of them per row (a row below the last one restarts the walk)
  struct BinReader {
    const FeatureGroup* g = nullptr;
    size_t k = 0;
    uint32_t lo = 0, hi = 0, mfb = 0, add = 0;
    inline uint32_t Get(data_size_t row) {
      uint32_t gb;
      if (!g->sparse) {
        gb = g->ValAt(static_cast<size_t>(row));
      } else {
        const std::vector<data_size_t>& r = g->sp_rows;
        const size_t n = r.size();
        if (k > 0 && r[k - 1] >= row) k = 0;
        size_t lo_i = k, hi_i = k, step = 1;
        while (hi_i < n && r[hi_i] < row) {
          lo_i = hi_i + 1;
          hi_i += step;
          step <<= 1;
        }
        if (hi_i > n) hi_i = n;
        k = static_cast<size_t>(std::lower_bound(r.begin() + lo_i, r.begin() + hi_i, row) - r.begin());
        gb = (k < n && r[k] == row) ? g->ValAt(k) : 0u;
      }
      if (gb < lo || gb >= hi) return mfb;
      return gb - lo + add;
    }
  };
  BinReader FeatureBinReader(int inner) const {
    BinReader b;
    const FeatureGroup& g = groups_[feature2group_[inner]];
    const int s = feature2subfeature_[inner];
    const BinMapper* m = bin_mappers_[inner].get();
    b.g = &g;
    b.lo = g.bin_offsets[s];
    b.hi = g.bin_offsets[s + 1];
    b.mfb = m->GetMostFreqBin();
    b.add = m->GetMostFreqBin() == 0 ? 1 : 0;
    return b;
  }

  double RealThreshold(int inner, uint32_t threshold) const { return bin_mappers_[inner]->BinToValue(threshold); }
  // feature value -> bin threshold for forced splits
  uint32_t BinThreshold(int inner, double threshold_double) const;
  bool CheckAlign(const Dataset& other) const;

  Metadata& metadata() { return metadata_; }
  const Metadata& metadata() const { return metadata_; }

  // --- CPU training kernels -----------------------------------------------------
  // Accumulate gradient/hessian histograms (double) of rows `indices[0..n)` (or all rows
  // when indices == nullptr) for groups with group_used[g] != 0.  hist has 2*num_total_bin entries.
  // col-wise (reference dataset.cpp:1283-1384): threads over groups, each walks its column;
  // row-wise (dataset.cpp:1046-1281, MultiValDenseBin): threads over row blocks of a row-major
  // copy (built on first use), private histograms merged over bin blocks
  // Row-wise mode: `scratch` holds the caller's per-thread private histograms -- each learner
  // owns its own, since one Dataset may train several boosters at once (reference: the
  // per-learner TrainingShareStates).  The row-major copy is built once, under a lock, and kept
  // for the Dataset's lifetime.
  struct RowWiseScratch {
    std::vector<std::vector<hist_t>> bufs;
  };
  void ConstructHistograms(const std::vector<int8_t>& group_used, const data_size_t* indices, data_size_t n,
                           const score_t* grad, const score_t* hess, hist_t* hist, bool row_wise = false,
                           RowWiseScratch* scratch = nullptr) const;
  // reconstruct the most-frequent-bin entry of a feature slice from the leaf totals
  void FixHistogram(int inner, double sum_grad, double sum_hess, hist_t* feature_hist) const;

  // --- persistence ----------------------------------------------------------------
  // Dataset binary files in the reference's format (src/io/dataset.cpp:890-992, read as
  // dataset_loader.cpp:273-525; src/io/dataset_binary.cpp): token, header, metadata, then one
  // block per feature group.  Files written here load in the reference and vice versa.
  void SaveBinaryFile(const std::string& path) const;
  // rank / num_machines / partition: keep this rank's rows (or whole queries) as the reference
  // does for a binary file under distributed training without pre_partition (Random(seed)
  // NextShort(0, num_machines) == rank per row / query); *used gets the kept global rows
  static std::unique_ptr<Dataset> LoadBinaryFile(const std::string& path, int rank = 0, int num_machines = 1,
                                                 bool partition = false, int seed = 0,
                                                 std::vector<data_size_t>* used = nullptr);
  static bool IsBinaryFile(const std::string& path);
  void DumpText(const std::string& path) const;

  // append the features of `other` (same rows) -- LGBM_DatasetAddFeaturesFrom
  void AddFeaturesFrom(const Dataset& other);

  // config snapshot used to build this dataset (needed by CreateValid / parameter checks)
  int max_bin() const { return max_bin_; }
  const std::vector<std::vector<double>>& forced_bins() const { return forced_bin_bounds_; }
  std::vector<int> FeatureNeedPushZeros() const { return need_push_zeros_; }

 private:
  void BuildGroups(const std::vector<std::vector<int>>& features_in_group);
  FeatureGroup NewGroup(const std::vector<int>& inner_features);  // offsets, width, storage
  static std::unique_ptr<Dataset> LoadPrivateBinary(const std::string& path);
  static std::unique_ptr<Dataset> LoadReferenceBinary(const std::string& path, int rank, int num_machines,
                                                      bool partition, int seed, std::vector<data_size_t>* used);
  void ConstructHistogramsRowWise(const std::vector<int8_t>& group_used, const data_size_t* indices, data_size_t n,
                                  const score_t* grad, const score_t* hess, hist_t* hist, RowWiseScratch* scratch) const;
  void BuildRowMajor() const;

 public:
  // learners in row-wise mode hold the row-major copy (a use count under row_major_mu_): the
  // last release frees it, so a Dataset whose learners chose col-wise (the auto threading
  // test builds the copy once) keeps no second copy of its bins (reference: the row-wise
  // multi-val bin is dropped when col-wise wins)
  void RetainRowMajor() const;
  void ReleaseRowMajor() const;

 private:
  mutable int row_major_users_ = 0;
  // row-wise histograms: every group's bin of a row, contiguous (bytes per group as stored);
  // built on first use under row_major_mu_ (concurrent learners on one Dataset), then read-only
  mutable std::vector<uint8_t> row_major_;
  mutable std::vector<uint32_t> row_goff_;  // byte offset of each group in a row
  mutable size_t row_stride_ = 0;
  std::unique_ptr<std::mutex> row_major_mu_ = std::make_unique<std::mutex>();

  data_size_t num_data_ = 0;
  int num_total_features_ = 0;
  int num_features_ = 0;
  int label_idx_ = 0;
  bool finished_ = false;
  std::vector<std::unique_ptr<BinMapper>> bin_mappers_;  // by inner feature
  std::vector<int> used_feature_map_;                    // real -> inner (-1 unused)
  std::vector<int> real_feature_idx_;                    // inner -> real
  std::vector<int> feature2group_, feature2subfeature_;
  std::vector<FeatureGroup> groups_;
  std::vector<uint64_t> group_bin_boundaries_;
  std::vector<int> need_push_zeros_;
  std::vector<std::string> feature_names_;
  std::vector<std::vector<double>> forced_bin_bounds_;
  int max_bin_ = 255;
  // dataset parameters the binary file records (reference dataset.h:676-692)
  int bin_construct_sample_cnt_ = 200000;
  int min_data_in_bin_ = 3;
  bool use_missing_ = true;
  bool zero_as_missing_ = false;
  std::vector<int32_t> max_bin_by_feature_;
  // per group: the reference multi-value group (EFB's second-round bundle of sparse leftovers,
  // reference feature_group.h:352-377) it was expanded from -- consecutive groups with one id
  // -- or -1.  Multi-value groups are stored here as singleton groups; the binary file writes
  // them back as the reference's one multi-value group.
  std::vector<int> group_mv_;
  Metadata metadata_;
};

}  // namespace lgbm_amd
