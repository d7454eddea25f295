// Dataset construction (bin finding + Exclusive Feature Bundling), row pushing, CPU
// histogram construction and binary persistence.
// EFB follows reference src/io/dataset.cpp:97-313 (greedy conflict-bounded grouping
// tried in two feature orders, smaller result kept, groups shuffled with an LCG seeded
// by num_data) so that inner feature order -- which feature_fraction sampling depends
// on -- matches the reference.  Multi-value (row-wise sparse) groups of the reference
// are stored here as singleton dense groups: a storage choice that does not change
// the model.
#include "lgbm_amd/dataset.h"

#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <sstream>

#include "lgbm_amd/common.h"
#include "lgbm_amd/log.h"
#include "lgbm_amd/network.h"
#include "lgbm_amd/random.h"
#include "lgbm_amd/tuning.h"

namespace lgbm_amd {

namespace {

int ConflictCount(const std::vector<bool>& mark, const int* idx, int n, data_size_t max_cnt) {
  int c = 0;
  for (int i = 0; i < n; ++i) {
    if (mark[idx[i]]) ++c;
    if (c > max_cnt) return -1;
  }
  return c;
}

void Mark(std::vector<bool>* mark, const int* idx, int n) {
  for (int i = 0; i < n; ++i) (*mark)[idx[i]] = true;
}

// rows of the sample whose bin differs from the most frequent bin (only needed when
// the zero bin is not the most frequent one)
std::vector<int> NonMostFreqRows(const BinMapper* m, int total, int n, const int* idx, const double* vals) {
  std::vector<int> out;
  if (m->GetDefaultBin() == m->GetMostFreqBin()) return out;
  int i = 0, j = 0;
  while (i < total) {
    if (j < n && idx[j] < i) {
      ++j;
    } else if (j < n && idx[j] == i) {
      if (m->ValueToBin(vals[j]) != m->GetMostFreqBin()) out.push_back(i);
      ++i;
    } else {
      out.push_back(i++);
    }
  }
  return out;
}

std::vector<std::vector<int>> GreedyGroups(const std::vector<std::unique_ptr<BinMapper>>& mappers,
                                           const std::vector<int>& order, int** sidx, const int* nper,
                                           int num_sample_col, data_size_t total_sample, data_size_t num_data,
                                           bool limit_256, bool is_sparse, std::vector<int8_t>* multi_val) {
  const int kMaxSearch = 100;
  const int kMaxBinPerGroup = 256;
  const data_size_t max_conflict = static_cast<data_size_t>(total_sample / 10000);
  multi_val->clear();
  Random rnd(num_data);
  std::vector<std::vector<int>> groups;
  std::vector<std::vector<bool>> marks;
  std::vector<data_size_t> used_rows, total_rows;
  std::vector<int> group_bins;
  auto extra_bins = [&](int f) { return mappers[f]->num_bin() + (mappers[f]->GetDefaultBin() == 0 ? -1 : 0); };

  for (int f : order) {
    const bool filtered = f >= num_sample_col;
    const data_size_t nz = filtered ? 0 : nper[f];
    std::vector<int> avail;
    for (int g = 0; g < static_cast<int>(groups.size()); ++g) {
      int nb = group_bins[g] + extra_bins(f);
      if (total_rows[g] + nz <= total_sample + max_conflict) {
        if (!limit_256 || nb <= kMaxBinPerGroup) avail.push_back(g);
      }
    }
    std::vector<int> search;
    if (!avail.empty()) {
      int last = static_cast<int>(avail.size()) - 1;
      auto picks = rnd.Sample(last, std::min(last, kMaxSearch - 1));
      search.push_back(avail.back());
      for (int p : picks) search.push_back(avail[p]);
    }
    int best = -1, best_conf = -1;
    for (int g : search) {
      const data_size_t rest = max_conflict - total_rows[g] + used_rows[g];
      const data_size_t c = filtered ? 0 : ConflictCount(marks[g], sidx[f], nper[f], rest);
      if (c >= 0 && c <= rest && c <= nz / 2) {
        best = g;
        best_conf = c;
        break;
      }
    }
    if (best >= 0) {
      groups[best].push_back(f);
      total_rows[best] += nz;
      used_rows[best] += nz - best_conf;
      if (!filtered) Mark(&marks[best], sidx[f], nper[f]);
      group_bins[best] += extra_bins(f);
    } else {
      groups.emplace_back(1, f);
      marks.emplace_back(total_sample, false);
      if (!filtered) Mark(&marks.back(), sidx[f], nper[f]);
      total_rows.push_back(nz);
      used_rows.push_back(nz);
      group_bins.push_back(1 + extra_bins(f));
    }
  }
  if (!is_sparse) {
    multi_val->assign(groups.size(), 0);
    return groups;
  }
  // second round: sparse leftovers go into one (multi-value) group
  std::vector<int> leftovers;
  std::vector<std::vector<int>> groups2;
  std::vector<std::vector<bool>> marks2;
  const double kDense = 0.4;
  for (int g = 0; g < static_cast<int>(groups.size()); ++g) {
    if (static_cast<double>(used_rows[g]) / total_sample >= kDense) {
      groups2.push_back(std::move(groups[g]));
      marks2.push_back(std::move(marks[g]));
    } else {
      for (int f : groups[g]) leftovers.push_back(f);
    }
  }
  groups = std::move(groups2);
  multi_val->assign(groups.size(), 0);
  if (!leftovers.empty()) {
    groups.emplace_back();
    std::vector<bool> m(total_sample, false);
    bool is_multi = limit_256;
    int conflicts = 0;
    for (int f : leftovers) {
      groups.back().push_back(f);
      if (!is_multi) {
        const int rest = max_conflict - conflicts;
        const int c = ConflictCount(m, sidx[f], nper[f], rest);
        conflicts += c;
        if (c < 0 || conflicts > max_conflict) {
          is_multi = true;
          continue;
        }
        Mark(&m, sidx[f], nper[f]);
      }
    }
    multi_val->push_back(is_multi ? 1 : 0);
  }
  return groups;
}

std::vector<std::vector<int>> BundleFeatures(const std::vector<std::unique_ptr<BinMapper>>& mappers,
                                             std::vector<std::vector<int>>* sample_indices,
                                             std::vector<std::vector<double>>* sample_values, int num_sample_col,
                                             data_size_t total_sample, const std::vector<int>& used,
                                             data_size_t num_data, bool limit_256, bool is_sparse,
                                             std::vector<int8_t>* multi_val) {
  std::vector<size_t> nz;
  for (int f : used) nz.push_back(f < num_sample_col ? (*sample_indices)[f].size() : 0);
  std::vector<int> by_cnt(used.size());
  for (size_t i = 0; i < used.size(); ++i) by_cnt[i] = static_cast<int>(i);
  std::stable_sort(by_cnt.begin(), by_cnt.end(), [&](int a, int b) { return nz[a] > nz[b]; });
  std::vector<int> order2;
  for (int i : by_cnt) order2.push_back(used[i]);

  std::vector<std::vector<int>> fixed(num_sample_col);
  std::vector<int*> sidx(num_sample_col, nullptr);
  std::vector<int> nper(num_sample_col, 0);
  for (int f = 0; f < num_sample_col; ++f) {
    sidx[f] = (*sample_indices)[f].data();
    nper[f] = static_cast<int>((*sample_indices)[f].size());
  }
  for (int f : used) {
    if (f >= num_sample_col) continue;
    auto r = NonMostFreqRows(mappers[f].get(), static_cast<int>(total_sample), nper[f], sidx[f],
                             (*sample_values)[f].data());
    if (!r.empty()) {
      fixed[f] = std::move(r);
      sidx[f] = fixed[f].data();
      nper[f] = static_cast<int>(fixed[f].size());
    }
  }
  std::vector<int8_t> mv1, mv2;
  auto g1 = GreedyGroups(mappers, used, sidx.data(), nper.data(), num_sample_col, total_sample, num_data,
                         limit_256, is_sparse, &mv1);
  auto g2 = GreedyGroups(mappers, order2, sidx.data(), nper.data(), num_sample_col, total_sample, num_data,
                         limit_256, is_sparse, &mv2);
  if (g1.size() > g2.size()) {
    g1 = g2;
    mv1 = mv2;
  }
  const int ng = static_cast<int>(g1.size());
  Random shuf(num_data);
  for (int i = 0; i < ng - 1; ++i) {
    int j = shuf.NextShort(i + 1, ng);
    std::swap(g1[i], g1[j]);
    std::swap(mv1[i], mv1[j]);
  }
  *multi_val = mv1;
  return g1;
}

}  // namespace

void Dataset::ConstructFromSample(std::vector<std::vector<double>>* sample_values,
                                  std::vector<std::vector<int>>* sample_indices, int num_col,
                                  size_t total_sample_cnt, data_size_t num_data, const Config& cfg,
                                  const std::unordered_set<int>& categorical, const std::unordered_set<int>& ignored,
                                  const std::vector<std::vector<double>>& forced_bins) {
  num_data_ = num_data;
  std::vector<std::unique_ptr<BinMapper>> mappers(num_col);
  if (!cfg.max_bin_by_feature.empty()) {
    LGBM_CHECK_EQ(static_cast<int>(cfg.max_bin_by_feature.size()), num_col);
  }
  const data_size_t filter_cnt =
      static_cast<data_size_t>(static_cast<double>(cfg.min_data_in_leaf * total_sample_cnt) / num_data);
  std::string err;
  common::OmpErrors errors;
  // distributed: each rank bins a contiguous block of columns from its local sample and
  // the serialized mappers are allgathered, so every rank ends with identical bins
  // (reference dataset_loader.cpp:680-760)
  const int nm = Network::num_machines();
  const int rank = Network::rank();
  int col_begin = 0, col_end = num_col;
  if (nm > 1) {
    const int step = (num_col + nm - 1) / nm;
    col_begin = std::min(num_col, step * rank);
    col_end = std::min(num_col, col_begin + step);
  }
#pragma omp parallel for schedule(guided)
  for (int i = col_begin; i < col_end; ++i) {
    if (ignored.count(i)) continue;
    BinType t = BinType::Numerical;
    if (categorical.count(i)) {
      t = BinType::Categorical;
      if (!cfg.monotone_constraints.empty() && cfg.monotone_constraints[i] != 0) {
#pragma omp critical
        err = "The output cannot be monotone with respect to categorical features";
        continue;
      }
    }
    mappers[i].reset(new BinMapper());
    int mb = cfg.max_bin_by_feature.empty() ? cfg.max_bin : cfg.max_bin_by_feature[i];
    std::vector<double> vals = (*sample_values)[i];
    static const std::vector<double> kNoForced;
    const std::vector<double>& fb = i < static_cast<int>(forced_bins.size()) ? forced_bins[i] : kNoForced;
    errors.Run([&] {
      mappers[i]->FindBin(vals.data(), static_cast<int>(vals.size()), total_sample_cnt, mb, cfg.min_data_in_bin,
                          filter_cnt, cfg.feature_pre_filter, t, cfg.use_missing, cfg.zero_as_missing, fb);
    });
  }
  errors.Check();
  if (!err.empty()) Log::Fatal("%s", err.c_str());
  if (nm > 1) {
    // wire: per column [int8 present][mapper bytes]
    std::string mine;
    for (int i = col_begin; i < col_end; ++i) {
      const char present = mappers[i] != nullptr ? 1 : 0;
      mine.push_back(present);
      if (present) {
        std::string b(mappers[i]->SizesInByte(), '\0');
        mappers[i]->CopyTo(&b[0]);
        const uint64_t len = b.size();
        mine.append(reinterpret_cast<const char*>(&len), sizeof(len));
        mine += b;
      }
    }
    auto sizes = Network::GlobalArray<comm_size_t>(static_cast<comm_size_t>(mine.size()));
    std::vector<comm_size_t> starts(nm, 0);
    for (int r = 1; r < nm; ++r) starts[r] = starts[r - 1] + sizes[r - 1];
    std::string all(static_cast<size_t>(starts[nm - 1] + sizes[nm - 1]), '\0');
    Network::Allgather(&mine[0], starts.data(), sizes.data(), &all[0], static_cast<comm_size_t>(all.size()));
    const int step = (num_col + nm - 1) / nm;
    for (int r = 0; r < nm; ++r) {
      const char* p = all.data() + starts[r];
      const int b = std::min(num_col, step * r), e = std::min(num_col, b + step);
      for (int i = b; i < e; ++i) {
        const char present = *p++;
        if (!present) {
          mappers[i].reset();
          continue;
        }
        uint64_t len;
        std::memcpy(&len, p, sizeof(len));
        p += sizeof(len);
        mappers[i].reset(new BinMapper());
        mappers[i]->CopyFrom(p);
        p += len;
      }
    }
  }
  forced_bin_bounds_ = forced_bins;
  ConstructFromBinMappers(&mappers, num_data, cfg, sample_indices, sample_values, total_sample_cnt);
}

void Dataset::ConstructFromBinMappers(std::vector<std::unique_ptr<BinMapper>>* mappers, data_size_t num_data,
                                      const Config& cfg, std::vector<std::vector<int>>* sample_indices,
                                      std::vector<std::vector<double>>* sample_values, size_t total_sample_cnt) {
  num_data_ = num_data;
  max_bin_ = cfg.max_bin;
  num_total_features_ = static_cast<int>(mappers->size());
  std::vector<int> used;
  for (int i = 0; i < num_total_features_; ++i) {
    if ((*mappers)[i] != nullptr && !(*mappers)[i]->is_trivial()) used.push_back(i);
  }
  if (used.empty()) Log::Warning("There are no meaningful features, as all feature values are constant.");
  std::vector<std::vector<int>> fig;
  std::vector<int8_t> multi_val(used.size(), 0);
  for (int f : used) fig.emplace_back(1, f);
  const bool can_bundle = sample_indices != nullptr && sample_values != nullptr &&
                          static_cast<int>(sample_indices->size()) > 0;
  const int nm = Network::num_machines();
  if (cfg.enable_bundle && !used.empty() && can_bundle && (nm <= 1 || Network::rank() == 0)) {
    fig = BundleFeatures(*mappers, sample_indices, sample_values, static_cast<int>(sample_indices->size()),
                         static_cast<data_size_t>(total_sample_cnt), used, num_data, cfg.device_type == "gpu",
                         cfg.is_enable_sparse, &multi_val);
  }
  if (nm > 1) {
    // bundling depends on the sample, which is rank-local: every rank takes rank 0's groups so
    // the feature layout (and every histogram offset) is the same everywhere
    std::vector<int32_t> wire;  // [groups] then per group [size][multi][features...]
    wire.push_back(static_cast<int32_t>(fig.size()));
    for (size_t g = 0; g < fig.size(); ++g) {
      wire.push_back(static_cast<int32_t>(fig[g].size()));
      wire.push_back(multi_val[g]);
      wire.insert(wire.end(), fig[g].begin(), fig[g].end());
    }
    const comm_size_t mine = Network::rank() == 0 ? static_cast<comm_size_t>(sizeof(int32_t) * wire.size()) : 0;
    auto sizes = Network::GlobalArray<comm_size_t>(mine);
    std::vector<comm_size_t> starts(nm, 0);
    for (int r = 1; r < nm; ++r) starts[r] = starts[r - 1] + sizes[r - 1];
    std::vector<int32_t> got(sizes[0] / sizeof(int32_t));
    Network::Allgather(reinterpret_cast<char*>(wire.data()), starts.data(), sizes.data(),
                       reinterpret_cast<char*>(got.data()), sizes[0]);
    fig.clear();
    multi_val.clear();
    size_t p = 1;
    for (int32_t g = 0; g < got[0]; ++g) {
      const int n = got[p++];
      multi_val.push_back(static_cast<int8_t>(got[p++]));
      fig.emplace_back(got.begin() + p, got.begin() + p + n);
      p += n;
    }
  }
  std::vector<int> group_mv;
  {
    // multi-value groups are stored as singleton dense groups (same inner feature order)
    std::vector<std::vector<int>> expanded;
    int mv_id = 0;
    for (size_t g = 0; g < fig.size(); ++g) {
      if (multi_val[g]) {
        for (int f : fig[g]) {
          expanded.emplace_back(1, f);
          group_mv.push_back(mv_id);
        }
        ++mv_id;
      } else {
        expanded.push_back(fig[g]);
        group_mv.push_back(-1);
      }
    }
    fig = std::move(expanded);
  }
  bin_construct_sample_cnt_ = cfg.bin_construct_sample_cnt;
  min_data_in_bin_ = cfg.min_data_in_bin;
  use_missing_ = cfg.use_missing;
  zero_as_missing_ = cfg.zero_as_missing;
  max_bin_by_feature_.assign(cfg.max_bin_by_feature.begin(), cfg.max_bin_by_feature.end());
  // inner feature numbering follows group order
  used_feature_map_.assign(num_total_features_, -1);
  real_feature_idx_.clear();
  feature2group_.clear();
  feature2subfeature_.clear();
  bin_mappers_.clear();
  for (size_t g = 0; g < fig.size(); ++g) {
    for (size_t j = 0; j < fig[g].size(); ++j) {
      int real = fig[g][j];
      used_feature_map_[real] = static_cast<int>(real_feature_idx_.size());
      real_feature_idx_.push_back(real);
      feature2group_.push_back(static_cast<int>(g));
      feature2subfeature_.push_back(static_cast<int>(j));
      bin_mappers_.emplace_back((*mappers)[real].release());
    }
  }
  num_features_ = static_cast<int>(real_feature_idx_.size());
  std::vector<std::vector<int>> inner_groups;
  int k = 0;
  for (auto& g : fig) {
    inner_groups.emplace_back();
    for (size_t j = 0; j < g.size(); ++j) inner_groups.back().push_back(k++);
  }
  BuildGroups(inner_groups);
  group_mv_ = group_mv;
  if (feature_names_.empty()) {
    for (int i = 0; i < num_total_features_; ++i) feature_names_.push_back("Column_" + std::to_string(i));
  }
}

FeatureGroup Dataset::NewGroup(const std::vector<int>& fs) {
  FeatureGroup g;
  g.inner_features = fs;
  g.bin_offsets.push_back(1);
  int total = 1;
  for (int f : fs) {
    int nb = bin_mappers_[f]->num_bin();
    if (bin_mappers_[f]->GetMostFreqBin() == 0) nb -= 1;
    total += nb;
    g.bin_offsets.push_back(static_cast<uint32_t>(total));
    if (bin_mappers_[f]->GetDefaultBin() != bin_mappers_[f]->GetMostFreqBin()) need_push_zeros_.push_back(f);
  }
  g.num_total_bin = total;
  g.bin_bytes = total <= 256 ? 1 : (total <= 65536 ? 2 : 4);
  // sparse storage when at most kSparseGroupRate of the rows can hold a non-zero group bin
  // (the members' shares outside their most frequent bins, summed: an upper bound)
  double nonzero = 0.0;
  for (int f : fs) nonzero += 1.0 - bin_mappers_[f]->sparse_rate();
  g.sparse = nonzero <= kSparseGroupRate;
  if (const char* e = tuning::Get(tuning::Knob::HostSparse)) g.sparse = e[0] == '1';
  if (g.sparse) {
    g.push_buf.resize(static_cast<size_t>(std::max(omp_get_max_threads(), omp_get_num_procs())));
  } else {
    g.data.assign(static_cast<size_t>(num_data_) * g.bin_bytes, 0);
  }
  return g;
}

void Dataset::BuildGroups(const std::vector<std::vector<int>>& features_in_group) {
  groups_.clear();
  need_push_zeros_.clear();
  for (auto& fs : features_in_group) groups_.push_back(NewGroup(fs));
  group_mv_.assign(groups_.size(), -1);
  group_bin_boundaries_.assign(1, 0);
  for (auto& g : groups_) group_bin_boundaries_.push_back(group_bin_boundaries_.back() + g.num_total_bin);
}

void FeatureGroup::SetSparse(data_size_t row, uint32_t v) {
  static std::mutex overflow_mu;  // (a thread id beyond the buffers: shared, locked)
  const size_t t = static_cast<size_t>(omp_get_thread_num());
  if (t < push_buf.size()) {
    push_buf[t].emplace_back(row, v);
  } else {
    std::lock_guard<std::mutex> lock(overflow_mu);
    push_buf[0].emplace_back(row, v);
  }
}

void FeatureGroup::MergePushes() {
  if (!sparse) return;
  std::vector<std::pair<data_size_t, uint32_t>> all;
  size_t total = sp_rows.size();
  for (const auto& b : push_buf) total += b.size();
  all.reserve(total);
  for (size_t k = 0; k < sp_rows.size(); ++k) all.emplace_back(sp_rows[k], ValAt(k));  // (earlier merges)
  for (auto& b : push_buf) {
    all.insert(all.end(), b.begin(), b.end());
    std::vector<std::pair<data_size_t, uint32_t>>().swap(b);
  }
  // a row's pushes come from one thread, in push order: after a stable sort by row the last
  // one is the value a dense column would hold
  std::stable_sort(all.begin(), all.end(),
                   [](const std::pair<data_size_t, uint32_t>& x, const std::pair<data_size_t, uint32_t>& y) {
                     return x.first < y.first;
                   });
  sp_rows.clear();
  data.clear();
  sp_rows.reserve(all.size());
  data.reserve(all.size() * bin_bytes);
  for (size_t k = 0; k < all.size(); ++k) {
    if (k + 1 < all.size() && all[k + 1].first == all[k].first) continue;
    if (all[k].second == 0) continue;
    sp_rows.push_back(all[k].first);
    const uint32_t v = all[k].second;
    data.insert(data.end(), reinterpret_cast<const uint8_t*>(&v), reinterpret_cast<const uint8_t*>(&v) + bin_bytes);
  }
}

void Dataset::FinishLoad() {
  for (auto& g : groups_) g.MergePushes();
  finished_ = true;
}

int Dataset::num_sparse_groups() const {
  int n = 0;
  for (const auto& g : groups_) n += g.sparse ? 1 : 0;
  return n;
}

void Dataset::CreateValid(const Dataset& ref, data_size_t num_data) {
  num_data_ = num_data;
  num_total_features_ = ref.num_total_features_;
  num_features_ = ref.num_features_;
  label_idx_ = ref.label_idx_;
  used_feature_map_ = ref.used_feature_map_;
  real_feature_idx_ = ref.real_feature_idx_;
  feature2group_ = ref.feature2group_;
  feature2subfeature_ = ref.feature2subfeature_;
  feature_names_ = ref.feature_names_;
  forced_bin_bounds_ = ref.forced_bin_bounds_;
  max_bin_ = ref.max_bin_;
  bin_construct_sample_cnt_ = ref.bin_construct_sample_cnt_;
  min_data_in_bin_ = ref.min_data_in_bin_;
  use_missing_ = ref.use_missing_;
  zero_as_missing_ = ref.zero_as_missing_;
  max_bin_by_feature_ = ref.max_bin_by_feature_;
  bin_mappers_.clear();
  for (auto& m : ref.bin_mappers_) bin_mappers_.emplace_back(new BinMapper(*m));
  std::vector<std::vector<int>> fig;
  for (auto& g : ref.groups_) fig.push_back(g.inner_features);
  BuildGroups(fig);
  group_mv_ = ref.group_mv_;
}

void Dataset::CopySubrow(const Dataset& full, const data_size_t* idx, data_size_t n) {
  CreateValid(full, n);
  std::vector<data_size_t> new_of;  // sparse groups: full row -> subset row (-1: not taken)
  bool ascending = true;
  for (data_size_t i = 1; i < n && ascending; ++i) ascending = idx[i] > idx[i - 1];
  for (size_t g = 0; g < groups_.size(); ++g) {
    const auto& src = full.groups_[g];
    auto& dst = groups_[g];
    if (dst.sparse != src.sparse) {  // (the subset keeps the full dataset's storage)
      dst.sparse = src.sparse;
      dst.data.clear();
      dst.push_buf.clear();
      if (!dst.sparse) dst.data.assign(static_cast<size_t>(n) * dst.bin_bytes, 0);
    }
    if (src.sparse) {
      if (new_of.empty()) {
        new_of.assign(static_cast<size_t>(full.num_data_), -1);
        for (data_size_t i = 0; i < n; ++i) new_of[idx[i]] = i;
      }
      std::vector<std::pair<data_size_t, uint32_t>> kept;
      src.ForEachStored(full.num_data_, [&](data_size_t r, uint32_t v) {
        if (new_of[r] >= 0) kept.emplace_back(new_of[r], v);
      });
      if (!ascending) std::sort(kept.begin(), kept.end());
      dst.sp_rows.resize(kept.size());
      dst.data.assign(kept.size() * dst.bin_bytes, 0);
      for (size_t k = 0; k < kept.size(); ++k) {
        dst.sp_rows[k] = kept[k].first;
        std::memcpy(dst.data.data() + k * dst.bin_bytes, &kept[k].second, dst.bin_bytes);  // (little endian)
      }
      continue;
    }
#pragma omp parallel for schedule(static)
    for (data_size_t i = 0; i < n; ++i) {
      std::memcpy(dst.data.data() + static_cast<size_t>(i) * dst.bin_bytes,
                  src.data.data() + static_cast<size_t>(idx[i]) * src.bin_bytes, dst.bin_bytes);
    }
  }
  metadata_.Subset(full.metadata_, idx, n);
  finished_ = true;
}

void Dataset::set_feature_names(const std::vector<std::string>& names) {
  if (names.empty()) return;
  if (static_cast<int>(names.size()) != num_total_features_ && num_total_features_ > 0) {
    Log::Fatal("Size of feature_names error, should be %d, got %d", num_total_features_,
               static_cast<int>(names.size()));
  }
  feature_names_.clear();
  for (auto n : names) {
    // the model format is whitespace-separated: replace blanks
    for (auto& c : n) {
      if (c == ' ' || c == '\t' || c == '\n' || c == '\r') c = '_';
    }
    feature_names_.push_back(n);
  }
}

std::vector<std::string> Dataset::feature_infos() const {
  std::vector<std::string> out;
  for (int i = 0; i < num_total_features_; ++i) {
    int inner = used_feature_map_[i];
    out.push_back(inner < 0 ? std::string("none") : bin_mappers_[inner]->bin_info_string());
  }
  return out;
}

void Dataset::PushColumnValue(data_size_t row, int real_col, double value) {
  if (real_col >= num_total_features_) return;
  int inner = used_feature_map_[real_col];
  if (inner < 0) return;
  const BinMapper* m = bin_mappers_[inner].get();
  uint32_t bin = m->ValueToBin(value);
  if (bin == m->GetMostFreqBin()) return;
  if (m->GetMostFreqBin() == 0) bin -= 1;
  FeatureGroup& g = groups_[feature2group_[inner]];
  g.Set(row, bin + g.bin_offsets[feature2subfeature_[inner]]);
}

void Dataset::PushDenseRow(data_size_t row, const double* values, int ncol) {
  const int n = std::min(ncol, num_total_features_);
  for (int i = 0; i < n; ++i) PushColumnValue(row, i, values[i]);
}

void Dataset::PushSparseRow(data_size_t row, const std::vector<std::pair<int, double>>& values) {
  if (need_push_zeros_.empty()) {
    for (auto& kv : values) PushColumnValue(row, kv.first, kv.second);
    return;
  }
  std::vector<char> added(num_features_, 0);
  for (auto& kv : values) {
    if (kv.first >= num_total_features_) continue;
    int inner = used_feature_map_[kv.first];
    if (inner >= 0) added[inner] = 1;
    PushColumnValue(row, kv.first, kv.second);
  }
  for (int inner : need_push_zeros_) {
    if (!added[inner]) PushColumnValue(row, real_feature_idx_[inner], 0.0);
  }
}

uint32_t Dataset::BinThreshold(int inner, double threshold_double) const {
  const BinMapper* m = bin_mappers_[inner].get();
  uint32_t b = m->ValueToBin(threshold_double);
  // ValueToBin gives the bin containing the value; the split threshold is the bin whose
  // upper bound is >= value
  return b;
}

bool Dataset::CheckAlign(const Dataset& o) const {
  if (num_features_ != o.num_features_ || num_total_features_ != o.num_total_features_ ||
      label_idx_ != o.label_idx_) {
    return false;
  }
  for (int i = 0; i < num_features_; ++i) {
    if (!bin_mappers_[i]->CheckAlign(*o.bin_mappers_[i])) return false;
  }
  return true;
}

void Dataset::BuildRowMajor() const {
  std::lock_guard<std::mutex> lock(*row_major_mu_);
  if (row_stride_ > 0 || groups_.empty()) return;
  row_goff_.assign(groups_.size(), 0);
  size_t off = 0;
  for (size_t g = 0; g < groups_.size(); ++g) {
    row_goff_[g] = static_cast<uint32_t>(off);
    off += groups_[g].bin_bytes;
  }
  row_stride_ = off;
  row_major_.assign(static_cast<size_t>(num_data_) * row_stride_, 0);
#pragma omp parallel for schedule(static)
  for (data_size_t r = 0; r < num_data_; ++r) {
    uint8_t* dst = row_major_.data() + static_cast<size_t>(r) * row_stride_;
    for (size_t g = 0; g < groups_.size(); ++g) {
      const FeatureGroup& grp = groups_[g];
      if (grp.sparse) continue;
      std::memcpy(dst + row_goff_[g], grp.data.data() + static_cast<size_t>(r) * grp.bin_bytes, grp.bin_bytes);
    }
  }
  for (size_t g = 0; g < groups_.size(); ++g) {  // sparse groups: their stored rows only
    const FeatureGroup& grp = groups_[g];
    if (!grp.sparse) continue;
#pragma omp parallel for schedule(static)
    for (size_t k = 0; k < grp.sp_rows.size(); ++k) {
      std::memcpy(row_major_.data() + static_cast<size_t>(grp.sp_rows[k]) * row_stride_ + row_goff_[g],
                  grp.data.data() + k * grp.bin_bytes, grp.bin_bytes);
    }
  }
}

void Dataset::RetainRowMajor() const {
  std::lock_guard<std::mutex> lock(*row_major_mu_);
  ++row_major_users_;
}

void Dataset::ReleaseRowMajor() const {
  std::lock_guard<std::mutex> lock(*row_major_mu_);
  if (row_major_users_ > 0 && --row_major_users_ == 0) {
    std::vector<uint8_t>().swap(row_major_);
    row_stride_ = 0;
  }
}

void Dataset::ConstructHistogramsRowWise(const std::vector<int8_t>& group_used, const data_size_t* indices,
                                         data_size_t n, const score_t* grad, const score_t* hess,
                                         hist_t* hist, RowWiseScratch* scratch) const {
  BuildRowMajor();
  RowWiseScratch local;
  std::vector<std::vector<hist_t>>& row_bufs_ = (scratch != nullptr ? scratch : &local)->bufs;
  std::vector<int> used;
  for (int g = 0; g < num_groups(); ++g) {
    if (group_used[g]) used.push_back(g);
  }
  if (used.empty()) return;
  const size_t nb = 2 * static_cast<size_t>(num_total_bin());
  // row blocks of at least 1024 rows, one private histogram per block
  const int nt = std::max(1, std::min(omp_get_max_threads(), static_cast<int>((n + 1023) / 1024)));
  if (static_cast<int>(row_bufs_.size()) < nt) row_bufs_.resize(nt);
  for (int t = 0; t < nt; ++t) {
    if (row_bufs_[t].size() != nb) row_bufs_[t].assign(nb, 0.0);
  }
  const bool narrow = std::all_of(used.begin(), used.end(), [&](int g) { return groups_[g].bin_bytes == 1; });
#pragma omp parallel for schedule(static, 1) num_threads(nt)
  for (int t = 0; t < nt; ++t) {
    hist_t* h = row_bufs_[t].data();
    for (int g : used) std::fill(h + 2 * group_bin_boundaries_[g], h + 2 * group_bin_boundaries_[g + 1], 0.0);
    const data_size_t i0 = static_cast<data_size_t>(static_cast<int64_t>(n) * t / nt);
    const data_size_t i1 = static_cast<data_size_t>(static_cast<int64_t>(n) * (t + 1) / nt);
    for (data_size_t i = i0; i < i1; ++i) {
      const data_size_t r = indices ? indices[i] : i;
      const uint8_t* row = row_major_.data() + static_cast<size_t>(r) * row_stride_;
      const double g = grad[r], hs = hess[r];
      if (narrow) {
        for (int grp : used) {
          const size_t b = 2 * (group_bin_boundaries_[grp] + row[row_goff_[grp]]);
          h[b] += g;
          h[b + 1] += hs;
        }
      } else {
        for (int grp : used) {
          const uint8_t* p = row + row_goff_[grp];
          const int bytes = groups_[grp].bin_bytes;
          const uint32_t v = bytes == 1 ? *p : bytes == 2 ? *reinterpret_cast<const uint16_t*>(p)
                                                          : *reinterpret_cast<const uint32_t*>(p);
          const size_t b = 2 * (group_bin_boundaries_[grp] + v);
          h[b] += g;
          h[b + 1] += hs;
        }
      }
    }
  }
  // merge the private histograms, threads over bin blocks of the used groups (fixed block
  // order per bin: the sums do not depend on the thread schedule)
  std::vector<std::pair<size_t, size_t>> ranges;
  for (int g : used) {
    const size_t lo = 2 * group_bin_boundaries_[g], hi = 2 * group_bin_boundaries_[g + 1];
    for (size_t b = lo; b < hi; b += 1024) ranges.emplace_back(b, std::min(hi, b + 1024));
  }
#pragma omp parallel for schedule(static)
  for (int k = 0; k < static_cast<int>(ranges.size()); ++k) {
    for (size_t b = ranges[k].first; b < ranges[k].second; ++b) {
      double v = 0.0;
      for (int t = 0; t < nt; ++t) v += row_bufs_[t][b];
      hist[b] = v;
    }
  }
}

void Dataset::ConstructHistograms(const std::vector<int8_t>& group_used, const data_size_t* indices,
                                  data_size_t n, const score_t* grad, const score_t* hess, hist_t* hist,
                                  bool row_wise, RowWiseScratch* scratch) const {
  if (row_wise) {
    ConstructHistogramsRowWise(group_used, indices, n, grad, hess, hist, scratch);
    return;
  }
  const int ng = num_groups();
  // gather gradients once in leaf order (the reference's "ordered gradients")
  std::vector<score_t> og, oh;
  const score_t* pg = grad;
  const score_t* ph = hess;
  if (indices != nullptr) {
    og.resize(n);
    oh.resize(n);
#pragma omp parallel for schedule(static) if (n >= 16384)
    for (data_size_t i = 0; i < n; ++i) {
      og[i] = grad[indices[i]];
      oh[i] = hess[indices[i]];
    }
    pg = og.data();
    ph = oh.data();
  }
  bool leaf_ascending = true;  // (sparse groups: merge walk of the leaf's rows)
  if (indices != nullptr && num_sparse_groups() > 0) {
    for (data_size_t i = 1; i < n && leaf_ascending; ++i) leaf_ascending = indices[i] > indices[i - 1];
  }
#pragma omp parallel for schedule(dynamic, 1)
  for (int g = 0; g < ng; ++g) {
    if (!group_used[g]) continue;
    const FeatureGroup& grp = groups_[g];
    hist_t* h = hist + 2 * group_bin_boundaries_[g];
    std::fill(h, h + 2 * grp.num_total_bin, 0.0);
    if (grp.sparse) {
      // the stored rows only (reference SparseBin::ConstructHistogram): all rows -- every entry;
      // a leaf -- a merge walk of its ascending rows with the entries, or a search per row
      const size_t nnz = grp.sp_rows.size();
      if (indices == nullptr) {
        for (size_t k = 0; k < nnz; ++k) {
          const uint32_t b = grp.ValAt(k);
          h[2 * b] += pg[grp.sp_rows[k]];
          h[2 * b + 1] += ph[grp.sp_rows[k]];
        }
      } else if (leaf_ascending) {
        size_t k = 0;
        for (data_size_t i = 0; i < n && k < nnz; ++i) {
          const data_size_t r = indices[i];
          if (grp.sp_rows[k] < r) {
            k = static_cast<size_t>(std::lower_bound(grp.sp_rows.begin() + k, grp.sp_rows.end(), r) - grp.sp_rows.begin());
            if (k >= nnz) break;
          }
          if (grp.sp_rows[k] == r) {
            const uint32_t b = grp.ValAt(k);
            h[2 * b] += pg[i];
            h[2 * b + 1] += ph[i];
            ++k;
          }
        }
      } else {
        for (data_size_t i = 0; i < n; ++i) {
          const uint32_t b = grp.Get(indices[i]);
          if (b == 0) continue;
          h[2 * b] += pg[i];
          h[2 * b + 1] += ph[i];
        }
      }
    } else if (grp.bin_bytes == 1) {
      const uint8_t* col = grp.data.data();
      if (indices) {
        for (data_size_t i = 0; i < n; ++i) {
          const uint32_t b = col[indices[i]];
          h[2 * b] += pg[i];
          h[2 * b + 1] += ph[i];
        }
      } else {
        for (data_size_t i = 0; i < n; ++i) {
          const uint32_t b = col[i];
          h[2 * b] += pg[i];
          h[2 * b + 1] += ph[i];
        }
      }
    } else {
      for (data_size_t i = 0; i < n; ++i) {
        const data_size_t r = indices ? indices[i] : i;
        const uint32_t b = grp.Get(r);
        h[2 * b] += pg[i];
        h[2 * b + 1] += ph[i];
      }
    }
  }
}

void Dataset::FixHistogram(int inner, double sum_grad, double sum_hess, hist_t* data) const {
  const BinMapper* m = bin_mappers_[inner].get();
  const int mfb = static_cast<int>(m->GetMostFreqBin());
  if (mfb > 0) {
    const int nb = m->num_bin();
    data[2 * mfb] = sum_grad;
    data[2 * mfb + 1] = sum_hess;
    for (int i = 0; i < nb; ++i) {
      if (i != mfb) {
        data[2 * mfb] -= data[2 * i];
        data[2 * mfb + 1] -= data[2 * i + 1];
      }
    }
  }
}

void Dataset::DumpText(const std::string& path) const {
  std::ofstream f(path);
  f << "num_features: " << num_features_ << "\n";
  f << "num_total_features: " << num_total_features_ << "\n";
  f << "num_groups: " << groups_.size() << "\n";
  f << "num_data: " << num_data_ << "\n";
  f << "feature_names: " << common::Join(feature_names_, ", ") << "\n";
  for (data_size_t i = 0; i < num_data_; ++i) {
    for (int j = 0; j < num_features_; ++j) f << (j ? " " : "") << FeatureBin(j, i);
    f << "\n";
  }
}

void Dataset::AddFeaturesFrom(const Dataset& other) {
  if (other.num_data_ != num_data_) Log::Fatal("Cannot add features from other Dataset with a different number of rows");
  {
    std::lock_guard<std::mutex> lock(*row_major_mu_);
    row_stride_ = 0;  // the row-major copy follows the new groups
    row_major_.clear();
  }
  const int old_total = num_total_features_;
  const int old_inner = num_features_;
  const int old_groups = num_groups();
  for (int i = 0; i < other.num_total_features_; ++i) {
    used_feature_map_.push_back(other.used_feature_map_[i] < 0 ? -1 : other.used_feature_map_[i] + old_inner);
    feature_names_.push_back(i < static_cast<int>(other.feature_names_.size()) ? other.feature_names_[i]
                                                                             : "Column_" + std::to_string(old_total + i));
  }
  for (int j = 0; j < other.num_features_; ++j) {
    real_feature_idx_.push_back(other.real_feature_idx_[j] + old_total);
    feature2group_.push_back(other.feature2group_[j] + old_groups);
    feature2subfeature_.push_back(other.feature2subfeature_[j]);
    bin_mappers_.emplace_back(new BinMapper(*other.bin_mappers_[j]));
  }
  int mv_base = 0;
  for (int v : group_mv_) mv_base = std::max(mv_base, v + 1);
  group_mv_.resize(old_groups, -1);
  for (int g = 0; g < other.num_groups(); ++g) {
    const int v = g < static_cast<int>(other.group_mv_.size()) ? other.group_mv_[g] : -1;
    group_mv_.push_back(v < 0 ? -1 : v + mv_base);
  }
  if (!max_bin_by_feature_.empty() || !other.max_bin_by_feature_.empty()) {
    max_bin_by_feature_.resize(old_total, -1);
    for (int i = 0; i < other.num_total_features_; ++i) {
      max_bin_by_feature_.push_back(i < static_cast<int>(other.max_bin_by_feature_.size()) ? other.max_bin_by_feature_[i] : -1);
    }
  }
  if (!forced_bin_bounds_.empty() || !other.forced_bin_bounds_.empty()) {
    forced_bin_bounds_.resize(old_total);
    for (int i = 0; i < other.num_total_features_; ++i) {
      forced_bin_bounds_.push_back(i < static_cast<int>(other.forced_bin_bounds_.size()) ? other.forced_bin_bounds_[i]
                                                                                        : std::vector<double>());
    }
  }
  for (auto g : other.groups_) {
    for (auto& f : g.inner_features) f += old_inner;
    groups_.push_back(std::move(g));
  }
  for (int f : other.need_push_zeros_) need_push_zeros_.push_back(f + old_inner);
  num_total_features_ += other.num_total_features_;
  num_features_ += other.num_features_;
  group_bin_boundaries_.assign(1, 0);
  for (auto& g : groups_) group_bin_boundaries_.push_back(group_bin_boundaries_.back() + g.num_total_bin);
}

}  // namespace lgbm_amd
