// Text data loading: format auto-detection, column specs, bin-construction sampling,
// distributed row sharding and feature extraction.
// Reference behaviour: src/io/parser.cpp:45-262, src/io/parser.hpp:18-132,
// src/io/dataset_loader.cpp:19-225 (SetHeader, LoadFromFile), :713-790 (sharding:
// a line belongs to rank r when Random(data_random_seed).NextShort(0, num_machines) == r),
// :823-1003 (sampling + bin construction from text).
#include "lgbm_amd/dataset_loader.h"

#include <omp.h>

#include <cmath>
#include <fstream>
#include <sstream>

#include "lgbm_amd/common.h"
#include "lgbm_amd/log.h"
#include "lgbm_amd/random.h"
#include "text_reader.h"

namespace lgbm_amd {

namespace {

void CountSeparators(const std::string& s, int* comma, int* tab, int* colon) {
  *comma = *tab = *colon = 0;
  for (char c : s) {
    if (c == ',') ++*comma;
    else if (c == '\t') ++*tab;
    else if (c == ':') ++*colon;
  }
}

const char* SkipSpaceTab(const char* p) {
  while (*p == ' ' || *p == '\t') ++p;
  return p;
}

std::vector<std::string> FirstLines(const std::string& filename, bool header, int k) {
  std::ifstream f(filename);
  if (!f) Log::Fatal("Data file %s doesn't exist.", filename.c_str());
  std::vector<std::string> out;
  std::string line;
  if (header) std::getline(f, line);
  while (static_cast<int>(out.size()) < k && std::getline(f, line)) {
    line = common::Trim(line);
    if (!line.empty()) out.push_back(line);
  }
  if (out.empty()) Log::Fatal("Data file %s should have at least one line.", filename.c_str());
  return out;
}

int LibSVMNumCols(const std::string& filename, bool header) {
  std::ifstream f(filename);
  std::string line;
  if (header) std::getline(f, line);
  int max_idx = 0, max_line = 0;
  for (int i = 0; i < (1 << 13) && std::getline(f, line); ++i) {
    line = common::Trim(line);
    auto colon = line.find_last_of(':');
    auto space = line.find_last_of(" \f\t\v");
    if (colon == std::string::npos) continue;
    std::string sub = line.substr(space == std::string::npos ? 0 : space + 1);
    int idx = 0;
    common::Atoi(sub.c_str(), &idx);
    if (idx > max_idx) { max_idx = idx; max_line = i; }
    if (i - max_line >= (1 << 7)) break;
  }
  return max_idx;
}

}  // namespace

void Parser::ParseOneLine(const char* s, std::vector<std::pair<int, double>>* feats, double* label) const {
  double v = 0;
  if (kind_ == Kind::LibSVM) {
    if (label_idx_ == 0) {
      s = common::Atof(s, &v);
      *label = v;
      s = SkipSpaceTab(s);
    }
    while (*s != '\0') {
      int idx = 0;
      s = common::Atoi(s, &idx);
      s = SkipSpaceTab(s);
      if (*s != ':') Log::Fatal("Input format error when parsing as LibSVM");
      ++s;
      s = common::Atof(s, &v);
      feats->emplace_back(idx, v);
      s = SkipSpaceTab(s);
    }
    return;
  }
  const char sep = kind_ == Kind::CSV ? ',' : '\t';
  int idx = 0, offset = 0;
  while (*s != '\0') {
    s = common::Atof(s, &v);
    if (idx == label_idx_) {
      *label = v;
      offset = -1;
    } else if (std::fabs(v) > kZeroThreshold || std::isnan(v)) {
      feats->emplace_back(idx + offset, v);
    }
    ++idx;
    if (*s == sep) ++s;
    else if (*s != '\0') Log::Fatal("Input format error when parsing as %s", kind_ == Kind::CSV ? "CSV" : "TSV");
  }
}

std::unique_ptr<Parser> Parser::Create(const std::string& filename, bool header, int num_features, int label_idx) {
  auto lines = FirstLines(filename, header, 32);
  int c0, t0, k0;
  CountSeparators(lines[0], &c0, &t0, &k0);
  Kind kind;
  bool ok = false;
  if (lines.size() == 1) {
    if (k0 > 0) { kind = Kind::LibSVM; ok = true; }
    else if (t0 > 0) { kind = Kind::TSV; ok = true; }
    else if (c0 > 0) { kind = Kind::CSV; ok = true; }
  } else {
    int c1, t1, k1;
    CountSeparators(lines[1], &c1, &t1, &k1);
    if (k0 > 0 || k1 > 0) { kind = Kind::LibSVM; ok = true; }
    else if (t0 == t1 && t0 > 0) { kind = Kind::TSV; ok = true; }
    else if (c0 == c1 && c0 > 0) { kind = Kind::CSV; ok = true; }
    if (ok && kind != Kind::LibSVM) {
      for (size_t i = 2; i < lines.size(); ++i) {
        CountSeparators(lines[i], &c1, &t1, &k1);
        if ((kind == Kind::TSV && t1 != t0) || (kind == Kind::CSV && c1 != c0)) { ok = false; break; }
      }
    }
  }
  if (!ok) {
    // single-column files (label only) are CSV with one column
    if (lines.size() >= 1 && c0 == 0 && t0 == 0 && k0 == 0) {
      kind = Kind::CSV;
      ok = true;
    } else {
      Log::Fatal("Unknown format of training data.");
    }
  }
  int num_col = 0;
  int out_label = label_idx;
  if (kind == Kind::LibSVM) {
    num_col = LibSVMNumCols(filename, header) + 1;
    if (num_features > 0) {
      // prediction input without a label: first token contains ':'
      auto first = common::Split(lines[0].c_str(), " \t");
      if (!first.empty() && first[0].find(':') != std::string::npos) out_label = -1;
    }
    if (out_label > 0) Log::Fatal("Label should be the first column in a LibSVM file");
  } else {
    char sep = kind == Kind::CSV ? ',' : '\t';
    num_col = (kind == Kind::CSV ? c0 : t0) + 1;
    if (num_features > 0) {
      auto toks = common::SplitKeepEmpty(common::Trim(lines[0]), sep);
      if (static_cast<int>(toks.size()) == num_features) out_label = -1;
    }
  }
  const char* names[] = {"CSV", "TSV", "LibSVM"};
  if (out_label < 0) Log::Info("Data file %s doesn't contain a label column.", filename.c_str());
  Log::Debug("Parsing %s as %s", filename.c_str(), names[static_cast<int>(kind)]);
  return std::unique_ptr<Parser>(new Parser(kind, out_label, num_col));
}

DatasetLoader::DatasetLoader(const Config& cfg, int num_machines, int rank)
    : cfg_(cfg), num_machines_(num_machines), rank_(rank) {}

void DatasetLoader::SetHeader(const std::vector<std::string>& header_names) {
  const std::string prefix = "name:";
  std::vector<std::string> names = header_names;
  label_idx_ = 0;
  if (!cfg_.label_column.empty()) {
    if (common::StartsWith(cfg_.label_column, prefix)) {
      std::string n = cfg_.label_column.substr(prefix.size());
      label_idx_ = -1;
      for (int i = 0; i < static_cast<int>(names.size()); ++i) {
        if (names[i] == n) { label_idx_ = i; break; }
      }
      if (label_idx_ < 0) Log::Fatal("Could not find label column %s in data file \nor data file doesn't contain header", n.c_str());
      Log::Info("Using column %s as label", n.c_str());
    } else {
      if (!common::AtoiAndCheck(cfg_.label_column.c_str(), &label_idx_)) {
        Log::Fatal("label_column is not a number,\nif you want to use a column name,\nplease add the prefix \"name:\" to the column name");
      }
      Log::Info("Using column number %d as label", label_idx_);
    }
  }
  std::unordered_map<std::string, int> name2idx;
  if (!names.empty()) {
    if (label_idx_ >= 0 && label_idx_ < static_cast<int>(names.size())) names.erase(names.begin() + label_idx_);
    for (int i = 0; i < static_cast<int>(names.size()); ++i) name2idx[names[i]] = i;
    feature_names_ = names;
  }
  auto resolve_list = [&](const std::string& spec, const char* what, std::unordered_set<int>* out) {
    if (spec.empty()) return;
    if (common::StartsWith(spec, prefix)) {
      for (auto& n : common::Split(spec.substr(prefix.size()).c_str(), ',')) {
        if (!name2idx.count(n)) Log::Fatal("Could not find %s %s in data file", what, n.c_str());
        out->insert(name2idx[n]);
      }
    } else {
      for (auto& t : common::Split(spec.c_str(), ',')) {
        int v = 0;
        if (!common::AtoiAndCheck(common::Trim(t).c_str(), &v)) {
          Log::Fatal("%s is not a number,\nif you want to use a column name,\nplease add the prefix \"name:\" to the column name", what);
        }
        out->insert(v);
      }
    }
  };
  auto resolve_one = [&](const std::string& spec, const char* what) -> int {
    if (spec.empty()) return -1;
    int idx = -1;
    if (common::StartsWith(spec, prefix)) {
      std::string n = spec.substr(prefix.size());
      if (!name2idx.count(n)) Log::Fatal("Could not find %s column %s in data file", what, n.c_str());
      idx = name2idx[n];
    } else if (!common::AtoiAndCheck(spec.c_str(), &idx)) {
      Log::Fatal("%s_column is not a number,\nif you want to use a column name,\nplease add the prefix \"name:\" to the column name", what);
    }
    ignored_.insert(idx);
    return idx;
  };
  resolve_list(cfg_.ignore_column, "ignore_column", &ignored_);
  weight_idx_ = resolve_one(cfg_.weight_column, "weight");
  group_idx_ = resolve_one(cfg_.group_column, "group/query");
  resolve_list(cfg_.categorical_feature, "categorical_feature", &categorical_);
}

std::vector<std::vector<double>> DatasetLoader::GetForcedBins(const std::string& path, int num_total_features,
                                                              const std::unordered_set<int>& categorical) {
  std::vector<std::vector<double>> out(num_total_features);
  if (path.empty()) return out;
  std::ifstream f(path);
  if (!f) {
    Log::Warning("Forced bins file %s does not exist", path.c_str());
    return out;
  }
  std::stringstream ss;
  ss << f.rdbuf();
  std::string s = ss.str();
  // minimal JSON scan: [{"feature": i, "bin_upper_bound": [..]}, ...]
  size_t pos = 0;
  while ((pos = s.find("\"feature\"", pos)) != std::string::npos) {
    size_t colon = s.find(':', pos);
    int fidx = 0;
    common::Atoi(s.c_str() + colon + 1, &fidx);
    size_t ub = s.find("\"bin_upper_bound\"", pos);
    size_t lb = s.find('[', ub);
    size_t rb = s.find(']', lb);
    auto vals = common::StringToArray<double>(s.substr(lb + 1, rb - lb - 1), ',');
    if (fidx >= 0 && fidx < num_total_features) {
      if (categorical.count(fidx)) {
        Log::Warning("Feature %d is categorical. Will ignore forced bins for this feature.", fidx);
      } else {
        std::sort(vals.begin(), vals.end());
        vals.erase(std::unique(vals.begin(), vals.end()), vals.end());
        out[fidx] = vals;
      }
    }
    pos = rb;
  }
  return out;
}

std::vector<std::string> DatasetLoader::ReadLines(const std::string& filename, bool skip_header) {
  std::ifstream f(filename);
  if (!f) Log::Fatal("Data file %s doesn't exist.", filename.c_str());
  std::vector<std::string> lines;
  std::string line;
  if (skip_header) std::getline(f, line);
  while (std::getline(f, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (common::Trim(line).empty()) continue;
    lines.push_back(line);
  }
  return lines;
}

void DatasetLoader::ExtractFeatures(const std::vector<std::string>& lines, const Parser& parser, Dataset* ds,
                                    data_size_t first_row) {
  const data_size_t n = static_cast<data_size_t>(lines.size());
  Metadata& md = ds->metadata();
  common::OmpErrors errors;
#pragma omp parallel for schedule(static)
  for (data_size_t j = 0; j < n; ++j) {
    const data_size_t i = first_row + j;
    std::vector<std::pair<int, double>> feats;
    double label = 0;
    bool parsed = false;
    errors.Run([&] {
      parser.ParseOneLine(lines[j].c_str(), &feats, &label);
      parsed = true;
    });
    if (!parsed) continue;
    md.SetLabelAt(i, static_cast<label_t>(label));
    std::vector<std::pair<int, double>> kept;
    kept.reserve(feats.size());
    for (auto& kv : feats) {
      if (kv.first == weight_idx_) md.SetWeightAt(i, static_cast<label_t>(kv.second));
      else if (kv.first == group_idx_) md.SetQueryIdAt(i, static_cast<data_size_t>(kv.second));
      if (!ignored_.count(kv.first)) kept.push_back(kv);
    }
    errors.Run([&] { ds->PushSparseRow(i, kept); });
  }
  errors.Check();
}

std::unique_ptr<Dataset> DatasetLoader::ConstructFromSampleLines(const std::vector<std::string>& sample_lines,
                                                                 const Parser& parser, data_size_t n) {
  int num_col = parser.NumFeatures();
  std::vector<std::vector<double>> svals(num_col);
  std::vector<std::vector<int>> sidx(num_col);
  for (size_t i = 0; i < sample_lines.size(); ++i) {
    std::vector<std::pair<int, double>> feats;
    double label;
    parser.ParseOneLine(sample_lines[i].c_str(), &feats, &label);
    for (auto& kv : feats) {
      if (kv.first >= num_col) {
        num_col = kv.first + 1;
        svals.resize(num_col);
        sidx.resize(num_col);
      }
      if (std::fabs(kv.second) > kZeroThreshold || std::isnan(kv.second)) {
        svals[kv.first].push_back(kv.second);
        sidx[kv.first].push_back(static_cast<int>(i));
      }
    }
  }
  std::unique_ptr<Dataset> ds(new Dataset(n));
  if (feature_names_.size() == static_cast<size_t>(num_col)) ds->set_feature_names(feature_names_);
  auto forced = GetForcedBins(cfg_.forcedbins_filename, num_col, categorical_);
  ds->ConstructFromSample(&svals, &sidx, num_col, sample_lines.size(), n, cfg_, categorical_, ignored_, forced);
  if (feature_names_.size() == static_cast<size_t>(num_col)) ds->set_feature_names(feature_names_);
  ds->set_label_idx(label_idx_);
  ds->metadata().Init(n, weight_idx_ >= 0, group_idx_ >= 0);
  return ds;
}

std::unique_ptr<Dataset> DatasetLoader::LoadTwoRound(const std::string& filename, const Parser& parser,
                                                     data_size_t* num_all) {
  // pass 1: the local lines' offsets (row sharding draws exactly as the one-round path)
  Random rnd(cfg_.data_random_seed);
  const bool shard = num_machines_ > 1 && !cfg_.pre_partition;
  std::vector<int64_t> offsets;
  data_size_t total = 0;
  used_rows_.clear();
  TextReader::ForEachLine(filename, cfg_.header, [&](const char*, size_t, int64_t off) {
    if (!shard || rnd.NextShort(0, num_machines_) == rank_) {
      if (shard) used_rows_.push_back(total);
      offsets.push_back(off);
    }
    ++total;
  });
  *num_all = total;
  const data_size_t n = static_cast<data_size_t>(offsets.size());
  if (n == 0) Log::Fatal("Data file %s is empty", filename.c_str());
  const int sample_cnt = std::min<int>(n, cfg_.bin_construct_sample_cnt);
  auto sample_rows = rnd.Sample(n, sample_cnt);
  std::vector<int64_t> sample_off(sample_rows.size());
  for (size_t i = 0; i < sample_rows.size(); ++i) sample_off[i] = offsets[sample_rows[i]];
  auto ds = ConstructFromSampleLines(TextReader::ReadAt(filename, sample_off), parser, n);
  std::vector<int64_t>().swap(offsets);
  // pass 2: stream the local rows into the dataset in chunks
  const size_t kChunk = size_t(1) << 18;
  std::vector<std::string> chunk;
  chunk.reserve(kChunk);
  data_size_t line = 0, row = 0;
  size_t next_used = 0;
  auto flush = [&] {
    ExtractFeatures(chunk, parser, ds.get(), row);
    row += static_cast<data_size_t>(chunk.size());
    chunk.clear();
  };
  TextReader::ForEachLine(filename, cfg_.header, [&](const char* p, size_t len, int64_t) {
    const bool mine = !shard || (next_used < used_rows_.size() && used_rows_[next_used] == line);
    ++line;
    if (!mine) return;
    if (shard) ++next_used;
    chunk.emplace_back(p, len);
    if (chunk.size() >= kChunk) flush();
  });
  if (!chunk.empty()) flush();
  if (row != n) Log::Fatal("Data file %s changed while it was loaded", filename.c_str());
  return ds;
}

std::unique_ptr<Dataset> DatasetLoader::LoadFromFile(const std::string& filename) {
  // a dataset binary file -- <data>.bin first, then the file itself (reference
  // dataset_loader.cpp:1171-1195); under distributed training without pre_partition each rank
  // keeps its random share of the rows (:414-456)
  for (const std::string& bin_path : {filename + ".bin", filename}) {
    if (Dataset::IsBinaryFile(bin_path)) {
      Log::Info("Load from binary file %s", bin_path.c_str());
      const bool partition = num_machines_ > 1 && !cfg_.pre_partition;
      return Dataset::LoadBinaryFile(bin_path, rank_, num_machines_, partition, cfg_.data_random_seed);
    }
  }
  std::vector<std::string> header_names;
  if (cfg_.header) {
    std::ifstream f(filename);
    std::string first;
    std::getline(f, first);
    header_names = common::Split(common::Trim(first).c_str(), "\t,");
  }
  SetHeader(header_names);
  auto parser = Parser::Create(filename, cfg_.header, 0, label_idx_);
  if (cfg_.two_round) {
    data_size_t num_all = 0;
    auto ds = LoadTwoRound(filename, *parser, &num_all);
    ds->metadata().FinishQueryIds();
    FinishFromFile(filename, num_all, ds.get());
    return ds;
  }
  auto lines = ReadLines(filename, cfg_.header);
  Random rnd(cfg_.data_random_seed);
  const data_size_t num_all = static_cast<data_size_t>(lines.size());
  used_rows_.clear();
  if (num_machines_ > 1 && !cfg_.pre_partition) {
    std::vector<std::string> mine;
    for (data_size_t i = 0; i < num_all; ++i) {
      if (rnd.NextShort(0, num_machines_) == rank_) {
        used_rows_.push_back(i);
        mine.push_back(std::move(lines[i]));
      }
    }
    lines = std::move(mine);
  }
  const data_size_t n = static_cast<data_size_t>(lines.size());
  if (n == 0) Log::Fatal("Data file %s is empty", filename.c_str());
  // bin-construction sample
  int sample_cnt = std::min<int>(n, cfg_.bin_construct_sample_cnt);
  auto sample_rows = rnd.Sample(n, sample_cnt);
  std::vector<std::string> sample_lines(sample_rows.size());
  for (size_t i = 0; i < sample_rows.size(); ++i) sample_lines[i] = lines[sample_rows[i]];
  auto ds = ConstructFromSampleLines(sample_lines, *parser, n);
  ExtractFeatures(lines, *parser, ds.get());
  ds->metadata().FinishQueryIds();
  FinishFromFile(filename, num_all, ds.get());
  return ds;
}

void DatasetLoader::FinishFromFile(const std::string& filename, data_size_t num_all, Dataset* ds) {
  // side files override in-file weights/queries (reference metadata.cpp:23-60)
  Metadata side;
  side.InitFromFile(filename);
  Metadata& md = ds->metadata();
  if (side.weights()) {
    std::vector<label_t> w(side.weights(), side.weights() + (side.weights() ? ds->num_data() : 0));
    Metadata tmp = side;
    tmp.CheckOrPartition(num_all, used_rows_);
    md.SetWeights(tmp.weights(), tmp.num_data());
  }
  if (side.query_boundaries()) {
    if (!used_rows_.empty()) Log::Fatal("Query files are not supported with random row sharding; set pre_partition=true");
    std::vector<int32_t> counts;
    for (data_size_t q = 0; q < side.num_queries(); ++q) {
      counts.push_back(side.query_boundaries()[q + 1] - side.query_boundaries()[q]);
    }
    md.SetQuery(counts.data(), static_cast<data_size_t>(counts.size()));
  }
  if (side.init_score()) {
    Metadata tmp = side;
    std::vector<label_t> dummy(num_all, 0.0f);
    tmp.SetLabel(dummy.data(), num_all);
    tmp.CheckOrPartition(num_all, used_rows_);
    md.SetInitScore(tmp.init_score(), tmp.num_init_score());
  }
  ds->FinishLoad();
  if (cfg_.save_binary) ds->SaveBinaryFile(filename + ".bin");
}

std::unique_ptr<Dataset> DatasetLoader::LoadFromFileAlignWithOtherDataset(const std::string& filename,
                                                                         const Dataset& train) {
  if (Dataset::IsBinaryFile(filename)) return Dataset::LoadBinaryFile(filename);
  std::vector<std::string> header_names;
  if (cfg_.header) {
    std::ifstream f(filename);
    std::string first;
    std::getline(f, first);
    header_names = common::Split(common::Trim(first).c_str(), "\t,");
  }
  SetHeader(header_names);
  auto parser = Parser::Create(filename, cfg_.header, 0, label_idx_);
  auto lines = ReadLines(filename, cfg_.header);
  const data_size_t n = static_cast<data_size_t>(lines.size());
  std::unique_ptr<Dataset> ds(new Dataset(n));
  ds->CreateValid(train, n);
  ds->metadata().Init(n, weight_idx_ >= 0, group_idx_ >= 0);
  ExtractFeatures(lines, *parser, ds.get());
  ds->metadata().FinishQueryIds();
  Metadata side;
  side.InitFromFile(filename);
  if (side.weights()) ds->metadata().SetWeights(side.weights(), n);
  if (side.query_boundaries()) {
    std::vector<int32_t> counts;
    for (data_size_t q = 0; q < side.num_queries(); ++q) {
      counts.push_back(side.query_boundaries()[q + 1] - side.query_boundaries()[q]);
    }
    ds->metadata().SetQuery(counts.data(), static_cast<data_size_t>(counts.size()));
  }
  if (side.init_score()) ds->metadata().SetInitScore(side.init_score(), side.num_init_score());
  ds->FinishLoad();
  return ds;
}

}  // namespace lgbm_amd
