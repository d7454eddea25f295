// Text/binary file loading and in-memory matrix ingestion.
// Reference: src/io/dataset_loader.cpp:19-1236 (file loading, sampling, row sharding for
// distributed training, label/weight/group/ignore/categorical column specs),
// src/io/parser.cpp:45-262 (CSV/TSV/LibSVM auto-detection).
#pragma once

#include <functional>
#include <memory>
#include <string>
#include <unordered_set>
#include <utility>
#include <vector>

#include "lgbm_amd/config.h"
#include "lgbm_amd/dataset.h"

namespace lgbm_amd {

class Parser {
 public:
  enum class Kind { CSV, TSV, LibSVM };
  Parser(Kind k, int label_idx, int total_cols) : kind_(k), label_idx_(label_idx), total_cols_(total_cols) {}
  // non-zero (or NaN) features with their column index (label removed) + label
  void ParseOneLine(const char* s, std::vector<std::pair<int, double>>* feats, double* label) const;
  int NumFeatures() const {
    return kind_ == Kind::LibSVM ? total_cols_ : total_cols_ - (label_idx_ >= 0 ? 1 : 0);
  }
  int label_idx() const { return label_idx_; }
  static std::unique_ptr<Parser> Create(const std::string& filename, bool header, int num_features, int label_idx);

 private:
  Kind kind_;
  int label_idx_;
  int total_cols_;
};

class DatasetLoader {
 public:
  DatasetLoader(const Config& cfg, int num_machines, int rank);
  // training data
  std::unique_ptr<Dataset> LoadFromFile(const std::string& filename);
  // validation data aligned with `train`
  std::unique_ptr<Dataset> LoadFromFileAlignWithOtherDataset(const std::string& filename, const Dataset& train);

  // resolve the label/weight/group/ignore/categorical specs given feature names (may be empty)
  void SetHeader(const std::vector<std::string>& names);
  const std::unordered_set<int>& categorical() const { return categorical_; }
  const std::unordered_set<int>& ignored() const { return ignored_; }
  static std::vector<std::vector<double>> GetForcedBins(const std::string& path, int num_total_features,
                                                        const std::unordered_set<int>& categorical);

 private:
  std::vector<std::string> ReadLines(const std::string& filename, bool keep_header_line);
  // parse `lines` (rows first_row, first_row + 1, ...) into the dataset and its metadata
  // (Metadata::Init before the first chunk, FinishQueryIds after the last)
  void ExtractFeatures(const std::vector<std::string>& lines, const Parser& parser, Dataset* ds,
                       data_size_t first_row = 0);
  // bin mappers from sampled lines, then the dataset of n rows
  std::unique_ptr<Dataset> ConstructFromSampleLines(const std::vector<std::string>& sample_lines, const Parser& parser,
                                                    data_size_t n);
  // two_round: pass 1 indexes the (local) lines, the sample is read by offset, pass 2 streams
  // the rows into the dataset -- the file is never held in memory
  std::unique_ptr<Dataset> LoadTwoRound(const std::string& filename, const Parser& parser, data_size_t* num_all);
  // side files (.weight / .query / .init) and the binary cache
  void FinishFromFile(const std::string& filename, data_size_t num_all, Dataset* ds);

  Config cfg_;
  int num_machines_;
  int rank_;
  int label_idx_ = 0;
  int weight_idx_ = -1;
  int group_idx_ = -1;
  std::unordered_set<int> ignored_;
  std::unordered_set<int> categorical_;
  std::vector<std::string> feature_names_;
  std::vector<data_size_t> used_rows_;  // row sharding (empty = all)
};

}  // namespace lgbm_amd
