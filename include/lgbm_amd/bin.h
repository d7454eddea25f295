// Per-feature value -> bin mapping, computed on the host from a row sample.
// Semantics (equal-frequency greedy binning with big-value isolation, zero as its own
// bin, NaN bin last, categorical "keep 99% mass" rule, trivial-feature filter,
// most-frequent-bin choice) follow reference src/io/bin.cpp:23-633 and
// include/LightGBM/bin.h:61-225,457-495 so that bin boundaries -- and therefore the
// model's thresholds and `feature_infos` -- are identical.
#pragma once

#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

#include "lgbm_amd/meta.h"

namespace lgbm_amd {

class BinMapper {
 public:
  BinMapper();

  void FindBin(double* values, int num_values, size_t total_sample_cnt, int max_bin, int min_data_in_bin,
               int min_split_data, bool pre_filter, BinType bin_type, bool use_missing, bool zero_as_missing,
               const std::vector<double>& forced_upper_bounds);

  uint32_t ValueToBin(double value) const;
  double BinToValue(uint32_t bin) const {
    return bin_type_ == BinType::Numerical ? bin_upper_bound_[bin] : static_cast<double>(bin_2_categorical_[bin]);
  }

  int num_bin() const { return num_bin_; }
  MissingType missing_type() const { return missing_type_; }
  bool is_trivial() const { return is_trivial_; }
  double sparse_rate() const { return sparse_rate_; }
  BinType bin_type() const { return bin_type_; }
  uint32_t GetDefaultBin() const { return default_bin_; }
  uint32_t GetMostFreqBin() const { return most_freq_bin_; }
  double min_val() const { return min_val_; }
  double max_val() const { return max_val_; }
  const std::vector<double>& upper_bounds() const { return bin_upper_bound_; }
  const std::vector<int>& bin_2_categorical() const { return bin_2_categorical_; }

  bool CheckAlign(const BinMapper& other) const;
  std::string bin_info_string() const;

  // fixed binary layout (used for distributed bin-mapper exchange and dataset binary files)
  size_t SizesInByte() const;
  void CopyTo(char* buffer) const;
  void CopyFrom(const char* buffer);

 private:
  int num_bin_;
  MissingType missing_type_;
  std::vector<double> bin_upper_bound_;
  bool is_trivial_;
  double sparse_rate_;
  BinType bin_type_;
  std::unordered_map<int, unsigned> categorical_2_bin_;
  std::vector<int> bin_2_categorical_;
  double min_val_;
  double max_val_;
  uint32_t default_bin_;
  uint32_t most_freq_bin_;
};

}  // namespace lgbm_amd
