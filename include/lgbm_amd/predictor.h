// Row-wise predictor shared by the C API and the CLI (reference
// src/application/predictor.hpp:30-260): normal / raw / leaf-index / SHAP outputs,
// margin-based early stopping for classification, sparse rows via hash maps for very
// wide models, and text-file prediction with header-name feature remapping.
#pragma once

#include <omp.h>

#include <cmath>
#include <fstream>
#include <functional>
#include <memory>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "lgbm_amd/boosting.h"
#include "lgbm_amd/common.h"
#include "lgbm_amd/dataset_loader.h"
#include "lgbm_amd/log.h"

namespace lgbm_amd {

class Predictor {
 public:
  using Row = std::vector<std::pair<int, double>>;

  // init_predict = false: the booster's prediction range is already this one (concurrent
  // predictors under a shared lock must not write it)
  Predictor(GBDT* boosting, int start_iteration, int num_iteration, bool is_raw_score, bool predict_leaf_index,
            bool predict_contrib, bool early_stop, int early_stop_freq, double early_stop_margin,
            bool init_predict = true)
      : boosting_(boosting) {
    early_stop_ = CreatePredictionEarlyStopInstance("none", PredictionEarlyStopConfig());
    if (early_stop && !boosting->NeedAccuratePrediction()) {
      PredictionEarlyStopConfig c;
      LGBM_CHECK_GT(early_stop_freq, 0);
      LGBM_CHECK_GE(early_stop_margin, 0);
      c.margin_threshold = early_stop_margin;
      c.round_period = early_stop_freq;
      early_stop_ = CreatePredictionEarlyStopInstance(boosting->NumberOfClasses() == 1 ? "binary" : "multiclass", c);
    }
    if (init_predict) boosting->InitPredict(start_iteration, num_iteration, predict_contrib);
    num_pred_one_row_ = boosting->NumPredictOneRow(start_iteration, num_iteration, predict_leaf_index, predict_contrib);
    num_feature_ = boosting->MaxFeatureIdx() + 1;
    buf_.assign(omp_get_max_threads(), std::vector<double>(num_feature_, 0.0));
    const int kWide = 100000;
    const size_t kSparse = static_cast<size_t>(0.01 * num_feature_);
    auto use_map = [=](const Row& r) { return num_feature_ > kWide && r.size() < kSparse; };
    if (predict_leaf_index) {
      fun_ = [=](const Row& r, double* out) {
        if (use_map(r)) {
          boosting_->PredictLeafIndexByMap(ToMap(r), out);
        } else {
          double* b = Fill(r);
          boosting_->PredictLeafIndex(b, out);
          Clear(r);
        }
      };
    } else if (predict_contrib) {
      fun_ = [=](const Row& r, double* out) {
        double* b = Fill(r);
        boosting_->PredictContrib(b, out);
        Clear(r);
      };
    } else if (is_raw_score) {
      fun_ = [=](const Row& r, double* out) {
        if (use_map(r)) {
          boosting_->PredictRawByMap(ToMap(r), out, &early_stop_);
        } else {
          double* b = Fill(r);
          boosting_->PredictRaw(b, out, &early_stop_);
          Clear(r);
        }
      };
    } else {
      fun_ = [=](const Row& r, double* out) {
        if (use_map(r)) {
          boosting_->PredictByMap(ToMap(r), out, &early_stop_);
        } else {
          double* b = Fill(r);
          boosting_->Predict(b, out, &early_stop_);
          Clear(r);
        }
      };
    }
  }

  int num_pred_one_row() const { return num_pred_one_row_; }
  void Predict(const Row& r, double* out) const { fun_(r, out); }

  void PredictFile(const std::string& data_filename, const std::string& result_filename, bool header,
                   bool disable_shape_check) const {
    std::ofstream out(result_filename);
    if (!out) Log::Fatal("Prediction results file %s cannot be found", result_filename.c_str());
    const int label_idx = header ? -1 : boosting_->LabelIdx();
    auto parser = Parser::Create(data_filename, header, num_feature_, label_idx);
    if (parser == nullptr) Log::Fatal("Could not recognize the data format of data file %s", data_filename.c_str());
    if (!header && !disable_shape_check && parser->NumFeatures() != num_feature_) {
      Log::Fatal("The number of features in data (%d) is not the same as it was in training data (%d).\n"
                 "You can set ``predict_disable_shape_check=true`` to discard this error, but please be aware what you are doing.",
                 parser->NumFeatures(), num_feature_);
    }
    std::ifstream in(data_filename);
    if (!in) Log::Fatal("Data file %s doesn't exist.", data_filename.c_str());
    std::string line;
    std::vector<int> remap;
    bool need_adjust = false;
    if (header) {
      std::getline(in, line);
      auto words = common::Split(common::Trim(line).c_str(), "\t,");
      std::unordered_map<std::string, int> pos;
      for (int i = 0; i < static_cast<int>(words.size()); ++i) {
        if (pos.count(words[i])) Log::Fatal("Feature (%s) appears more than one time.", words[i].c_str());
        pos[words[i]] = i;
      }
      remap.assign(std::max<int>(parser->NumFeatures(), static_cast<int>(words.size())), -1);
      const auto& names = boosting_->FeatureNames();
      for (int i = 0; i < static_cast<int>(names.size()); ++i) {
        auto it = pos.find(names[i]);
        if (it == pos.end()) {
          Log::Warning("Feature (%s) is missed in data file. If it is weight/query/group/ignore_column, you can ignore this warning.",
                       names[i].c_str());
        } else {
          remap[it->second] = i;
        }
      }
      for (int i = 0; i < static_cast<int>(remap.size()); ++i) {
        if (remap[i] >= 0 && remap[i] != i) need_adjust = true;
      }
    }
    const size_t kChunk = 1 << 16;
    std::vector<std::string> lines;
    lines.reserve(kChunk);
    auto flush = [&]() {
      std::vector<std::string> res(lines.size());
      common::OmpErrors errors;
#pragma omp parallel for schedule(static)
      for (int64_t i = 0; i < static_cast<int64_t>(lines.size()); ++i) {
        errors.Run([&] {
          Row feats;
          double label;
          parser->ParseOneLine(lines[i].c_str(), &feats, &label);
          if (need_adjust) {
            Row kept;
            for (auto& kv : feats) {
              if (kv.first < static_cast<int>(remap.size()) && remap[kv.first] >= 0) kept.emplace_back(remap[kv.first], kv.second);
            }
            feats.swap(kept);
          }
          std::vector<double> r(num_pred_one_row_);
          fun_(feats, r.data());
          res[i] = common::Join(r, "\t");
        });
      }
      errors.Check();
      for (auto& s : res) out << s << '\n';
      lines.clear();
    };
    while (std::getline(in, line)) {
      if (!line.empty() && line.back() == '\r') line.pop_back();
      if (line.empty()) continue;
      lines.push_back(line);
      if (lines.size() >= kChunk) flush();
    }
    flush();
  }

 private:
  double* Fill(const Row& r) const {
    double* b = const_cast<double*>(buf_[omp_get_thread_num()].data());
    for (auto& kv : r) {
      if (kv.first < num_feature_) b[kv.first] = kv.second;
    }
    return b;
  }
  void Clear(const Row& r) const {
    double* b = const_cast<double*>(buf_[omp_get_thread_num()].data());
    for (auto& kv : r) {
      if (kv.first < num_feature_) b[kv.first] = 0.0;
    }
  }
  static std::unordered_map<int, double> ToMap(const Row& r) {
    std::unordered_map<int, double> m;
    for (auto& kv : r) {
      if (std::fabs(kv.second) > kZeroThreshold || std::isnan(kv.second)) m[kv.first] = kv.second;
    }
    return m;
  }

  GBDT* boosting_;
  PredictionEarlyStopInstance early_stop_;
  int num_pred_one_row_ = 0;
  int num_feature_ = 0;
  std::vector<std::vector<double>> buf_;
  std::function<void(const Row&, double*)> fun_;
};

}  // namespace lgbm_amd
