// C API implementation (reference src/c_api.cpp:40-2100 for the semantics of every entry
// point: dataset construction by row sampling + FindBin + parallel push, booster
// lifecycle, prediction for dense/CSR/CSC/file inputs, model IO, network setup).
// Errors are reported as return code -1 with the message in LGBM_GetLastError().
#include "lgbm_amd/c_api.h"

#include <hip/hip_runtime_api.h>
#include <omp.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "lgbm_amd/boosting.h"
#include "lgbm_amd/common.h"
#include "lgbm_amd/device_binning.h"
#include "lgbm_amd/config.h"
#include "lgbm_amd/dataset.h"
#include "lgbm_amd/dataset_loader.h"
#include "lgbm_amd/log.h"
#include "lgbm_amd/metric.h"
#include "lgbm_amd/network.h"
#include "lgbm_amd/objective.h"
#include "lgbm_amd/predictor.h"
#include "lgbm_amd/random.h"
#include "lgbm_amd/tuning.h"

using namespace lgbm_amd;

namespace {

thread_local std::string g_last_error = "Everything is fine";

inline int ApiError(const char* msg) {
  g_last_error = msg;
  return -1;
}

#define API_BEGIN() try {
#define API_END()                           \
  }                                         \
  catch (std::exception & ex) {             \
    return ApiError(ex.what());             \
  }                                         \
  catch (std::string & ex) {                \
    return ApiError(ex.c_str());            \
  }                                         \
  catch (...) {                             \
    return ApiError("unknown exception");   \
  }                                         \
  return 0;

using Row = std::vector<std::pair<int, double>>;

// ------------------------------------------------------------------ row accessors
std::function<std::vector<double>(int)> DenseRowFun(const void* data, int dtype, int nrow, int ncol, int row_major) {
  if (dtype == C_API_DTYPE_FLOAT32) {
    const float* p = static_cast<const float*>(data);
    if (row_major) {
      return [=](int r) {
        std::vector<double> v(ncol);
        const float* q = p + static_cast<int64_t>(ncol) * r;
        for (int j = 0; j < ncol; ++j) v[j] = static_cast<double>(q[j]);
        return v;
      };
    }
    return [=](int r) {
      std::vector<double> v(ncol);
      for (int j = 0; j < ncol; ++j) v[j] = static_cast<double>(p[static_cast<int64_t>(nrow) * j + r]);
      return v;
    };
  } else if (dtype == C_API_DTYPE_FLOAT64) {
    const double* p = static_cast<const double*>(data);
    if (row_major) {
      return [=](int r) {
        const double* q = p + static_cast<int64_t>(ncol) * r;
        return std::vector<double>(q, q + ncol);
      };
    }
    return [=](int r) {
      std::vector<double> v(ncol);
      for (int j = 0; j < ncol; ++j) v[j] = p[static_cast<int64_t>(nrow) * j + r];
      return v;
    };
  }
  Log::Fatal("Unknown data type in RowFunctionFromDenseMatric");
  return nullptr;
}

std::function<Row(int)> DenseRowPairFun(const void* data, int dtype, int nrow, int ncol, int row_major) {
  auto inner = DenseRowFun(data, dtype, nrow, ncol, row_major);
  return [inner](int r) {
    auto v = inner(r);
    Row out;
    for (int j = 0; j < static_cast<int>(v.size()); ++j) {
      if (std::fabs(v[j]) > kZeroThreshold || std::isnan(v[j])) out.emplace_back(j, v[j]);
    }
    return out;
  };
}

// row-major matrices given as an array of row pointers
std::function<Row(int)> MatsRowPairFun(const void** data, int dtype, int nrow, int ncol) {
  (void)nrow;
  return [=](int r) {
    Row out;
    if (dtype == C_API_DTYPE_FLOAT32) {
      const float* p = static_cast<const float*>(data[r]);
      for (int j = 0; j < ncol; ++j) {
        const double v = p[j];
        if (std::fabs(v) > kZeroThreshold || std::isnan(v)) out.emplace_back(j, v);
      }
    } else {
      const double* p = static_cast<const double*>(data[r]);
      for (int j = 0; j < ncol; ++j) {
        const double v = p[j];
        if (std::fabs(v) > kZeroThreshold || std::isnan(v)) out.emplace_back(j, v);
      }
    }
    return out;
  };
}

template <typename T>
inline double ValAt(const void* data, int64_t i) {
  return static_cast<double>(static_cast<const T*>(data)[i]);
}

std::function<Row(int64_t)> CSRRowFun(const void* indptr, int indptr_type, const int32_t* indices, const void* data,
                                      int dtype, int64_t nindptr, int64_t nelem) {
  (void)nindptr;
  (void)nelem;
  auto ptr_at = [=](int64_t i) -> int64_t {
    return indptr_type == C_API_DTYPE_INT32 ? static_cast<const int32_t*>(indptr)[i]
                                            : static_cast<const int64_t*>(indptr)[i];
  };
  if (indptr_type != C_API_DTYPE_INT32 && indptr_type != C_API_DTYPE_INT64) Log::Fatal("Unknown indptr type");
  if (dtype != C_API_DTYPE_FLOAT32 && dtype != C_API_DTYPE_FLOAT64) Log::Fatal("Unknown data type in CSR");
  return [=](int64_t r) {
    Row out;
    const int64_t s = ptr_at(r), e = ptr_at(r + 1);
    out.reserve(e - s);
    for (int64_t i = s; i < e; ++i) {
      out.emplace_back(indices[i], dtype == C_API_DTYPE_FLOAT32 ? ValAt<float>(data, i) : ValAt<double>(data, i));
    }
    return out;
  };
}

// column-major sparse input converted to rows (one pass, O(nnz))
std::vector<Row> CSCToRows(const void* col_ptr, int col_ptr_type, const int32_t* indices, const void* data,
                           int dtype, int64_t ncol_ptr, int64_t num_row) {
  std::vector<Row> rows(num_row);
  auto ptr_at = [=](int64_t i) -> int64_t {
    return col_ptr_type == C_API_DTYPE_INT32 ? static_cast<const int32_t*>(col_ptr)[i]
                                             : static_cast<const int64_t*>(col_ptr)[i];
  };
  for (int64_t c = 0; c + 1 < ncol_ptr; ++c) {
    for (int64_t i = ptr_at(c); i < ptr_at(c + 1); ++i) {
      const double v = dtype == C_API_DTYPE_FLOAT32 ? ValAt<float>(data, i) : ValAt<double>(data, i);
      rows[indices[i]].emplace_back(static_cast<int>(c), v);
    }
  }
  return rows;
}

std::vector<int> SampleRows(const Config& cfg, data_size_t nrow) {
  Random rnd(cfg.data_random_seed);
  const int cnt = static_cast<int>(std::min<int64_t>(nrow, cfg.bin_construct_sample_cnt));
  return rnd.Sample(nrow, cnt);
}

Dataset* ConstructFromSamples(std::vector<std::vector<double>>* sv, std::vector<std::vector<int>>* si, int ncol,
                              size_t sample_cnt, data_size_t nrow, const Config& cfg) {
  DatasetLoader loader(cfg, 1, 0);
  loader.SetHeader({});
  auto forced = DatasetLoader::GetForcedBins(cfg.forcedbins_filename, ncol, loader.categorical());
  std::unique_ptr<Dataset> ds(new Dataset(nrow));
  ds->ConstructFromSample(sv, si, ncol, sample_cnt, nrow, cfg, loader.categorical(), loader.ignored(), forced);
  std::vector<std::string> names;
  for (int i = 0; i < ncol; ++i) names.push_back("Column_" + std::to_string(i));
  ds->set_feature_names(names);
  ds->metadata().Init(nrow, false, false);
  return ds.release();
}

// build a dataset from a row accessor: sample -> bins -> parallel push
Dataset* DatasetFromRows(const std::function<Row(int64_t)>& get_row, data_size_t nrow, int ncol, const Config& cfg,
                         const Dataset* reference) {
  std::unique_ptr<Dataset> ds;
  if (reference == nullptr) {
    auto idx = SampleRows(cfg, nrow);
    std::vector<std::vector<double>> sv(ncol);
    std::vector<std::vector<int>> si(ncol);
    for (size_t i = 0; i < idx.size(); ++i) {
      for (auto& kv : get_row(idx[i])) {
        if (kv.first >= ncol) {
          ncol = kv.first + 1;
          sv.resize(ncol);
          si.resize(ncol);
        }
        if (std::fabs(kv.second) > kZeroThreshold || std::isnan(kv.second)) {
          sv[kv.first].push_back(kv.second);
          si[kv.first].push_back(static_cast<int>(i));
        }
      }
    }
    ds.reset(ConstructFromSamples(&sv, &si, ncol, idx.size(), nrow, cfg));
  } else {
    ds.reset(new Dataset(nrow));
    ds->CreateValid(*reference, nrow);
    ds->metadata().Init(nrow, false, false);
  }
  common::OmpErrors errors;
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < nrow; ++r) {
    errors.Run([&] { ds->PushSparseRow(static_cast<data_size_t>(r), get_row(r)); });
  }
  errors.Check();
  ds->FinishLoad();
  return ds.release();
}

Config ParamsToConfig(const char* parameters) {
  auto p = Config::Str2Map(parameters);
  Config cfg;
  cfg.Set(p);
  if (cfg.num_threads > 0) omp_set_num_threads(cfg.num_threads);
  return cfg;
}

// ------------------------------------------------------------------ booster
class Booster {
 public:
  explicit Booster(const char* filename) {
    boosting_.reset(GBDT::CreateBoosting("gbdt", filename));
  }

  Booster(const Dataset* train, const char* parameters) {
    auto param = Config::Str2Map(parameters);
    config_.Set(param);
    if (config_.num_threads > 0) omp_set_num_threads(config_.num_threads);
    if (!config_.input_model.empty()) {
      Log::Warning("Continued train from model is not supported for c_api,\nplease use continued train with input score");
    }
    boosting_.reset(GBDT::CreateBoosting(config_.boosting, nullptr));
    train_data_ = train;
    CreateObjectiveAndMetrics();
    // feature-parallel needs the same full dataset on every rank (the reference refuses it in
    // the C API, c_api.cpp:133; here the caller is trusted to pass identical data)
    if (config_.tree_learner == "feature" && Network::num_machines() > 1) {
      Log::Info("feature-parallel training: every rank must hold the same rows");
    }
    if (Network::num_machines() == 1 && config_.tree_learner != "serial") {
      Log::Warning("Only find one worker, will switch to serial tree learner");
      config_.tree_learner = "serial";
    }
    boosting_->Init(&config_, train_data_, objective_.get(), Ptrs(train_metric_));
  }

  Booster() { boosting_.reset(GBDT::CreateBoosting("gbdt", nullptr)); }

  void LoadModelFromString(const char* s) {
    boosting_->LoadModelFromString(s, std::strlen(s));
  }

  void MergeFrom(const Booster* other) {
    std::unique_lock<std::shared_mutex> l(mu_);
    boosting_->MergeFrom(other->boosting_.get());
  }

  void ResetTrainingData(const Dataset* train) {
    if (train != train_data_) {
      std::unique_lock<std::shared_mutex> l(mu_);
      train_data_ = train;
      CreateObjectiveAndMetrics();
      boosting_->ResetTrainingData(train_data_, objective_.get(), Ptrs(train_metric_));
    }
  }

  static void CheckDatasetResetConfig(const Config& old_cfg, const std::unordered_map<std::string, std::string>& p) {
    Config nc = old_cfg;
    nc.Set(p);
    auto fail = [](const char* n) { Log::Fatal("Cannot change %s after constructed Dataset handle.", n); };
    if (nc.max_bin != old_cfg.max_bin) fail("max_bin");
    if (nc.max_bin_by_feature != old_cfg.max_bin_by_feature) fail("max_bin_by_feature");
    if (nc.bin_construct_sample_cnt != old_cfg.bin_construct_sample_cnt) fail("bin_construct_sample_cnt");
    if (nc.min_data_in_bin != old_cfg.min_data_in_bin) fail("min_data_in_bin");
    if (nc.use_missing != old_cfg.use_missing) fail("use_missing");
    if (nc.zero_as_missing != old_cfg.zero_as_missing) fail("zero_as_missing");
    if (nc.categorical_feature != old_cfg.categorical_feature) fail("categorical_feature");
    if (nc.feature_pre_filter != old_cfg.feature_pre_filter) fail("feature_pre_filter");
    if (nc.is_enable_sparse != old_cfg.is_enable_sparse) fail("is_enable_sparse");
    if (nc.pre_partition != old_cfg.pre_partition) fail("pre_partition");
    if (nc.enable_bundle != old_cfg.enable_bundle) fail("enable_bundle");
    if (nc.header != old_cfg.header) fail("header");
    if (nc.two_round != old_cfg.two_round) fail("two_round");
    if (nc.label_column != old_cfg.label_column) fail("label_column");
    if (nc.weight_column != old_cfg.weight_column) fail("weight_column");
    if (nc.group_column != old_cfg.group_column) fail("group_column");
    if (nc.ignore_column != old_cfg.ignore_column) fail("ignore_column");
    if (nc.forcedbins_filename != old_cfg.forcedbins_filename) fail("forcedbins_filename");
    if (nc.min_data_in_leaf != old_cfg.min_data_in_leaf && old_cfg.feature_pre_filter) {
      Log::Fatal("Reducing `min_data_in_leaf` with `feature_pre_filter=true` may cause unexpected behaviour "
                 "for features that were pre-filtered by the larger `min_data_in_leaf`.\n"
                 "You need to set `feature_pre_filter=false` to dynamically change the `min_data_in_leaf`.");
    }
  }

  void ResetConfig(const char* parameters) {
    std::unique_lock<std::shared_mutex> l(mu_);
    auto param = Config::Str2Map(parameters);
    if (param.count("num_class")) Log::Fatal("Cannot change num_class during training");
    if (param.count("boosting")) Log::Fatal("Cannot change boosting during training");
    if (param.count("metric")) Log::Fatal("Cannot change metric during training");
    CheckDatasetResetConfig(config_, param);
    config_.Set(param);
    if (config_.num_threads > 0) omp_set_num_threads(config_.num_threads);
    if (param.count("objective")) {
      objective_.reset(ObjectiveFunction::CreateObjectiveFunction(config_.objective, config_));
      if (objective_ == nullptr) Log::Info("Using self-defined objective function");
      if (objective_ != nullptr) objective_->Init(train_data_->metadata(), train_data_->num_data());
      boosting_->ResetTrainingData(train_data_, objective_.get(), Ptrs(train_metric_));
    }
    boosting_->ResetConfig(&config_);
  }

  void AddValidData(const Dataset* valid) {
    std::unique_lock<std::shared_mutex> l(mu_);
    valid_metrics_.emplace_back();
    for (auto& t : config_.metric) {
      std::unique_ptr<Metric> m(Metric::CreateMetric(t, config_));
      if (m == nullptr) continue;
      m->Init(valid->metadata(), valid->num_data());
      valid_metrics_.back().push_back(std::move(m));
    }
    valid_metrics_.back().shrink_to_fit();
    boosting_->AddValidDataset(valid, Ptrs(valid_metrics_.back()));
  }

  bool TrainOneIter() {
    std::unique_lock<std::shared_mutex> l(mu_);
    return boosting_->TrainOneIter(nullptr, nullptr);
  }

  void Refit(const int32_t* leaf_preds, int32_t nrow, int32_t ncol) {
    std::unique_lock<std::shared_mutex> l(mu_);
    std::vector<std::vector<int32_t>> v(nrow, std::vector<int32_t>(ncol));
    for (int32_t i = 0; i < nrow; ++i) {
      for (int32_t j = 0; j < ncol; ++j) v[i][j] = leaf_preds[static_cast<size_t>(i) * ncol + j];
    }
    boosting_->RefitTree(v);
  }

  bool TrainOneIter(const score_t* g, const score_t* h) {
    std::unique_lock<std::shared_mutex> l(mu_);
    return boosting_->TrainOneIter(g, h);
  }

  void RollbackOneIter() {
    std::unique_lock<std::shared_mutex> l(mu_);
    boosting_->RollbackOneIter();
  }

  // the lock a host prediction holds while it runs: shared when the booster's prediction range
  // already is this one (and no SHAP, whose setup rewrites the trees' depths), else exclusive
  // after setting it
  struct PredictLock {
    std::shared_lock<std::shared_mutex> shared;
    std::unique_lock<std::shared_mutex> unique;
    bool init = false;  // the predictor must run InitPredict (exclusive lock held)
  };
  void LockForPredict(int predict_type, int start_iteration, int num_iteration, PredictLock* pl) {
    if (predict_type != C_API_PREDICT_CONTRIB) {
      pl->shared = std::shared_lock<std::shared_mutex>(mu_);
      if (boosting_->PredictRangeIs(start_iteration, num_iteration)) return;
      pl->shared.unlock();
    }
    pl->unique = std::unique_lock<std::shared_mutex>(mu_);
    pl->init = true;
  }

  std::unique_ptr<Predictor> MakePredictor(int predict_type, int start_iteration, int num_iteration,
                                           const Config& cfg, bool init_predict = true) {
    bool raw = false, leaf = false, contrib = false;
    if (predict_type == C_API_PREDICT_LEAF_INDEX) leaf = true;
    else if (predict_type == C_API_PREDICT_RAW_SCORE) raw = true;
    else if (predict_type == C_API_PREDICT_CONTRIB) contrib = true;
    return std::unique_ptr<Predictor>(new Predictor(boosting_.get(), start_iteration, num_iteration, raw, leaf,
                                                    contrib, cfg.pred_early_stop, cfg.pred_early_stop_freq,
                                                    cfg.pred_early_stop_margin, init_predict));
  }

  void PredictRows(const std::function<Row(int64_t)>& get_row, int64_t nrow, int64_t ncol, int predict_type,
                   int start_iteration, int num_iteration, const Config& cfg, double* out, int64_t* out_len) {
    if (!cfg.predict_disable_shape_check && ncol != boosting_->MaxFeatureIdx() + 1) {
      Log::Fatal("The number of features in data (%d) is not the same as it was in training data (%d).\n"
                 "You can set ``predict_disable_shape_check=true`` to discard this error, but please be aware what you are doing.",
                 static_cast<int>(ncol), boosting_->MaxFeatureIdx() + 1);
    }
    PredictLock pl;
    LockForPredict(predict_type, start_iteration, num_iteration, &pl);
    auto pred = MakePredictor(predict_type, start_iteration, num_iteration, cfg, pl.init);
    const int k = pred->num_pred_one_row();
    common::OmpErrors errors;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < nrow; ++i) {
      errors.Run([&] { pred->Predict(get_row(i), out + k * i); });
    }
    errors.Check();
    *out_len = k * nrow;
  }

  // dense matrices from a booster trained (or predicted) with device_type=gpu go to the
  // device forest kernel; single rows, leaf / contrib predictions and early stopping stay on
  // the host
  bool PredictDenseOnDevice(const void* data, int data_type, int32_t nrow, int32_t ncol, int is_row_major,
                            int predict_type, int start_iteration, int num_iteration, const Config& cfg, double* out,
                            int64_t* out_len) {
    if (predict_type != C_API_PREDICT_NORMAL && predict_type != C_API_PREDICT_RAW_SCORE) return false;
    if (cfg.pred_early_stop || nrow < 1024) return false;
    if (data_type != C_API_DTYPE_FLOAT32 && data_type != C_API_DTYPE_FLOAT64) return false;
    if (cfg.device_type != "gpu" && config_.device_type != "gpu") return false;
    const char* e = tuning::Get(tuning::Knob::HostPredict);
    if (e != nullptr && e[0] == '1') return false;
    if (!cfg.predict_disable_shape_check && ncol != boosting_->MaxFeatureIdx() + 1) return false;  // host path reports it
    std::unique_lock<std::shared_mutex> l(mu_);
    const bool raw = predict_type == C_API_PREDICT_RAW_SCORE;
    if (!boosting_->PredictDenseOnDevice(data, data_type == C_API_DTYPE_FLOAT64, nrow, ncol, is_row_major != 0,
                                         start_iteration, num_iteration, raw, out)) {
      return false;
    }
    *out_len = static_cast<int64_t>(nrow) * boosting_->NumPredictOneRow(start_iteration, num_iteration, false, false);
    return true;
  }

  void PredictFile(const char* data, int header, int predict_type, int start_iteration, int num_iteration,
                   const Config& cfg, const char* result) {
    PredictLock pl;
    LockForPredict(predict_type, start_iteration, num_iteration, &pl);
    auto pred = MakePredictor(predict_type, start_iteration, num_iteration, cfg, pl.init);
    pred->PredictFile(data, result, header != 0, cfg.predict_disable_shape_check);
  }

  std::vector<double> GetEval(int idx) { return boosting_->GetEvalAt(idx); }
  GBDT* boosting() { return boosting_.get(); }
  const Config& config() const { return config_; }
  std::shared_mutex& mutex() { return mu_; }

 private:
  template <typename T>
  static std::vector<const T*> Ptrs(const std::vector<std::unique_ptr<T>>& v) {
    std::vector<const T*> out;
    for (auto& p : v) out.push_back(p.get());
    return out;
  }

  void CreateObjectiveAndMetrics() {
    objective_.reset(ObjectiveFunction::CreateObjectiveFunction(config_.objective, config_));
    if (objective_ == nullptr) Log::Info("Using self-defined objective function");
    if (objective_ != nullptr) objective_->Init(train_data_->metadata(), train_data_->num_data());
    train_metric_.clear();
    for (auto& t : config_.metric) {
      std::unique_ptr<Metric> m(Metric::CreateMetric(t, config_));
      if (m == nullptr) continue;
      m->Init(train_data_->metadata(), train_data_->num_data());
      train_metric_.push_back(std::move(m));
    }
  }

  const Dataset* train_data_ = nullptr;
  std::unique_ptr<GBDT> boosting_;
  Config config_;
  std::unique_ptr<ObjectiveFunction> objective_;
  std::vector<std::unique_ptr<Metric>> train_metric_;
  std::vector<std::vector<std::unique_ptr<Metric>>> valid_metrics_;
  // exclusive: training, model changes, device prediction; shared: host predictions of the
  // current prediction range (reference c_api.cpp SHARED_LOCK / UNIQUE_LOCK)
  std::shared_mutex mu_;
};

struct FastConfig {
  Booster* booster;
  Config config;
  int predict_type, start_iteration, num_iteration, data_type;
  int64_t ncol;
  std::unique_ptr<Predictor> predictor;
};

int CopyStrings(const std::vector<std::string>& v, int len, int* out_len, size_t buffer_len, size_t* out_buffer_len,
                char** out) {
  *out_len = static_cast<int>(v.size());
  *out_buffer_len = 0;
  for (size_t i = 0; i < v.size(); ++i) {
    const size_t need = v[i].size() + 1;
    *out_buffer_len = std::max(*out_buffer_len, need);
    if (static_cast<int>(i) < len && out != nullptr && out[i] != nullptr) {
      std::memcpy(out[i], v[i].c_str(), std::min(need, buffer_len));
      if (need > buffer_len && buffer_len > 0) out[i][buffer_len - 1] = '\0';
    }
  }
  return 0;
}

}  // namespace

// ====================================================================== exports
const char* LGBM_GetLastError() { return g_last_error.c_str(); }

int LGBM_RegisterLogCallback(void (*callback)(const char*)) {
  API_BEGIN();
  Log::ResetCallback(callback);
  API_END();
}

int LGBM_DatasetCreateFromFile(const char* filename, const char* parameters, const DatasetHandle reference,
                               DatasetHandle* out) {
  API_BEGIN();
  Config cfg = ParamsToConfig(parameters);
  DatasetLoader loader(cfg, Network::num_machines(), Network::rank());
  if (reference == nullptr) {
    *out = loader.LoadFromFile(filename).release();
  } else {
    *out = loader.LoadFromFileAlignWithOtherDataset(filename, *static_cast<const Dataset*>(reference)).release();
  }
  API_END();
}

int LGBM_DatasetCreateFromSampledColumn(double** sample_data, int** sample_indices, int32_t ncol,
                                        const int* num_per_col, int32_t num_sample_row, int32_t num_total_row,
                                        const char* parameters, DatasetHandle* out) {
  API_BEGIN();
  Config cfg = ParamsToConfig(parameters);
  std::vector<std::vector<double>> sv(ncol);
  std::vector<std::vector<int>> si(ncol);
  for (int i = 0; i < ncol; ++i) {
    sv[i].assign(sample_data[i], sample_data[i] + num_per_col[i]);
    si[i].assign(sample_indices[i], sample_indices[i] + num_per_col[i]);
  }
  *out = ConstructFromSamples(&sv, &si, ncol, num_sample_row, num_total_row, cfg);
  API_END();
}

int LGBM_DatasetCreateByReference(const DatasetHandle reference, int64_t num_total_row, DatasetHandle* out) {
  API_BEGIN();
  std::unique_ptr<Dataset> ds(new Dataset(static_cast<data_size_t>(num_total_row)));
  ds->CreateValid(*static_cast<const Dataset*>(reference), static_cast<data_size_t>(num_total_row));
  ds->metadata().Init(static_cast<data_size_t>(num_total_row), false, false);
  *out = ds.release();
  API_END();
}

int LGBM_DatasetPushRows(DatasetHandle dataset, const void* data, int data_type, int32_t nrow, int32_t ncol,
                         int32_t start_row) {
  API_BEGIN();
  auto* ds = static_cast<Dataset*>(dataset);
  auto get = DenseRowPairFun(data, data_type, nrow, ncol, 1);
  common::OmpErrors errors;
#pragma omp parallel for schedule(static)
  for (int i = 0; i < nrow; ++i) {
    errors.Run([&] { ds->PushSparseRow(start_row + i, get(i)); });
  }
  errors.Check();
  if (start_row + nrow == ds->num_data()) ds->FinishLoad();
  API_END();
}

int LGBM_DatasetPushRowsByCSR(DatasetHandle dataset, const void* indptr, int indptr_type, const int32_t* indices,
                              const void* data, int data_type, int64_t nindptr, int64_t nelem, int64_t,
                              int64_t start_row) {
  API_BEGIN();
  auto* ds = static_cast<Dataset*>(dataset);
  auto get = CSRRowFun(indptr, indptr_type, indices, data, data_type, nindptr, nelem);
  const int64_t nrow = nindptr - 1;
  common::OmpErrors errors;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < nrow; ++i) {
    errors.Run([&] { ds->PushSparseRow(static_cast<data_size_t>(start_row + i), get(i)); });
  }
  errors.Check();
  if (start_row + nrow == ds->num_data()) ds->FinishLoad();
  API_END();
}

int LGBM_DatasetCreateFromCSR(const void* indptr, int indptr_type, const int32_t* indices, const void* data,
                              int data_type, int64_t nindptr, int64_t nelem, int64_t num_col, const char* parameters,
                              const DatasetHandle reference, DatasetHandle* out) {
  API_BEGIN();
  if (num_col <= 0) Log::Fatal("The number of columns should be greater than zero.");
  if (num_col >= INT32_MAX) Log::Fatal("The number of columns should be smaller than INT32_MAX.");
  Config cfg = ParamsToConfig(parameters);
  auto get = CSRRowFun(indptr, indptr_type, indices, data, data_type, nindptr, nelem);
  *out = DatasetFromRows(get, static_cast<data_size_t>(nindptr - 1), static_cast<int>(num_col), cfg,
                         static_cast<const Dataset*>(reference));
  API_END();
}

int LGBM_DatasetCreateFromCSRFunc(void* get_row_funptr, int num_rows, int64_t num_col, const char* parameters,
                                  const DatasetHandle reference, DatasetHandle* out) {
  API_BEGIN();
  if (num_col <= 0) Log::Fatal("The number of columns should be greater than zero.");
  Config cfg = ParamsToConfig(parameters);
  auto& fn = *static_cast<std::function<void(int, Row&)>*>(get_row_funptr);
  auto get = [&fn](int64_t r) {
    Row row;
    fn(static_cast<int>(r), row);
    return row;
  };
  // the callback is not required to be thread-safe: materialise rows serially
  std::vector<Row> rows(num_rows);
  for (int i = 0; i < num_rows; ++i) rows[i] = get(i);
  *out = DatasetFromRows([&rows](int64_t r) { return rows[r]; }, num_rows, static_cast<int>(num_col), cfg,
                         static_cast<const Dataset*>(reference));
  API_END();
}

int LGBM_DatasetCreateFromCSC(const void* col_ptr, int col_ptr_type, const int32_t* indices, const void* data,
                              int data_type, int64_t ncol_ptr, int64_t, int64_t num_row, const char* parameters,
                              const DatasetHandle reference, DatasetHandle* out) {
  API_BEGIN();
  Config cfg = ParamsToConfig(parameters);
  auto rows = CSCToRows(col_ptr, col_ptr_type, indices, data, data_type, ncol_ptr, num_row);
  *out = DatasetFromRows([&rows](int64_t r) { return rows[r]; }, static_cast<data_size_t>(num_row),
                         static_cast<int>(ncol_ptr - 1), cfg, static_cast<const Dataset*>(reference));
  API_END();
}

int LGBM_DatasetCreateFromMat(const void* data, int data_type, int32_t nrow, int32_t ncol, int is_row_major,
                              const char* parameters, const DatasetHandle reference, DatasetHandle* out) {
  API_BEGIN();
  Config cfg = ParamsToConfig(parameters);
  if (data_type != C_API_DTYPE_FLOAT32 && data_type != C_API_DTYPE_FLOAT64) Log::Fatal("Unknown data type");
  // dense fast path: bins from a row sample, then every row pushed column by column
  std::unique_ptr<Dataset> ds;
  if (reference == nullptr) {
    auto get = DenseRowPairFun(data, data_type, nrow, ncol, is_row_major);
    auto idx = SampleRows(cfg, nrow);
    std::vector<std::vector<double>> sv(ncol);
    std::vector<std::vector<int>> si(ncol);
    for (size_t i = 0; i < idx.size(); ++i) {
      for (auto& kv : get(idx[i])) {
        sv[kv.first].push_back(kv.second);
        si[kv.first].push_back(static_cast<int>(i));
      }
    }
    ds.reset(ConstructFromSamples(&sv, &si, ncol, idx.size(), nrow, cfg));
  } else {
    ds.reset(new Dataset(nrow));
    ds->CreateValid(*static_cast<const Dataset*>(reference), nrow);
    ds->metadata().Init(nrow, false, false);
  }
  const int64_t rs = is_row_major ? ncol : 1, cs = is_row_major ? 1 : nrow;
  // numerical groups binned on the device (large matrices, device_type=gpu); the host pushes
  // the remaining columns
  std::vector<int> host_cols;
  if (UseDeviceBinning(cfg, nrow, ncol)) {
    const auto done = DeviceBinDenseMatrix(ds.get(), data, data_type == C_API_DTYPE_FLOAT64, nrow, ncol,
                                           is_row_major != 0, cfg);
    for (int j = 0; j < ncol; ++j) {
      if (!done[j] && ds->InnerFeatureIndex(j) >= 0) host_cols.push_back(j);
    }
  } else {
    for (int j = 0; j < ncol; ++j) host_cols.push_back(j);
  }
  common::OmpErrors errors;
  if (!host_cols.empty()) {
#pragma omp parallel
    {
      std::vector<double> buf(ncol);
#pragma omp for schedule(static)
      for (int32_t r = 0; r < nrow; ++r) {
        errors.Run([&] {
          if (data_type == C_API_DTYPE_FLOAT32) {
            const float* p = static_cast<const float*>(data) + rs * r;
            for (int j : host_cols) buf[j] = p[cs * j];
          } else {
            const double* p = static_cast<const double*>(data) + rs * r;
            for (int j : host_cols) buf[j] = p[cs * j];
          }
          for (int j : host_cols) ds->PushColumnValue(r, j, buf[j]);
        });
      }
    }
  }
  errors.Check();
  ds->FinishLoad();
  *out = ds.release();
  API_END();
}

int LGBM_DatasetCreateFromMats(int32_t nmat, const void** data, int data_type, int32_t* nrow, int32_t ncol,
                               int is_row_major, const char* parameters, const DatasetHandle reference,
                               DatasetHandle* out) {
  API_BEGIN();
  Config cfg = ParamsToConfig(parameters);
  std::vector<std::function<Row(int)>> funs;
  std::vector<int64_t> starts(1, 0);
  for (int m = 0; m < nmat; ++m) {
    funs.push_back(DenseRowPairFun(data[m], data_type, nrow[m], ncol, is_row_major));
    starts.push_back(starts.back() + nrow[m]);
  }
  auto get = [&](int64_t r) {
    const int m = static_cast<int>(std::upper_bound(starts.begin(), starts.end(), r) - starts.begin()) - 1;
    return funs[m](static_cast<int>(r - starts[m]));
  };
  *out = DatasetFromRows(get, static_cast<data_size_t>(starts.back()), ncol, cfg,
                         static_cast<const Dataset*>(reference));
  API_END();
}

int LGBM_DatasetGetSubset(const DatasetHandle handle, const int32_t* used_row_indices, int32_t num_used_row_indices,
                          const char* parameters, DatasetHandle* out) {
  API_BEGIN();
  ParamsToConfig(parameters);
  const auto* full = static_cast<const Dataset*>(handle);
  for (int32_t i = 0; i < num_used_row_indices; ++i) {
    if (used_row_indices[i] < 0 || used_row_indices[i] >= full->num_data()) Log::Fatal("Used row index out of range");
  }
  std::unique_ptr<Dataset> ds(new Dataset(num_used_row_indices));
  ds->CopySubrow(*full, used_row_indices, num_used_row_indices);
  ds->FinishLoad();
  *out = ds.release();
  API_END();
}

int LGBM_DatasetSetFeatureNames(DatasetHandle handle, const char** feature_names, int num_feature_names) {
  API_BEGIN();
  std::vector<std::string> names(feature_names, feature_names + num_feature_names);
  static_cast<Dataset*>(handle)->set_feature_names(names);
  API_END();
}

int LGBM_DatasetGetFeatureNames(DatasetHandle handle, const int len, int* num_feature_names, const size_t buffer_len,
                                size_t* out_buffer_len, char** feature_names) {
  API_BEGIN();
  CopyStrings(static_cast<Dataset*>(handle)->feature_names(), len, num_feature_names, buffer_len, out_buffer_len,
              feature_names);
  API_END();
}

int LGBM_DatasetFree(DatasetHandle handle) {
  API_BEGIN();
  delete static_cast<Dataset*>(handle);
  API_END();
}

int LGBM_DatasetSaveBinary(DatasetHandle handle, const char* filename) {
  API_BEGIN();
  static_cast<Dataset*>(handle)->SaveBinaryFile(filename);
  API_END();
}

int LGBM_DatasetDumpText(DatasetHandle handle, const char* filename) {
  API_BEGIN();
  static_cast<Dataset*>(handle)->DumpText(filename);
  API_END();
}

int LGBM_DatasetSetField(DatasetHandle handle, const char* field_name, const void* field_data, int num_element,
                         int type) {
  API_BEGIN();
  auto* ds = static_cast<Dataset*>(handle);
  const std::string name(field_name);
  Metadata& md = ds->metadata();
  if (name == "label" || name == "target") {
    if (type != C_API_DTYPE_FLOAT32) Log::Fatal("label should be float32");
    md.SetLabel(static_cast<const label_t*>(field_data), num_element);
  } else if (name == "weight" || name == "weights") {
    if (type != C_API_DTYPE_FLOAT32) Log::Fatal("weight should be float32");
    md.SetWeights(static_cast<const label_t*>(field_data), num_element);
  } else if (name == "init_score") {
    if (type != C_API_DTYPE_FLOAT64) Log::Fatal("init_score should be float64");
    md.SetInitScore(static_cast<const double*>(field_data), num_element);
  } else if (name == "group" || name == "query") {
    if (type != C_API_DTYPE_INT32) Log::Fatal("group should be int32");
    md.SetQuery(static_cast<const int32_t*>(field_data), num_element);
  } else {
    Log::Fatal("Input data type error or field not found");
  }
  API_END();
}

int LGBM_DatasetGetField(DatasetHandle handle, const char* field_name, int* out_len, const void** out_ptr,
                         int* out_type) {
  API_BEGIN();
  auto* ds = static_cast<Dataset*>(handle);
  const std::string name(field_name);
  const Metadata& md = ds->metadata();
  *out_ptr = nullptr;
  *out_len = 0;
  if (name == "label" || name == "target") {
    *out_ptr = md.label();
    *out_len = md.num_data();
    *out_type = C_API_DTYPE_FLOAT32;
  } else if (name == "weight" || name == "weights") {
    if (md.weights() != nullptr) {
      *out_ptr = md.weights();
      *out_len = md.num_data();
    }
    *out_type = C_API_DTYPE_FLOAT32;
  } else if (name == "init_score") {
    if (md.init_score() != nullptr) {
      *out_ptr = md.init_score();
      *out_len = static_cast<int>(md.num_init_score());
    }
    *out_type = C_API_DTYPE_FLOAT64;
  } else if (name == "group" || name == "query") {
    if (md.query_boundaries() != nullptr) {
      *out_ptr = md.query_boundaries();
      *out_len = md.num_queries() + 1;
    }
    *out_type = C_API_DTYPE_INT32;
  } else {
    Log::Fatal("Field not found");
  }
  API_END();
}

int LGBM_DatasetUpdateParamChecking(const char* old_parameters, const char* new_parameters) {
  API_BEGIN();
  auto op = Config::Str2Map(old_parameters);
  Config oc;
  oc.Set(op);
  auto np = Config::Str2Map(new_parameters);
  Booster::CheckDatasetResetConfig(oc, np);
  API_END();
}

int LGBM_DatasetGetNumData(DatasetHandle handle, int* out) {
  API_BEGIN();
  *out = static_cast<Dataset*>(handle)->num_data();
  API_END();
}

int LGBM_DatasetGetNumFeature(DatasetHandle handle, int* out) {
  API_BEGIN();
  *out = static_cast<Dataset*>(handle)->num_total_features();
  API_END();
}

int LGBM_DatasetAddFeaturesFrom(DatasetHandle target, DatasetHandle source) {
  API_BEGIN();
  static_cast<Dataset*>(target)->AddFeaturesFrom(*static_cast<Dataset*>(source));
  API_END();
}

// ---------------------------------------------------------------------- booster
// the booster's reader / writer lock for C API calls outside the Booster methods (readers of
// the model and its state share it; training, model changes and evaluation take it alone)
static std::shared_lock<std::shared_mutex> ReadLock(BoosterHandle h) {
  return std::shared_lock<std::shared_mutex>(static_cast<Booster*>(h)->mutex());
}
static std::unique_lock<std::shared_mutex> WriteLock(BoosterHandle h) {
  return std::unique_lock<std::shared_mutex>(static_cast<Booster*>(h)->mutex());
}

int LGBM_BoosterCreate(const DatasetHandle train_data, const char* parameters, BoosterHandle* out) {
  API_BEGIN();
  *out = new Booster(static_cast<const Dataset*>(train_data), parameters);
  API_END();
}

int LGBM_BoosterCreateFromModelfile(const char* filename, int* out_num_iterations, BoosterHandle* out) {
  API_BEGIN();
  auto* b = new Booster(filename);
  *out_num_iterations = b->boosting()->GetCurrentIteration();
  *out = b;
  API_END();
}

int LGBM_BoosterLoadModelFromString(const char* model_str, int* out_num_iterations, BoosterHandle* out) {
  API_BEGIN();
  std::unique_ptr<Booster> b(new Booster());
  b->LoadModelFromString(model_str);
  *out_num_iterations = b->boosting()->GetCurrentIteration();
  *out = b.release();
  API_END();
}

int LGBM_BoosterFree(BoosterHandle handle) {
  API_BEGIN();
  delete static_cast<Booster*>(handle);
  API_END();
}

int LGBM_BoosterShuffleModels(BoosterHandle handle, int start_iter, int end_iter) {
  API_BEGIN();
  const auto booster_lock = WriteLock(handle);
  static_cast<Booster*>(handle)->boosting()->ShuffleModels(start_iter, end_iter);
  API_END();
}

int LGBM_BoosterMerge(BoosterHandle handle, BoosterHandle other_handle) {
  API_BEGIN();
  static_cast<Booster*>(handle)->MergeFrom(static_cast<Booster*>(other_handle));
  API_END();
}

int LGBM_BoosterAddValidData(BoosterHandle handle, const DatasetHandle valid_data) {
  API_BEGIN();
  static_cast<Booster*>(handle)->AddValidData(static_cast<const Dataset*>(valid_data));
  API_END();
}

int LGBM_BoosterResetTrainingData(BoosterHandle handle, const DatasetHandle train_data) {
  API_BEGIN();
  static_cast<Booster*>(handle)->ResetTrainingData(static_cast<const Dataset*>(train_data));
  API_END();
}

int LGBM_BoosterResetParameter(BoosterHandle handle, const char* parameters) {
  API_BEGIN();
  static_cast<Booster*>(handle)->ResetConfig(parameters);
  API_END();
}

int LGBM_BoosterGetNumClasses(BoosterHandle handle, int* out_len) {
  API_BEGIN();
  const auto booster_lock = ReadLock(handle);
  *out_len = static_cast<Booster*>(handle)->boosting()->NumberOfClasses();
  API_END();
}

int LGBM_BoosterUpdateOneIter(BoosterHandle handle, int* is_finished) {
  API_BEGIN();
  common::ScopedTimer timer("LGBM_BoosterUpdateOneIter");
  *is_finished = static_cast<Booster*>(handle)->TrainOneIter() ? 1 : 0;
  API_END();
}

int LGBM_BoosterRefit(BoosterHandle handle, const int32_t* leaf_preds, int32_t nrow, int32_t ncol) {
  API_BEGIN();
  static_cast<Booster*>(handle)->Refit(leaf_preds, nrow, ncol);
  API_END();
}

int LGBM_BoosterUpdateOneIterCustom(BoosterHandle handle, const float* grad, const float* hess, int* is_finished) {
  API_BEGIN();
  *is_finished = static_cast<Booster*>(handle)->TrainOneIter(grad, hess) ? 1 : 0;
  API_END();
}

int LGBM_BoosterRollbackOneIter(BoosterHandle handle) {
  API_BEGIN();
  static_cast<Booster*>(handle)->RollbackOneIter();
  API_END();
}

int LGBM_BoosterGetCurrentIteration(BoosterHandle handle, int* out_iteration) {
  API_BEGIN();
  const auto booster_lock = ReadLock(handle);
  *out_iteration = static_cast<Booster*>(handle)->boosting()->GetCurrentIteration();
  API_END();
}

int LGBM_BoosterNumModelPerIteration(BoosterHandle handle, int* out_tree_per_iteration) {
  API_BEGIN();
  const auto booster_lock = ReadLock(handle);
  *out_tree_per_iteration = static_cast<Booster*>(handle)->boosting()->NumModelPerIteration();
  API_END();
}

int LGBM_BoosterNumberOfTotalModel(BoosterHandle handle, int* out_models) {
  API_BEGIN();
  const auto booster_lock = ReadLock(handle);
  *out_models = static_cast<Booster*>(handle)->boosting()->NumberOfTotalModel();
  API_END();
}

int LGBM_BoosterGetEvalCounts(BoosterHandle handle, int* out_len) {
  API_BEGIN();
  const auto booster_lock = ReadLock(handle);
  *out_len = static_cast<Booster*>(handle)->boosting()->GetEvalCounts();
  API_END();
}

int LGBM_BoosterGetEvalNames(BoosterHandle handle, const int len, int* out_len, const size_t buffer_len,
                             size_t* out_buffer_len, char** out_strs) {
  API_BEGIN();
  const auto booster_lock = ReadLock(handle);
  CopyStrings(static_cast<Booster*>(handle)->boosting()->GetEvalNames(), len, out_len, buffer_len, out_buffer_len,
              out_strs);
  API_END();
}

int LGBM_BoosterGetFeatureNames(BoosterHandle handle, const int len, int* out_len, const size_t buffer_len,
                                size_t* out_buffer_len, char** out_strs) {
  API_BEGIN();
  const auto booster_lock = ReadLock(handle);
  CopyStrings(static_cast<Booster*>(handle)->boosting()->FeatureNames(), len, out_len, buffer_len, out_buffer_len,
              out_strs);
  API_END();
}

int LGBM_BoosterGetNumFeature(BoosterHandle handle, int* out_len) {
  API_BEGIN();
  const auto booster_lock = ReadLock(handle);
  *out_len = static_cast<Booster*>(handle)->boosting()->MaxFeatureIdx() + 1;
  API_END();
}

int LGBM_BoosterGetEval(BoosterHandle handle, int data_idx, int* out_len, double* out_results) {
  API_BEGIN();
  const auto booster_lock = WriteLock(handle);
  auto r = static_cast<Booster*>(handle)->GetEval(data_idx);
  *out_len = static_cast<int>(r.size());
  std::copy(r.begin(), r.end(), out_results);
  API_END();
}

int LGBM_BoosterGetNumPredict(BoosterHandle handle, int data_idx, int64_t* out_len) {
  API_BEGIN();
  const auto booster_lock = ReadLock(handle);
  *out_len = static_cast<Booster*>(handle)->boosting()->GetNumPredictAt(data_idx);
  API_END();
}

int LGBM_BoosterGetPredict(BoosterHandle handle, int data_idx, int64_t* out_len, double* out_result) {
  API_BEGIN();
  const auto booster_lock = WriteLock(handle);
  static_cast<Booster*>(handle)->boosting()->GetPredictAt(data_idx, out_result, out_len);
  API_END();
}

int LGBM_BoosterPredictForFile(BoosterHandle handle, const char* data_filename, int data_has_header,
                               int predict_type, int start_iteration, int num_iteration, const char* parameter,
                               const char* result_filename) {
  API_BEGIN();
  Config cfg = ParamsToConfig(parameter);
  static_cast<Booster*>(handle)->PredictFile(data_filename, data_has_header, predict_type, start_iteration,
                                              num_iteration, cfg, result_filename);
  API_END();
}

int LGBM_BoosterCalcNumPredict(BoosterHandle handle, int num_row, int predict_type, int start_iteration,
                               int num_iteration, int64_t* out_len) {
  API_BEGIN();
  const auto booster_lock = ReadLock(handle);
  *out_len = static_cast<int64_t>(num_row) *
             static_cast<Booster*>(handle)->boosting()->NumPredictOneRow(
                 start_iteration, num_iteration, predict_type == C_API_PREDICT_LEAF_INDEX,
                 predict_type == C_API_PREDICT_CONTRIB);
  API_END();
}

int LGBM_FastConfigFree(FastConfigHandle fastConfig) {
  API_BEGIN();
  delete static_cast<FastConfig*>(fastConfig);
  API_END();
}

int LGBM_BoosterPredictForCSR(BoosterHandle handle, const void* indptr, int indptr_type, const int32_t* indices,
                              const void* data, int data_type, int64_t nindptr, int64_t nelem, int64_t num_col,
                              int predict_type, int start_iteration, int num_iteration, const char* parameter,
                              int64_t* out_len, double* out_result) {
  API_BEGIN();
  if (num_col <= 0) Log::Fatal("The number of columns should be greater than zero.");
  Config cfg = ParamsToConfig(parameter);
  auto get = CSRRowFun(indptr, indptr_type, indices, data, data_type, nindptr, nelem);
  static_cast<Booster*>(handle)->PredictRows(get, nindptr - 1, num_col, predict_type, start_iteration, num_iteration,
                                              cfg, out_result, out_len);
  API_END();
}

int LGBM_BoosterPredictSparseOutput(BoosterHandle handle, const void* indptr, int indptr_type, const int32_t* indices,
                                    const void* data, int data_type, int64_t nindptr, int64_t nelem,
                                    int64_t num_col_or_row, int predict_type, int start_iteration, int num_iteration,
                                    const char* parameter, int matrix_type, int64_t* out_len, void** out_indptr,
                                    int32_t** out_indices, void** out_data) {
  API_BEGIN();
  if (predict_type != C_API_PREDICT_CONTRIB) Log::Fatal("Sparse output is only supported for contributions");
  Config cfg = ParamsToConfig(parameter);
  auto* b = static_cast<Booster*>(handle);
  std::vector<Row> rows;
  int64_t nrow, ncol;
  if (matrix_type == C_API_MATRIX_TYPE_CSR) {
    auto get = CSRRowFun(indptr, indptr_type, indices, data, data_type, nindptr, nelem);
    nrow = nindptr - 1;
    ncol = num_col_or_row;
    rows.resize(nrow);
    for (int64_t i = 0; i < nrow; ++i) rows[i] = get(i);
  } else if (matrix_type == C_API_MATRIX_TYPE_CSC) {
    nrow = num_col_or_row;
    ncol = nindptr - 1;
    rows = CSCToRows(indptr, indptr_type, indices, data, data_type, nindptr, nrow);
  } else {
    Log::Fatal("Unknown matrix type in LGBM_BoosterPredictSparseOutput");
  }
  const int ntpi = b->boosting()->NumModelPerIteration();
  const int64_t width = ntpi * (b->boosting()->MaxFeatureIdx() + 2);
  std::vector<double> dense(static_cast<size_t>(nrow) * width);
  int64_t dl = 0;
  b->PredictRows([&rows](int64_t r) { return rows[r]; }, nrow, ncol, predict_type, start_iteration, num_iteration,
                 cfg, dense.data(), &dl);
  // per class k: matrix nrow x (nf+1).  CSR: indptr over (k, row); CSC: indptr over (k, col).
  const int64_t nfp1 = width / ntpi;
  std::vector<int64_t> ptr;
  std::vector<int32_t> idx;
  std::vector<double> val;
  if (matrix_type == C_API_MATRIX_TYPE_CSR) {
    ptr.push_back(0);
    for (int k = 0; k < ntpi; ++k) {
      for (int64_t r = 0; r < nrow; ++r) {
        for (int64_t c = 0; c < nfp1; ++c) {
          const double v = dense[r * width + k * nfp1 + c];
          if (v != 0.0) {
            idx.push_back(static_cast<int32_t>(c));
            val.push_back(v);
          }
        }
        ptr.push_back(static_cast<int64_t>(val.size()));
      }
      if (k + 1 < ntpi) ptr.push_back(static_cast<int64_t>(val.size()));
    }
  } else {
    for (int k = 0; k < ntpi; ++k) {
      ptr.push_back(static_cast<int64_t>(val.size()));
      for (int64_t c = 0; c < nfp1; ++c) {
        for (int64_t r = 0; r < nrow; ++r) {
          const double v = dense[r * width + k * nfp1 + c];
          if (v != 0.0) {
            idx.push_back(static_cast<int32_t>(r));
            val.push_back(v);
          }
        }
        ptr.push_back(static_cast<int64_t>(val.size()));
      }
    }
  }
  out_len[0] = static_cast<int64_t>(val.size());
  out_len[1] = static_cast<int64_t>(ptr.size());
  if (indptr_type == C_API_DTYPE_INT32) {
    auto* p = new int32_t[ptr.size()];
    for (size_t i = 0; i < ptr.size(); ++i) p[i] = static_cast<int32_t>(ptr[i]);
    *out_indptr = p;
  } else {
    auto* p = new int64_t[ptr.size()];
    std::copy(ptr.begin(), ptr.end(), p);
    *out_indptr = p;
  }
  auto* ii = new int32_t[std::max<size_t>(1, idx.size())];
  std::copy(idx.begin(), idx.end(), ii);
  *out_indices = ii;
  if (data_type == C_API_DTYPE_FLOAT32) {
    auto* d = new float[std::max<size_t>(1, val.size())];
    for (size_t i = 0; i < val.size(); ++i) d[i] = static_cast<float>(val[i]);
    *out_data = d;
  } else {
    auto* d = new double[std::max<size_t>(1, val.size())];
    std::copy(val.begin(), val.end(), d);
    *out_data = d;
  }
  API_END();
}

int LGBM_BoosterFreePredictSparse(void* indptr, int32_t* indices, void* data, int indptr_type, int data_type) {
  API_BEGIN();
  if (indptr_type == C_API_DTYPE_INT32) delete[] static_cast<int32_t*>(indptr);
  else delete[] static_cast<int64_t*>(indptr);
  delete[] indices;
  if (data_type == C_API_DTYPE_FLOAT32) delete[] static_cast<float*>(data);
  else delete[] static_cast<double*>(data);
  API_END();
}

int LGBM_BoosterPredictForCSRSingleRow(BoosterHandle handle, const void* indptr, int indptr_type,
                                       const int32_t* indices, const void* data, int data_type, int64_t nindptr,
                                       int64_t nelem, int64_t num_col, int predict_type, int start_iteration,
                                       int num_iteration, const char* parameter, int64_t* out_len,
                                       double* out_result) {
  return LGBM_BoosterPredictForCSR(handle, indptr, indptr_type, indices, data, data_type, nindptr, nelem, num_col,
                                   predict_type, start_iteration, num_iteration, parameter, out_len, out_result);
}

int LGBM_BoosterPredictForCSRSingleRowFastInit(BoosterHandle handle, const int predict_type,
                                               const int start_iteration, const int num_iteration,
                                               const int data_type, const int64_t num_col, const char* parameter,
                                               FastConfigHandle* out_fastConfig) {
  API_BEGIN();
  std::unique_ptr<FastConfig> fc(new FastConfig());
  fc->booster = static_cast<Booster*>(handle);
  fc->config = ParamsToConfig(parameter);
  fc->predict_type = predict_type;
  fc->start_iteration = start_iteration;
  fc->num_iteration = num_iteration;
  fc->data_type = data_type;
  fc->ncol = num_col;
  fc->predictor = fc->booster->MakePredictor(predict_type, start_iteration, num_iteration, fc->config);
  *out_fastConfig = fc.release();
  API_END();
}

int LGBM_BoosterPredictForCSRSingleRowFast(FastConfigHandle fastConfig_handle, const void* indptr,
                                           const int indptr_type, const int32_t* indices, const void* data,
                                           const int64_t nindptr, const int64_t nelem, int64_t* out_len,
                                           double* out_result) {
  API_BEGIN();
  auto* fc = static_cast<FastConfig*>(fastConfig_handle);
  auto get = CSRRowFun(indptr, indptr_type, indices, data, fc->data_type, nindptr, nelem);
  std::unique_lock<std::shared_mutex> l(fc->booster->mutex());
  fc->predictor->Predict(get(0), out_result);
  *out_len = fc->predictor->num_pred_one_row();
  API_END();
}

int LGBM_BoosterPredictForCSC(BoosterHandle handle, const void* col_ptr, int col_ptr_type, const int32_t* indices,
                              const void* data, int data_type, int64_t ncol_ptr, int64_t, int64_t num_row,
                              int predict_type, int start_iteration, int num_iteration, const char* parameter,
                              int64_t* out_len, double* out_result) {
  API_BEGIN();
  Config cfg = ParamsToConfig(parameter);
  auto rows = CSCToRows(col_ptr, col_ptr_type, indices, data, data_type, ncol_ptr, num_row);
  static_cast<Booster*>(handle)->PredictRows([&rows](int64_t r) { return rows[r]; }, num_row, ncol_ptr - 1,
                                              predict_type, start_iteration, num_iteration, cfg, out_result, out_len);
  API_END();
}

int LGBM_BoosterPredictForMat(BoosterHandle handle, const void* data, int data_type, int32_t nrow, int32_t ncol,
                              int is_row_major, int predict_type, int start_iteration, int num_iteration,
                              const char* parameter, int64_t* out_len, double* out_result) {
  API_BEGIN();
  Config cfg = ParamsToConfig(parameter);
  Booster* b = static_cast<Booster*>(handle);
  if (b->PredictDenseOnDevice(data, data_type, nrow, ncol, is_row_major, predict_type, start_iteration,
                              num_iteration, cfg, out_result, out_len)) {
    return 0;
  }
  auto get = DenseRowPairFun(data, data_type, nrow, ncol, is_row_major);
  b->PredictRows([&get](int64_t r) { return get(static_cast<int>(r)); }, nrow, ncol, predict_type, start_iteration,
                 num_iteration, cfg, out_result, out_len);
  API_END();
}

int LGBM_BoosterPredictForMatSingleRow(BoosterHandle handle, const void* data, int data_type, int ncol,
                                       int is_row_major, int predict_type, int start_iteration, int num_iteration,
                                       const char* parameter, int64_t* out_len, double* out_result) {
  return LGBM_BoosterPredictForMat(handle, data, data_type, 1, ncol, is_row_major, predict_type, start_iteration,
                                   num_iteration, parameter, out_len, out_result);
}

int LGBM_BoosterPredictForMatSingleRowFastInit(BoosterHandle handle, const int predict_type,
                                               const int start_iteration, const int num_iteration,
                                               const int data_type, const int32_t ncol, const char* parameter,
                                               FastConfigHandle* out_fastConfig) {
  return LGBM_BoosterPredictForCSRSingleRowFastInit(handle, predict_type, start_iteration, num_iteration, data_type,
                                                    ncol, parameter, out_fastConfig);
}

int LGBM_BoosterPredictForMatSingleRowFast(FastConfigHandle fastConfig_handle, const void* data, int64_t* out_len,
                                           double* out_result) {
  API_BEGIN();
  auto* fc = static_cast<FastConfig*>(fastConfig_handle);
  auto get = DenseRowPairFun(data, fc->data_type, 1, static_cast<int>(fc->ncol), 1);
  std::unique_lock<std::shared_mutex> l(fc->booster->mutex());
  fc->predictor->Predict(get(0), out_result);
  *out_len = fc->predictor->num_pred_one_row();
  API_END();
}

int LGBM_BoosterPredictForMats(BoosterHandle handle, const void** data, int data_type, int32_t nrow, int32_t ncol,
                               int predict_type, int start_iteration, int num_iteration, const char* parameter,
                               int64_t* out_len, double* out_result) {
  API_BEGIN();
  Config cfg = ParamsToConfig(parameter);
  auto get = MatsRowPairFun(data, data_type, nrow, ncol);
  static_cast<Booster*>(handle)->PredictRows([&get](int64_t r) { return get(static_cast<int>(r)); }, nrow, ncol,
                                              predict_type, start_iteration, num_iteration, cfg, out_result, out_len);
  API_END();
}

int LGBM_BoosterSaveModel(BoosterHandle handle, int start_iteration, int num_iteration, int feature_importance_type,
                          const char* filename) {
  API_BEGIN();
  const auto booster_lock = ReadLock(handle);
  static_cast<Booster*>(handle)->boosting()->SaveModelToFile(start_iteration, num_iteration, feature_importance_type,
                                                              filename);
  API_END();
}

int LGBM_BoosterSaveModelToString(BoosterHandle handle, int start_iteration, int num_iteration,
                                  int feature_importance_type, int64_t buffer_len, int64_t* out_len, char* out_str) {
  API_BEGIN();
  const auto booster_lock = ReadLock(handle);
  std::string s = static_cast<Booster*>(handle)->boosting()->SaveModelToString(start_iteration, num_iteration,
                                                                               feature_importance_type);
  *out_len = static_cast<int64_t>(s.size()) + 1;
  if (*out_len <= buffer_len) std::memcpy(out_str, s.c_str(), *out_len);
  API_END();
}

int LGBM_BoosterDumpModel(BoosterHandle handle, int start_iteration, int num_iteration, int feature_importance_type,
                          int64_t buffer_len, int64_t* out_len, char* out_str) {
  API_BEGIN();
  const auto booster_lock = ReadLock(handle);
  std::string s =
      static_cast<Booster*>(handle)->boosting()->DumpModel(start_iteration, num_iteration, feature_importance_type);
  *out_len = static_cast<int64_t>(s.size()) + 1;
  if (*out_len <= buffer_len) std::memcpy(out_str, s.c_str(), *out_len);
  API_END();
}

int LGBM_BoosterGetLeafValue(BoosterHandle handle, int tree_idx, int leaf_idx, double* out_val) {
  API_BEGIN();
  const auto booster_lock = ReadLock(handle);
  *out_val = static_cast<Booster*>(handle)->boosting()->GetLeafValue(tree_idx, leaf_idx);
  API_END();
}

int LGBM_BoosterSetLeafValue(BoosterHandle handle, int tree_idx, int leaf_idx, double val) {
  API_BEGIN();
  auto* b = static_cast<Booster*>(handle);
  std::unique_lock<std::shared_mutex> l(b->mutex());
  b->boosting()->SetLeafValue(tree_idx, leaf_idx, val);
  API_END();
}

int LGBM_BoosterFeatureImportance(BoosterHandle handle, int num_iteration, int importance_type, double* out_results) {
  API_BEGIN();
  const auto booster_lock = ReadLock(handle);
  auto v = static_cast<Booster*>(handle)->boosting()->FeatureImportance(num_iteration, importance_type);
  std::copy(v.begin(), v.end(), out_results);
  API_END();
}

int LGBM_BoosterGetUpperBoundValue(BoosterHandle handle, double* out_results) {
  API_BEGIN();
  const auto booster_lock = ReadLock(handle);
  *out_results = static_cast<Booster*>(handle)->boosting()->GetUpperBoundValue();
  API_END();
}

int LGBM_BoosterGetLowerBoundValue(BoosterHandle handle, double* out_results) {
  API_BEGIN();
  const auto booster_lock = ReadLock(handle);
  *out_results = static_cast<Booster*>(handle)->boosting()->GetLowerBoundValue();
  API_END();
}

int LGBM_NetworkInit(const char* machines, int local_listen_port, int listen_time_out, int num_machines) {
  API_BEGIN();
  Config cfg;
  cfg.machines = machines;
  cfg.local_listen_port = local_listen_port;
  cfg.time_out = listen_time_out;
  cfg.num_machines = num_machines;
  if (num_machines > 1) Network::Init(cfg);
  API_END();
}

int LGBM_NetworkFree() {
  API_BEGIN();
  Network::Dispose();
  API_END();
}

int LGBM_NetworkInitWithFunctions(int num_machines, int rank, void* reduce_scatter_ext_fun, void* allgather_ext_fun) {
  API_BEGIN();
  if (num_machines > 1) {
    Network::InitWithFunctions(num_machines, rank, reinterpret_cast<ReduceScatterFunctionPtr>(reduce_scatter_ext_fun),
                               reinterpret_cast<AllgatherFunctionPtr>(allgather_ext_fun));
  }
  API_END();
}

int LGBM_AMD_DatasetGetGroupBins(DatasetHandle handle, int32_t* bins, int64_t* boundaries, int* num_groups) {
  API_BEGIN();
  const Dataset* d = static_cast<const Dataset*>(handle);
  const int ng = d->num_groups();
  *num_groups = ng;
  if (boundaries != nullptr) {
    for (int g = 0; g <= ng; ++g) {
      boundaries[g] = static_cast<int64_t>(g < ng ? d->group_bin_boundary(g) : d->num_total_bin());
    }
  }
  if (bins != nullptr) {
    const data_size_t n = d->num_data();
#pragma omp parallel for schedule(static)
    for (data_size_t r = 0; r < n; ++r) {
      for (int g = 0; g < ng; ++g) bins[static_cast<size_t>(r) * ng + g] = static_cast<int32_t>(d->group(g).Get(r));
    }
  }
  API_END();
}

namespace {
DeviceTreeLearner* DeviceLearnerOf(BoosterHandle handle) {
  DeviceTreeLearner* dl = static_cast<Booster*>(handle)->boosting()->device_learner();
  if (dl == nullptr) Log::Fatal("the booster does not train on a device (device_type=gpu)");
  return dl;
}
}  // namespace

int LGBM_AMD_BoosterDeviceLeafState(BoosterHandle handle, int leaf, int32_t* rows, int* count, int64_t* hist,
                                    int8_t* bin_valid, int64_t* hist_len, double* sums) {
  API_BEGIN();
  std::vector<int32_t> r;
  std::vector<long long> h;
  std::vector<int8_t> valid;
  double s[3];
  GBDT* b = static_cast<Booster*>(handle)->boosting();
  const int nm = b->NumberOfTotalModel();
  if (!DeviceLearnerOf(handle)->DebugLeafState(nm > 0 ? b->model(nm - 1) : nullptr, leaf, &r, &h, &valid, s)) {
    Log::Fatal("no device-resident tree state for leaf %d", leaf);
  }
  *count = static_cast<int>(r.size());
  *hist_len = static_cast<int64_t>(h.size());
  if (rows != nullptr) std::memcpy(rows, r.data(), sizeof(int32_t) * r.size());
  if (hist != nullptr) std::memcpy(hist, h.data(), sizeof(long long) * h.size());
  if (bin_valid != nullptr) std::memcpy(bin_valid, valid.data(), valid.size());
  if (sums != nullptr) std::memcpy(sums, s, sizeof(s));
  API_END();
}

int LGBM_AMD_BoosterDeviceGradients(BoosterHandle handle, float* grad, float* hess, double* scales) {
  API_BEGIN();
  std::vector<float> g, h;
  if (!DeviceLearnerOf(handle)->DebugGradients(&g, &h, scales)) Log::Fatal("no device gradients");
  std::memcpy(grad, g.data(), sizeof(float) * g.size());
  std::memcpy(hess, h.data(), sizeof(float) * h.size());
  API_END();
}

// the gradients the last iteration trained on, from the device learner or the host learner
// (n: entries available; grad / hess may be null to query it)
int LGBM_AMD_BoosterLastGradients(BoosterHandle handle, float* grad, float* hess, int64_t* n) {
  API_BEGIN();
  GBDT* b = static_cast<Booster*>(handle)->boosting();
  std::vector<float> g, h;
  if (b->device_learner() != nullptr) {
    const int64_t n_all = static_cast<int64_t>(b->train_num_data()) * b->NumModelPerIteration();
    g.resize(n_all);
    h.resize(n_all);
    b->device_learner()->DownloadGradients(g.data(), h.data(), n_all);
  } else {
    g = b->host_gradients();
    h = b->host_hessians();
  }
  *n = static_cast<int64_t>(g.size());
  if (grad != nullptr) std::memcpy(grad, g.data(), sizeof(float) * g.size());
  if (hess != nullptr) std::memcpy(hess, h.data(), sizeof(float) * h.size());
  API_END();
}

// free / total bytes of the calling thread's current HIP device
int LGBM_AMD_DeviceMemInfo(int64_t* free_bytes, int64_t* total_bytes) {
  API_BEGIN();
  size_t f = 0, t = 0;
  if (hipMemGetInfo(&f, &t) != hipSuccess) {
    (void)hipGetLastError();
    Log::Fatal("hipMemGetInfo failed");
  }
  *free_bytes = static_cast<int64_t>(f);
  *total_bytes = static_cast<int64_t>(t);
  API_END();
}

int LGBM_AMD_BoosterGrowthStats(BoosterHandle handle, double* out, int n) {
  API_BEGIN();
  const double* s = static_cast<Booster*>(handle)->boosting()->growth_stats();
  for (int i = 0; i < n && i < 7; ++i) out[i] = s[i];
  API_END();
}

int LGBM_AMD_BoosterDeviceCheckSplits(BoosterHandle handle, int64_t buffer_len, int64_t* out_len, char* out_str) {
  API_BEGIN();
  GBDT* b = static_cast<Booster*>(handle)->boosting();
  const int n = b->NumberOfTotalModel();
  const std::string rep = DeviceLearnerOf(handle)->DebugCheckSplits(n > 0 ? b->model(n - 1) : nullptr);
  *out_len = static_cast<int64_t>(rep.size()) + 1;
  if (buffer_len >= *out_len) std::memcpy(out_str, rep.c_str(), rep.size() + 1);
  API_END();
}

int LGBM_AMD_NetworkReportExternalError(const char* msg) {
  API_BEGIN();
  Network::ReportExternalError(msg ? msg : "");
  API_END();
}

int LGBM_AMD_NetworkRank(int* out) {
  API_BEGIN();
  *out = Network::rank();
  API_END();
}

int LGBM_AMD_NetworkNumMachines(int* out) {
  API_BEGIN();
  *out = Network::num_machines();
  API_END();
}

int LGBM_AMD_NetworkAllgather(const void* input, const int64_t* block_len, void* output) {
  API_BEGIN();
  const int n = Network::num_machines();
  std::vector<comm_size_t> start(n), len(n);
  int64_t at = 0;
  for (int i = 0; i < n; ++i) {
    start[i] = static_cast<comm_size_t>(at);
    len[i] = static_cast<comm_size_t>(block_len[i]);
    at += block_len[i];
  }
  if (at > std::numeric_limits<comm_size_t>::max()) Log::Fatal("allgather of %lld bytes is too large", static_cast<long long>(at));
  Network::Allgather(static_cast<char*>(const_cast<void*>(input)), start.data(), len.data(), static_cast<char*>(output),
                     static_cast<comm_size_t>(at));
  API_END();
}

namespace {
void SumF64(const char* src, char* dst, int type_size, comm_size_t len) {
  (void)type_size;
  const double* s = reinterpret_cast<const double*>(src);
  double* d = reinterpret_cast<double*>(dst);
  for (comm_size_t i = 0; i < len / static_cast<comm_size_t>(sizeof(double)); ++i) d[i] += s[i];
}
}  // namespace

int LGBM_AMD_NetworkReduceScatterSumF64(const double* input, const int64_t* block_count, double* output) {
  API_BEGIN();
  const int n = Network::num_machines();
  std::vector<comm_size_t> start(n), len(n);
  int64_t at = 0;
  for (int i = 0; i < n; ++i) {
    start[i] = static_cast<comm_size_t>(at);
    len[i] = static_cast<comm_size_t>(block_count[i] * sizeof(double));
    at += block_count[i] * static_cast<int64_t>(sizeof(double));
  }
  if (at > std::numeric_limits<comm_size_t>::max()) Log::Fatal("reduce-scatter of %lld bytes is too large", static_cast<long long>(at));
  Network::ReduceScatter(reinterpret_cast<char*>(const_cast<double*>(input)), static_cast<comm_size_t>(at),
                         sizeof(double), start.data(), len.data(), reinterpret_cast<char*>(output),
                         len[Network::rank()], SumF64);
  API_END();
}

int LGBM_AMD_NetworkAllreduceSumF64(const double* input, int64_t count, double* output) {
  API_BEGIN();
  const int64_t bytes = count * static_cast<int64_t>(sizeof(double));
  if (bytes > std::numeric_limits<comm_size_t>::max()) Log::Fatal("all-reduce of %lld bytes is too large", static_cast<long long>(bytes));
  Network::Allreduce(reinterpret_cast<char*>(const_cast<double*>(input)), static_cast<comm_size_t>(bytes),
                     sizeof(double), reinterpret_cast<char*>(output), SumF64);
  API_END();
}

// in-process ranks (threads): a hub of thread transports; each rank's thread joins it
struct ThreadRankHub {
  std::vector<std::shared_ptr<HostTransport>> ranks;
};

int LGBM_AMD_NetworkCreateThreadHub(int num_ranks, double timeout_s, int fail_rank, int fail_at_call, void** out) {
  API_BEGIN();
  auto* h = new ThreadRankHub();
  h->ranks = MakeThreadTransports(num_ranks, timeout_s, fail_rank, fail_at_call);
  *out = h;
  API_END();
}

int LGBM_AMD_NetworkJoinThreadHub(void* hub, int rank) {
  API_BEGIN();
  auto* h = static_cast<ThreadRankHub*>(hub);
  if (rank < 0 || rank >= static_cast<int>(h->ranks.size())) Log::Fatal("rank %d out of range", rank);
  Network::InitWithTransport(h->ranks[rank]);
  API_END();
}

int LGBM_AMD_NetworkFreeThreadHub(void* hub) {
  API_BEGIN();
  delete static_cast<ThreadRankHub*>(hub);
  API_END();
}

// in-process device communicators for thread ranks sharing one GPU (src/network/
// inproc_device_comm.cpp); a rank thread joins after joining the host hub
struct DeviceRankHub {
  std::vector<std::shared_ptr<DeviceComm>> ranks;
};

int LGBM_AMD_DeviceCommCreateThreadHub(int num_ranks, double timeout_s, int fail_rank, int fail_at_call, void** out) {
  API_BEGIN();
  auto* h = new DeviceRankHub();
  h->ranks = MakeThreadDeviceComms(num_ranks, timeout_s, fail_rank, fail_at_call);
  *out = h;
  API_END();
}

// kind 0: host-rendezvous comm (eager launches); 1: capture-safe peer comm (one-shot kernels
// over the ranks' windows, src/network/peer_comm.cpp).  fail_at_call counts collectives
// (kind 1: executed on the device, so faults fire inside captured graphs too)
int LGBM_AMD_DeviceCommCreateThreadHubEx(int num_ranks, double timeout_s, int fail_rank, int fail_at_call, int kind,
                                         void** out) {
  API_BEGIN();
  auto* h = new DeviceRankHub();
  h->ranks = kind == 1 ? MakePeerThreadComms(num_ranks, timeout_s, fail_rank, fail_at_call)
                       : MakeThreadDeviceComms(num_ranks, timeout_s, fail_rank, fail_at_call);
  *out = h;
  API_END();
}

int LGBM_AMD_DeviceCommJoinThreadHub(void* hub, int rank) {
  API_BEGIN();
  auto* h = static_cast<DeviceRankHub*>(hub);
  if (rank < 0 || rank >= static_cast<int>(h->ranks.size())) Log::Fatal("rank %d out of range", rank);
  Network::SetDeviceComm(h->ranks[rank]);
  API_END();
}

int LGBM_AMD_DeviceCommFreeThreadHub(void* hub) {
  API_BEGIN();
  delete static_cast<DeviceRankHub*>(hub);
  API_END();
}

int LGBM_AMD_GetTimers(int64_t buffer_len, int64_t* out_len, char* out_str) {
  API_BEGIN();
  std::string s;
  for (auto& kv : common::PhaseTimer::Global().totals()) s += kv.first + "=" + std::to_string(kv.second / 1000.0) + ";";
  *out_len = static_cast<int64_t>(s.size()) + 1;
  if (*out_len <= buffer_len) std::memcpy(out_str, s.c_str(), *out_len);
  API_END();
}

int LGBM_AMD_BoosterSaveModelToIfElse(BoosterHandle handle, int num_iteration, const char* filename) {
  API_BEGIN();
  const auto booster_lock = ReadLock(handle);
  static_cast<Booster*>(handle)->boosting()->SaveModelToIfElse(num_iteration, filename);
  API_END();
}
