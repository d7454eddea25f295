// Config parsing, alias resolution and conflict checks.
// Behavioural parity with reference src/io/config.cpp:15-349 and
// include/LightGBM/config.h:1048-1146 (alias priority: shorter key wins, ties
// broken alphabetically; unknown keys warn; enum values normalised).
#include "lgbm_amd/config.h"

#include <cmath>
#include <sstream>

#include "lgbm_amd/common.h"
#include "lgbm_amd/log.h"
#include "lgbm_amd/random.h"

namespace lgbm_amd {

void Config::KV2Map(std::unordered_map<std::string, std::string>* params, const char* kv) {
  auto parts = common::Split(kv, '=');
  if (parts.size() != 1 && parts.size() != 2) {
    Log::Warning("Unknown parameter %s", kv);
    return;
  }
  std::string key = common::RemoveQuotationSymbol(common::Trim(parts[0]));
  std::string value = parts.size() == 2 ? common::RemoveQuotationSymbol(common::Trim(parts[1])) : "";
  if (key.empty()) return;
  auto it = params->find(key);
  if (it == params->end()) {
    params->emplace(key, value);
  } else {
    Log::Warning("%s is set=%s, %s=%s will be ignored. Current value: %s=%s", key.c_str(), it->second.c_str(),
                 key.c_str(), value.c_str(), key.c_str(), it->second.c_str());
  }
}

std::unordered_map<std::string, std::string> Config::Str2Map(const char* parameters) {
  std::unordered_map<std::string, std::string> params;
  for (const auto& arg : common::Split(parameters, " \t\n\r")) {
    KV2Map(&params, common::Trim(arg).c_str());
  }
  KeyAliasTransform(&params);
  return params;
}

void Config::KeyAliasTransform(std::unordered_map<std::string, std::string>* params) {
  // canonical name -> alias key chosen
  std::unordered_map<std::string, std::string> chosen;
  for (const auto& kv : *params) {
    auto a = alias_table().find(kv.first);
    if (a != alias_table().end()) {
      auto c = chosen.find(a->second);
      if (c == chosen.end()) {
        chosen.emplace(a->second, kv.first);
      } else {
        const std::string& prev = c->second;
        bool keep_prev = prev.size() < kv.first.size() || (prev.size() == kv.first.size() && prev < kv.first);
        if (keep_prev) {
          Log::Warning("%s is set with %s=%s, %s=%s will be ignored. Current value: %s=%s", a->second.c_str(),
                       prev.c_str(), params->at(prev).c_str(), kv.first.c_str(), kv.second.c_str(),
                       a->second.c_str(), params->at(prev).c_str());
        } else {
          Log::Warning("%s is set with %s=%s, will be overridden by %s=%s. Current value: %s=%s",
                       a->second.c_str(), prev.c_str(), params->at(prev).c_str(), kv.first.c_str(),
                       kv.second.c_str(), a->second.c_str(), kv.second.c_str());
          c->second = kv.first;
        }
      }
    } else if (parameter_set().count(kv.first) == 0) {
      Log::Warning("Unknown parameter: %s", kv.first.c_str());
    }
  }
  for (const auto& kv : chosen) {
    auto it = params->find(kv.first);
    if (it == params->end()) {
      std::string v = params->at(kv.second);
      params->emplace(kv.first, v);
      params->erase(kv.second);
    } else {
      Log::Warning("%s is set=%s, %s=%s will be ignored. Current value: %s=%s", kv.first.c_str(),
                   it->second.c_str(), kv.second.c_str(), params->at(kv.second).c_str(), kv.first.c_str(),
                   it->second.c_str());
    }
  }
}

bool Config::GetString(const std::unordered_map<std::string, std::string>& params, const std::string& name,
                       std::string* out) {
  auto it = params.find(name);
  if (it == params.end() || it->second.empty()) return false;
  *out = it->second;
  return true;
}

bool Config::GetInt(const std::unordered_map<std::string, std::string>& params, const std::string& name, int* out) {
  auto it = params.find(name);
  if (it == params.end() || it->second.empty()) return false;
  if (!common::AtoiAndCheck(it->second.c_str(), out)) {
    Log::Fatal("Parameter %s should be of type int, got \"%s\"", name.c_str(), it->second.c_str());
  }
  return true;
}

bool Config::GetDouble(const std::unordered_map<std::string, std::string>& params, const std::string& name,
                       double* out) {
  auto it = params.find(name);
  if (it == params.end() || it->second.empty()) return false;
  if (!common::AtofAndCheck(it->second.c_str(), out)) {
    Log::Fatal("Parameter %s should be of type double, got \"%s\"", name.c_str(), it->second.c_str());
  }
  return true;
}

bool Config::GetBool(const std::unordered_map<std::string, std::string>& params, const std::string& name,
                     bool* out) {
  auto it = params.find(name);
  if (it == params.end() || it->second.empty()) return false;
  std::string v = common::ToLower(it->second);
  if (v == "false" || v == "-") {
    *out = false;
  } else if (v == "true" || v == "+") {
    *out = true;
  } else {
    Log::Fatal("Parameter %s should be \"true\"/\"+\" or \"false\"/\"-\", got \"%s\"", name.c_str(),
               it->second.c_str());
  }
  return true;
}

std::string ParseObjectiveAlias(const std::string& t) {
  static const std::unordered_map<std::string, std::string> m = {
      {"regression", "regression"}, {"regression_l2", "regression"}, {"mean_squared_error", "regression"},
      {"mse", "regression"}, {"l2", "regression"}, {"l2_root", "regression"},
      {"root_mean_squared_error", "regression"}, {"rmse", "regression"},
      {"regression_l1", "regression_l1"}, {"mean_absolute_error", "regression_l1"}, {"l1", "regression_l1"},
      {"mae", "regression_l1"}, {"multiclass", "multiclass"}, {"softmax", "multiclass"},
      {"multiclassova", "multiclassova"}, {"multiclass_ova", "multiclassova"}, {"ova", "multiclassova"},
      {"ovr", "multiclassova"}, {"xentropy", "cross_entropy"}, {"cross_entropy", "cross_entropy"},
      {"xentlambda", "cross_entropy_lambda"}, {"cross_entropy_lambda", "cross_entropy_lambda"},
      {"mean_absolute_percentage_error", "mape"}, {"mape", "mape"}, {"rank_xendcg", "rank_xendcg"},
      {"xendcg", "rank_xendcg"}, {"xe_ndcg", "rank_xendcg"}, {"xe_ndcg_mart", "rank_xendcg"},
      {"xendcg_mart", "rank_xendcg"}, {"none", "custom"}, {"null", "custom"}, {"custom", "custom"},
      {"na", "custom"}};
  auto it = m.find(t);
  return it == m.end() ? t : it->second;
}

std::string ParseMetricAlias(const std::string& t) {
  static const std::unordered_map<std::string, std::string> m = {
      {"regression", "l2"}, {"regression_l2", "l2"}, {"l2", "l2"}, {"mean_squared_error", "l2"}, {"mse", "l2"},
      {"l2_root", "rmse"}, {"root_mean_squared_error", "rmse"}, {"rmse", "rmse"},
      {"regression_l1", "l1"}, {"l1", "l1"}, {"mean_absolute_error", "l1"}, {"mae", "l1"},
      {"binary_logloss", "binary_logloss"}, {"binary", "binary_logloss"},
      {"ndcg", "ndcg"}, {"lambdarank", "ndcg"}, {"rank_xendcg", "ndcg"}, {"xendcg", "ndcg"}, {"xe_ndcg", "ndcg"},
      {"xe_ndcg_mart", "ndcg"}, {"xendcg_mart", "ndcg"}, {"map", "map"}, {"mean_average_precision", "map"},
      {"multi_logloss", "multi_logloss"}, {"multiclass", "multi_logloss"}, {"softmax", "multi_logloss"},
      {"multiclassova", "multi_logloss"}, {"multiclass_ova", "multi_logloss"}, {"ova", "multi_logloss"},
      {"ovr", "multi_logloss"}, {"xentropy", "cross_entropy"}, {"cross_entropy", "cross_entropy"},
      {"xentlambda", "cross_entropy_lambda"}, {"cross_entropy_lambda", "cross_entropy_lambda"},
      {"kldiv", "kullback_leibler"}, {"kullback_leibler", "kullback_leibler"},
      {"mean_absolute_percentage_error", "mape"}, {"mape", "mape"}, {"auc_mu", "auc_mu"},
      {"none", "custom"}, {"null", "custom"}, {"custom", "custom"}, {"na", "custom"}};
  auto it = m.find(t);
  return it == m.end() ? t : it->second;
}

static void ParseMetricList(const std::string& value, std::vector<std::string>* out) {
  std::unordered_set<std::string> seen;
  out->clear();
  for (auto& m : common::Split(value.c_str(), ',')) {
    std::string t = ParseMetricAlias(common::Trim(m));
    if (seen.insert(t).second) out->push_back(t);
  }
}

void Config::GetAucMuWeights() {
  auc_mu_weights_matrix.assign(num_class, std::vector<double>(num_class, auc_mu_weights.empty() ? 1.0 : 0.0));
  if (auc_mu_weights.empty()) {
    for (int i = 0; i < num_class; ++i) auc_mu_weights_matrix[i][i] = 0;
    return;
  }
  if (auc_mu_weights.size() != static_cast<size_t>(num_class * num_class)) {
    Log::Fatal("auc_mu_weights must have %d elements, but found %d", num_class * num_class,
               static_cast<int>(auc_mu_weights.size()));
  }
  for (int i = 0; i < num_class; ++i) {
    for (int j = 0; j < num_class; ++j) {
      double w = auc_mu_weights[i * num_class + j];
      if (i == j) {
        auc_mu_weights_matrix[i][j] = 0;
      } else {
        if (std::fabs(w) < kZeroThreshold) {
          Log::Fatal("AUC-mu matrix must have non-zero values for non-diagonal entries. Found zero value in position %d of auc_mu_weights.",
                     i * num_class + j);
        }
        auc_mu_weights_matrix[i][j] = w;
      }
    }
  }
}

void Config::GetInteractionConstraints() {
  interaction_constraints_vector.clear();
  if (!interaction_constraints.empty()) {
    interaction_constraints_vector = common::StringToArrayOfArrays<int>(interaction_constraints, '[', ']', ',');
  }
}

void Config::Set(const std::unordered_map<std::string, std::string>& params) {
  for (auto& kv : params) explicit_keys.insert(kv.first);
  // derive the per-purpose seeds from `seed` (same derivation order as the reference)
  if (GetInt(params, "seed", &seed)) {
    Random r(seed);
    const int int_max = 32767;
    data_random_seed = r.NextShort(0, int_max);
    bagging_seed = r.NextShort(0, int_max);
    drop_seed = r.NextShort(0, int_max);
    feature_fraction_seed = r.NextShort(0, int_max);
    objective_seed = r.NextShort(0, int_max);
    extra_seed = r.NextShort(0, int_max);
  }
  std::string v;
  if (GetString(params, "task", &v)) {
    v = common::ToLower(v);
    if (v == "train" || v == "training") task = "train";
    else if (v == "predict" || v == "prediction" || v == "test") task = "predict";
    else if (v == "convert_model") task = "convert_model";
    else if (v == "refit" || v == "refit_tree") task = "refit";
    else if (v == "save_binary") task = "save_binary";
    else Log::Fatal("Unknown task type %s", v.c_str());
  }
  if (GetString(params, "boosting", &v)) {
    v = common::ToLower(v);
    if (v == "gbdt" || v == "gbrt") boosting = "gbdt";
    else if (v == "dart") boosting = "dart";
    else if (v == "goss") boosting = "goss";
    else if (v == "rf" || v == "random_forest") boosting = "rf";
    else Log::Fatal("Unknown boosting type %s", v.c_str());
  }
  {
    std::string mv;
    bool has_metric = GetString(params, "metric", &mv);
    if (has_metric) ParseMetricList(common::ToLower(mv), &metric);
    if (metric.empty() && mv.empty()) {
      std::string ov;
      if (GetString(params, "objective", &ov)) ParseMetricList(common::ToLower(ov), &metric);
    }
  }
  if (GetString(params, "objective", &v)) objective = ParseObjectiveAlias(common::ToLower(v));
  if (GetString(params, "device_type", &v)) {
    v = common::ToLower(v);
    // "cuda"/"hip"/"rocm" are accepted as synonyms of the device learner
    if (v == "cpu") device_type = "cpu";
    else if (v == "gpu" || v == "hip" || v == "rocm" || v == "cuda") device_type = "gpu";
    else Log::Fatal("Unknown device type %s", v.c_str());
  }
  if (GetString(params, "tree_learner", &v)) {
    v = common::ToLower(v);
    if (v == "serial") tree_learner = "serial";
    else if (v == "feature" || v == "feature_parallel") tree_learner = "feature";
    else if (v == "data" || v == "data_parallel") tree_learner = "data";
    else if (v == "voting" || v == "voting_parallel") tree_learner = "voting";
    else Log::Fatal("Unknown tree learner type %s", v.c_str());
  }
  GetMembersFromString(params);
  GetAucMuWeights();
  GetInteractionConstraints();
  std::sort(eval_at.begin(), eval_at.end());
  std::vector<std::string> kept;
  for (auto& f : valid) {
    if (f != data) kept.push_back(f);
    else is_provide_training_metric = true;
  }
  valid = kept;
  CheckParamConflict();
  if (verbosity == 1) Log::ResetLevel(LogLevel::Info);
  else if (verbosity == 0) Log::ResetLevel(LogLevel::Warning);
  else if (verbosity >= 2) Log::ResetLevel(LogLevel::Debug);
  else Log::ResetLevel(LogLevel::Fatal);
}

static bool IsMulticlassObjective(const std::string& o) { return o == "multiclass" || o == "multiclassova"; }

void Config::CheckParamConflict() {
  bool obj_multi = IsMulticlassObjective(objective) || (objective == "custom" && num_class > 1);
  if (obj_multi) {
    if (num_class <= 1) Log::Fatal("Number of classes should be specified and greater than 1 for multiclass training");
  } else if (task == "train" && num_class != 1) {
    Log::Fatal("Number of classes must be 1 for non-multiclass training");
  }
  for (auto& m : metric) {
    bool met_multi = IsMulticlassObjective(m) || m == "multi_logloss" || m == "multi_error" || m == "auc_mu" ||
                     (m == "custom" && num_class > 1);
    if (obj_multi != met_multi) Log::Fatal("Multiclass objective and metrics don't match");
  }
  is_parallel = num_machines > 1;
  if (!is_parallel) tree_learner = "serial";
  if (tree_learner == "serial") { is_parallel = false; num_machines = 1; }
  if (tree_learner == "serial" || tree_learner == "feature") {
    is_data_based_parallel = false;
  } else if (tree_learner == "data" || tree_learner == "voting") {
    is_data_based_parallel = true;
    if (histogram_pool_size >= 0 && tree_learner == "data") {
      Log::Warning("Histogram LRU queue was enabled (histogram_pool_size=%f).\nWill disable this to reduce communication costs",
                   histogram_pool_size);
      histogram_pool_size = -1;
    }
  }
  if (is_data_based_parallel && !forcedsplits_filename.empty()) {
    Log::Fatal("Don't support forcedsplits in %s tree learner", tree_learner.c_str());
  }
  if (max_depth > 0) {
    double full = std::pow(2.0, max_depth);
    if (full > num_leaves && num_leaves == kDefaultNumLeaves) {
      Log::Warning("Accuracy may be bad since you didn't set num_leaves and 2^max_depth > num_leaves");
    }
    if (full < num_leaves) num_leaves = static_cast<int>(full);
  }
  if (device_type == "gpu") {
    force_col_wise = true;
    force_row_wise = false;
  }
  if (path_smooth > kEpsilon && min_data_in_leaf < 2) {
    min_data_in_leaf = 2;
    Log::Warning("min_data_in_leaf has been increased to 2 because this is required when path smoothing is active.");
  }
  if (is_parallel && monotone_constraints_method == "intermediate") {
    Log::Warning("Cannot use \"intermediate\" monotone constraints in parallel learning, auto set to \"basic\" method.");
    monotone_constraints_method = "basic";
  }
  if (feature_fraction_bynode != 1.0 && monotone_constraints_method == "intermediate") {
    Log::Warning("Cannot use \"intermediate\" monotone constraints with feature fraction different from 1, auto set monotone constraints to \"basic\" method.");
    monotone_constraints_method = "basic";
  }
  if (max_depth > 0 && monotone_penalty >= max_depth) {
    Log::Warning("Monotone penalty greater than tree depth. Monotone features won't be used.");
  }
}

std::string Config::ToString() const {
  std::stringstream s;
  s << "[boosting: " << boosting << "]\n";
  s << "[objective: " << objective << "]\n";
  s << "[metric: " << common::Join(metric, ",") << "]\n";
  s << "[tree_learner: " << tree_learner << "]\n";
  s << "[device_type: " << device_type << "]\n";
  s << SaveMembersToString();
  return s.str();
}

}  // namespace lgbm_amd
