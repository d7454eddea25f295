// Configuration object.  Members are generated from tools/param_spec.py (the single
// parameter spec, reference equivalent: include/LightGBM/config.h:84-988 +
// helpers/parameter_generator.py).  Every reference parameter name and alias is
// accepted; key/alias priority and the conflict checks mirror
// src/io/config.cpp:15-349 of the reference.
#pragma once

#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "lgbm_amd/meta.h"

namespace lgbm_amd {

struct Config {
 public:
#include "lgbm_amd/config_fields.inc"

  // derived members
  bool is_parallel = false;
  bool is_data_based_parallel = false;
  std::vector<std::vector<double>> auc_mu_weights_matrix;
  std::vector<std::vector<int>> interaction_constraints_vector;
  // which keys were set explicitly by the user (after alias resolution)
  std::unordered_set<std::string> explicit_keys;

  Config() = default;
  explicit Config(const std::unordered_map<std::string, std::string>& params) { Set(params); }

  void Set(const std::unordered_map<std::string, std::string>& params);
  std::string ToString() const;

  static std::unordered_map<std::string, std::string> Str2Map(const char* parameters);
  static void KV2Map(std::unordered_map<std::string, std::string>* params, const char* kv);
  static void KeyAliasTransform(std::unordered_map<std::string, std::string>* params);
  static const std::unordered_map<std::string, std::string>& alias_table();
  static const std::unordered_set<std::string>& parameter_set();

  static bool GetString(const std::unordered_map<std::string, std::string>& params, const std::string& name,
                        std::string* out);
  static bool GetInt(const std::unordered_map<std::string, std::string>& params, const std::string& name, int* out);
  static bool GetDouble(const std::unordered_map<std::string, std::string>& params, const std::string& name,
                        double* out);
  static bool GetBool(const std::unordered_map<std::string, std::string>& params, const std::string& name,
                      bool* out);

  void GetMembersFromString(const std::unordered_map<std::string, std::string>& params);
  std::string SaveMembersToString() const;
  void CheckParamConflict();

 private:
  void GetAucMuWeights();
  void GetInteractionConstraints();
};

std::string ParseObjectiveAlias(const std::string& type);
std::string ParseMetricAlias(const std::string& type);

}  // namespace lgbm_amd
