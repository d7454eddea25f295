// Model IO (text v3 / JSON dump / C++ codegen), feature importance and prediction.
// Text format byte-compatible with reference src/boosting/gbdt_model_text.cpp:306-586;
// prediction and early-stopping semantics from gbdt_prediction.cpp:13-95 and
// prediction_early_stop.cpp:16-89.
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <sstream>

#include "lgbm_amd/boosting.h"
#include "lgbm_amd/common.h"
#include "lgbm_amd/log.h"

namespace lgbm_amd {

static const char* kModelVersion = "v3";

PredictionEarlyStopInstance CreatePredictionEarlyStopInstance(const std::string& type,
                                                              const PredictionEarlyStopConfig& cfg) {
  PredictionEarlyStopInstance es;
  if (type == "none") {
    es.callback = [](const double*, int) { return false; };
    es.round_period = std::numeric_limits<int>::max();
  } else if (type == "multiclass") {
    const double m = cfg.margin_threshold;
    es.callback = [m](const double* pred, int sz) {
      if (sz < 2) Log::Fatal("Multiclass early stopping needs predictions to be of length two or larger");
      std::vector<double> v(pred, pred + sz);
      std::partial_sort(v.begin(), v.begin() + 2, v.end(), std::greater<double>());
      return v[0] - v[1] > m;
    };
    es.round_period = cfg.round_period;
  } else if (type == "binary") {
    const double m = cfg.margin_threshold;
    es.callback = [m](const double* pred, int sz) {
      if (sz != 1) Log::Fatal("Binary early stopping needs predictions to be of length one");
      return 2.0 * std::fabs(pred[0]) > m;
    };
    es.round_period = cfg.round_period;
  } else {
    Log::Fatal("Unknown early stopping type: %s", type.c_str());
  }
  return es;
}

// ----------------------------------------------------------------------- text model
std::string GBDT::SaveModelToString(int start_iteration, int num_iteration, int importance_type) const {
  std::stringstream ss;
  ss << SubModelName() << '\n';
  ss << "version=" << kModelVersion << '\n';
  ss << "num_class=" << num_class_ << '\n';
  ss << "num_tree_per_iteration=" << num_tree_per_iteration_ << '\n';
  ss << "label_index=" << label_idx_ << '\n';
  ss << "max_feature_idx=" << max_feature_idx_ << '\n';
  if (objective_ != nullptr) ss << "objective=" << objective_->ToString() << '\n';
  if (average_output_) ss << "average_output" << '\n';
  ss << "feature_names=" << common::Join(feature_names_, " ") << '\n';
  if (!monotone_constraints_.empty()) ss << "monotone_constraints=" << common::Join(monotone_constraints_, " ") << '\n';
  ss << "feature_infos=" << common::Join(feature_infos_, " ") << '\n';
  int used = static_cast<int>(models_.size());
  const int total_iter = used / num_tree_per_iteration_;
  start_iteration = std::min(std::max(start_iteration, 0), total_iter);
  if (num_iteration > 0) used = std::min((start_iteration + num_iteration) * num_tree_per_iteration_, used);
  const int start_model = start_iteration * num_tree_per_iteration_;
  std::vector<std::string> strs(std::max(0, used - start_model));
  std::vector<size_t> sizes(strs.size());
#pragma omp parallel for schedule(static)
  for (int i = start_model; i < used; ++i) {
    const int j = i - start_model;
    strs[j] = "Tree=" + std::to_string(j) + '\n' + models_[i]->ToString() + '\n';
    sizes[j] = strs[j].size();
  }
  ss << "tree_sizes=" << common::Join(sizes, " ") << '\n';
  ss << '\n';
  for (auto& s : strs) ss << s;
  ss << "end of trees" << "\n";
  auto imp = FeatureImportance(num_iteration, importance_type);
  std::vector<std::pair<size_t, std::string>> pairs;
  for (size_t i = 0; i < imp.size(); ++i) {
    size_t v = static_cast<size_t>(imp[i]);
    if (v > 0) pairs.emplace_back(v, feature_names_[i]);
  }
  std::stable_sort(pairs.begin(), pairs.end(),
                   [](const std::pair<size_t, std::string>& a, const std::pair<size_t, std::string>& b) {
                     return a.first > b.first;
                   });
  ss << '\n' << "feature_importances:" << '\n';
  for (auto& p : pairs) ss << p.second << "=" << std::to_string(p.first) << '\n';
  if (config_ != nullptr) {
    ss << "\nparameters:" << '\n' << config_->ToString() << "\n" << "end of parameters" << '\n';
  } else if (!loaded_parameter_.empty()) {
    ss << "\nparameters:" << '\n' << loaded_parameter_ << "\n" << "end of parameters" << '\n';
  }
  return ss.str();
}

bool GBDT::SaveModelToFile(int start_iteration, int num_iteration, int importance_type, const char* filename) const {
  std::ofstream f(filename, std::ios::out | std::ios::binary);
  std::string s = SaveModelToString(start_iteration, num_iteration, importance_type);
  f.write(s.c_str(), static_cast<std::streamsize>(s.size()));
  return static_cast<bool>(f);
}

bool GBDT::LoadModelFromString(const char* buffer, size_t len) {
  models_.clear();
  const char* p = buffer;
  const char* end = buffer + len;
  std::unordered_map<std::string, std::string> kv;
  while (p < end) {
    size_t ll = common::GetLine(p);
    if (ll > 0) {
      std::string line(p, ll);
      if (common::StartsWith(line, "Tree=")) break;
      auto eq = line.find('=');
      if (eq == std::string::npos) {
        kv[line] = "";
      } else {
        std::string key = line.substr(0, eq);
        std::string val = line.substr(eq + 1);
        if (val.find('=') != std::string::npos && key != "feature_names" && key != "monotone_constraints") {
          Log::Fatal("Wrong line at model file: %s", line.substr(0, std::min<size_t>(128, line.size())).c_str());
        }
        kv[key] = val;
      }
    }
    p += ll;
    p = common::SkipNewLine(p);
  }
  if (!kv.count("num_class")) Log::Fatal("Model file doesn't specify the number of classes");
  common::Atoi(kv["num_class"].c_str(), &num_class_);
  num_tree_per_iteration_ = num_class_;
  if (kv.count("num_tree_per_iteration")) common::Atoi(kv["num_tree_per_iteration"].c_str(), &num_tree_per_iteration_);
  if (!kv.count("label_index")) Log::Fatal("Model file doesn't specify the label index");
  common::Atoi(kv["label_index"].c_str(), &label_idx_);
  if (!kv.count("max_feature_idx")) Log::Fatal("Model file doesn't specify max_feature_idx");
  common::Atoi(kv["max_feature_idx"].c_str(), &max_feature_idx_);
  if (kv.count("average_output")) average_output_ = true;
  if (!kv.count("feature_names")) Log::Fatal("Model file doesn't contain feature_names");
  feature_names_ = common::Split(kv["feature_names"].c_str(), ' ');
  if (feature_names_.size() != static_cast<size_t>(max_feature_idx_ + 1)) Log::Fatal("Wrong size of feature_names");
  if (kv.count("monotone_constraints")) {
    auto v = common::StringToArray<int>(kv["monotone_constraints"], ' ');
    monotone_constraints_.assign(v.begin(), v.end());
    if (monotone_constraints_.size() != static_cast<size_t>(max_feature_idx_ + 1)) {
      Log::Fatal("Wrong size of monotone_constraints");
    }
  }
  if (!kv.count("feature_infos")) Log::Fatal("Model file doesn't contain feature_infos");
  feature_infos_ = common::Split(kv["feature_infos"].c_str(), ' ');
  if (feature_infos_.size() != static_cast<size_t>(max_feature_idx_ + 1)) Log::Fatal("Wrong size of feature_infos");
  if (kv.count("objective")) {
    loaded_objective_.reset(ObjectiveFunction::CreateObjectiveFunction(kv["objective"]));
    objective_ = loaded_objective_.get();
  }
  if (!kv.count("tree_sizes")) {
    while (p < end) {
      size_t ll = common::GetLine(p);
      if (ll > 0) {
        std::string line(p, ll);
        if (!common::StartsWith(line, "Tree=")) break;
        p += ll;
        p = common::SkipNewLine(p);
        size_t used = 0;
        models_.emplace_back(new Tree(p, &used));
        p += used;
      }
      p = common::SkipNewLine(p);
    }
  } else {
    auto sizes = common::StringToArray<size_t>(kv["tree_sizes"], ' ');
    std::vector<size_t> bounds(sizes.size() + 1, 0);
    for (size_t i = 0; i < sizes.size(); ++i) bounds[i + 1] = bounds[i] + sizes[i];
    models_.resize(sizes.size());
    common::OmpErrors errors;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < static_cast<int>(sizes.size()); ++i) {
      errors.Run([&] {
        const char* cp = p + bounds[i];
        size_t ll = common::GetLine(cp);
        std::string line(cp, ll);
        if (!common::StartsWith(line, "Tree=")) {
          Log::Fatal("Model format error, expect a tree here. met %s", line.c_str());
        }
        cp = common::SkipNewLine(cp + ll);
        size_t used = 0;
        models_[i].reset(new Tree(cp, &used));
      });
    }
    errors.Check();
    p += bounds.back();
  }
  num_iteration_for_pred_ = static_cast<int>(models_.size()) / num_tree_per_iteration_;
  num_init_iteration_ = num_iteration_for_pred_;
  iter_ = 0;
  bool in_params = false;
  std::stringstream ps;
  while (p < end) {
    size_t ll = common::GetLine(p);
    if (ll > 0) {
      std::string line(p, ll);
      if (line == "parameters:") {
        in_params = true;
      } else if (line == "end of parameters") {
        break;
      } else if (in_params) {
        ps << line << "\n";
      }
    }
    p += ll;
    p = common::SkipNewLine(p);
  }
  if (!ps.str().empty()) loaded_parameter_ = ps.str();
  return true;
}

std::vector<double> GBDT::FeatureImportance(int num_iteration, int importance_type) const {
  int used = static_cast<int>(models_.size());
  if (num_iteration > 0) used = std::min(num_iteration * num_tree_per_iteration_, used);
  std::vector<double> imp(max_feature_idx_ + 1, 0.0);
  if (importance_type != 0 && importance_type != 1) Log::Fatal("Unknown importance type: only support split=0 and gain=1");
  for (int it = 0; it < used; ++it) {
    const Tree* t = models_[it].get();
    for (int s = 0; s < t->num_leaves() - 1; ++s) {
      if (t->split_gain(s) > 0) imp[t->split_feature(s)] += importance_type == 0 ? 1.0 : t->split_gain(s);
    }
  }
  return imp;
}

std::string GBDT::DumpModel(int start_iteration, int num_iteration, int importance_type) const {
  std::stringstream s;
  s << "{";
  s << "\"name\":\"" << SubModelName() << "\"," << '\n';
  s << "\"version\":\"" << kModelVersion << "\"," << '\n';
  s << "\"num_class\":" << num_class_ << "," << '\n';
  s << "\"num_tree_per_iteration\":" << num_tree_per_iteration_ << "," << '\n';
  s << "\"label_index\":" << label_idx_ << "," << '\n';
  s << "\"max_feature_idx\":" << max_feature_idx_ << "," << '\n';
  if (objective_ != nullptr) s << "\"objective\":\"" << objective_->ToString() << "\",\n";
  s << "\"average_output\":" << (average_output_ ? "true" : "false") << ",\n";
  s << "\"feature_names\":[\"" << common::Join(feature_names_, "\",\"") << "\"]," << '\n';
  s << "\"monotone_constraints\":[" << common::Join(monotone_constraints_, ",") << "]," << '\n';
  s << "\"feature_infos\":" << "{";
  bool first = true;
  for (size_t i = 0; i < feature_infos_.size(); ++i) {
    std::stringstream js;
    const std::string& fi = feature_infos_[i];
    if (fi == "none") continue;
    if (fi[0] == '[') {
      auto inner = fi.substr(1, fi.size() - 2);
      auto parts = common::Split(inner.c_str(), ':');
      double mn = 0, mx = 0;
      common::Atof(parts[0].c_str(), &mn);
      common::Atof(parts[1].c_str(), &mx);
      js << std::setprecision(std::numeric_limits<double>::digits10 + 2);
      js << "{\"min_value\":" << common::AvoidInf(mn) << ",\"max_value\":" << common::AvoidInf(mx) << ",\"values\":[]}";
    } else {
      auto vals = common::StringToArray<int>(fi, ':');
      js << "{\"min_value\":" << *std::min_element(vals.begin(), vals.end())
         << ",\"max_value\":" << *std::max_element(vals.begin(), vals.end()) << ",\"values\":[" << common::Join(vals, ",")
         << "]}";
    }
    if (!first) s << ",";
    s << "\"" << feature_names_[i] << "\":" << js.str();
    first = false;
  }
  s << "}," << '\n';
  s << "\"tree_info\":[";
  int used = static_cast<int>(models_.size());
  const int total_iter = used / num_tree_per_iteration_;
  start_iteration = std::min(std::max(start_iteration, 0), total_iter);
  if (num_iteration > 0) used = std::min((start_iteration + num_iteration) * num_tree_per_iteration_, used);
  const int sm = start_iteration * num_tree_per_iteration_;
  for (int i = sm; i < used; ++i) {
    if (i > sm) s << ",";
    s << "{\"tree_index\":" << i << "," << models_[i]->ToJSON() << "}";
  }
  s << "]," << '\n';
  auto imp = FeatureImportance(num_iteration, importance_type);
  std::vector<std::pair<size_t, std::string>> pairs;
  for (size_t i = 0; i < imp.size(); ++i) {
    size_t v = static_cast<size_t>(imp[i]);
    if (v > 0) pairs.emplace_back(v, feature_names_[i]);
  }
  s << '\n' << "\"feature_importances\":" << "{";
  for (size_t i = 0; i < pairs.size(); ++i) {
    if (i) s << ",";
    s << "\"" << pairs[i].second << "\":" << std::to_string(pairs[i].first);
  }
  s << "}" << '\n' << "}" << '\n';
  return s.str();
}

// Standalone C++ translation of the model: one function per tree plus C-ABI entry points
// `lgbm_predict_raw(const double* x, double* out)` / `lgbm_predict_leaf(...)`.
std::string GBDT::ModelToIfElse(int num_iteration) const {
  std::stringstream s;
  s << "// generated by lightgbmv1_amd convert_model\n";
  s << "#include <cmath>\n#include <cstdint>\n#include <cstring>\n#include <unordered_map>\n#include <vector>\n";
  s << "namespace {\nstruct Tree { static bool IsZero(double v) { return v >= -1e-35f && v <= 1e-35f; } };\n";
  int used = static_cast<int>(models_.size());
  if (num_iteration > 0) used = std::min(num_iteration * num_tree_per_iteration_, used);
  for (int i = 0; i < used; ++i) s << models_[i]->ToIfElse(i, false) << '\n';
  for (int i = 0; i < used; ++i) s << models_[i]->ToIfElse(i, true) << '\n';
  s << "double (*PredictTreePtr[])(const double*) = { ";
  for (int i = 0; i < used; ++i) s << (i ? " , " : "") << "PredictTree" << i;
  s << " };\n";
  s << "double (*PredictTreeLeafPtr[])(const double*) = { ";
  for (int i = 0; i < used; ++i) s << (i ? " , " : "") << "PredictTree" << i << "Leaf";
  s << " };\n}  // namespace\n";
  s << "extern \"C\" int lgbm_num_tree_per_iteration() { return " << num_tree_per_iteration_ << "; }\n";
  s << "extern \"C\" int lgbm_num_trees() { return " << used << "; }\n";
  s << "extern \"C\" void lgbm_predict_raw(const double* x, double* out) {\n";
  s << "  const int K = " << num_tree_per_iteration_ << ";\n";
  s << "  std::memset(out, 0, sizeof(double) * K);\n";
  s << "  for (int i = 0; i < " << used << "; ++i) out[i % K] += PredictTreePtr[i](x);\n";
  if (average_output_) s << "  for (int k = 0; k < K; ++k) out[k] /= " << std::max(1, used / num_tree_per_iteration_) << ";\n";
  s << "}\n";
  s << "extern \"C\" void lgbm_predict_leaf(const double* x, double* out) {\n";
  s << "  for (int i = 0; i < " << used << "; ++i) out[i] = PredictTreeLeafPtr[i](x);\n}\n";
  return s.str();
}

bool GBDT::SaveModelToIfElse(int num_iteration, const char* filename) const {
  std::ofstream f(filename);
  f << ModelToIfElse(num_iteration);
  return static_cast<bool>(f);
}

double GBDT::GetUpperBoundValue() const {
  double v = 0;
  for (auto& t : models_) v += t->GetUpperBoundValue();
  return v;
}

double GBDT::GetLowerBoundValue() const {
  double v = 0;
  for (auto& t : models_) v += t->GetLowerBoundValue();
  return v;
}

double GBDT::GetLeafValue(int tree_idx, int leaf_idx) const {
  LGBM_CHECK(tree_idx >= 0 && static_cast<size_t>(tree_idx) < models_.size());
  LGBM_CHECK(leaf_idx >= 0 && leaf_idx < models_[tree_idx]->num_leaves());
  return models_[tree_idx]->LeafOutput(leaf_idx);
}

void GBDT::SetLeafValue(int tree_idx, int leaf_idx, double val) {
  LGBM_CHECK(tree_idx >= 0 && static_cast<size_t>(tree_idx) < models_.size());
  LGBM_CHECK(leaf_idx >= 0 && leaf_idx < models_[tree_idx]->num_leaves());
  models_[tree_idx]->SetLeafOutput(leaf_idx, val);
}

// ----------------------------------------------------------------------- prediction
bool GBDT::PredictRangeIs(int start_iteration, int num_iteration) const {
  int num = static_cast<int>(models_.size()) / num_tree_per_iteration_;
  start_iteration = std::min(std::max(start_iteration, 0), num);
  num = num_iteration > 0 ? std::min(num_iteration, num - start_iteration) : num - start_iteration;
  return start_iteration == start_iteration_for_pred_ && num == num_iteration_for_pred_;
}

void GBDT::InitPredict(int start_iteration, int num_iteration, bool is_pred_contrib) {
  num_iteration_for_pred_ = static_cast<int>(models_.size()) / num_tree_per_iteration_;
  start_iteration = std::min(std::max(start_iteration, 0), num_iteration_for_pred_);
  if (num_iteration > 0) {
    num_iteration_for_pred_ = std::min(num_iteration, num_iteration_for_pred_ - start_iteration);
  } else {
    num_iteration_for_pred_ = num_iteration_for_pred_ - start_iteration;
  }
  start_iteration_for_pred_ = start_iteration;
  if (is_pred_contrib) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < static_cast<int>(models_.size()); ++i) models_[i]->RecomputeMaxDepth();
  }
}

int GBDT::NumPredictOneRow(int start_iteration, int num_iteration, bool is_pred_leaf, bool is_pred_contrib) const {
  int n = num_class_;
  if (is_pred_leaf) {
    const int mx = GetCurrentIteration();
    start_iteration = std::min(std::max(start_iteration, 0), mx);
    n *= num_iteration > 0 ? std::min(mx - start_iteration, num_iteration) : (mx - start_iteration);
  } else if (is_pred_contrib) {
    n = num_tree_per_iteration_ * (max_feature_idx_ + 2);
  }
  return n;
}

void GBDT::PredictRaw(const double* x, double* out, const PredictionEarlyStopInstance* es) const {
  int counter = 0;
  std::memset(out, 0, sizeof(double) * num_tree_per_iteration_);
  const int end = start_iteration_for_pred_ + num_iteration_for_pred_;
  for (int i = start_iteration_for_pred_; i < end; ++i) {
    for (int k = 0; k < num_tree_per_iteration_; ++k) out[k] += models_[i * num_tree_per_iteration_ + k]->Predict(x);
    if (es != nullptr && ++counter == es->round_period) {
      if (es->callback(out, num_tree_per_iteration_)) return;
      counter = 0;
    }
  }
}

void GBDT::PredictRawByMap(const std::unordered_map<int, double>& x, double* out,
                           const PredictionEarlyStopInstance* es) const {
  int counter = 0;
  std::memset(out, 0, sizeof(double) * num_tree_per_iteration_);
  const int end = start_iteration_for_pred_ + num_iteration_for_pred_;
  for (int i = start_iteration_for_pred_; i < end; ++i) {
    for (int k = 0; k < num_tree_per_iteration_; ++k) out[k] += models_[i * num_tree_per_iteration_ + k]->PredictByMap(x);
    if (es != nullptr && ++counter == es->round_period) {
      if (es->callback(out, num_tree_per_iteration_)) return;
      counter = 0;
    }
  }
}

void GBDT::Predict(const double* x, double* out, const PredictionEarlyStopInstance* es) const {
  PredictRaw(x, out, es);
  if (average_output_) {
    for (int k = 0; k < num_tree_per_iteration_; ++k) out[k] /= num_iteration_for_pred_;
  }
  if (objective_ != nullptr) objective_->ConvertOutput(out, out);
}

void GBDT::PredictByMap(const std::unordered_map<int, double>& x, double* out,
                        const PredictionEarlyStopInstance* es) const {
  PredictRawByMap(x, out, es);
  if (average_output_) {
    for (int k = 0; k < num_tree_per_iteration_; ++k) out[k] /= num_iteration_for_pred_;
  }
  if (objective_ != nullptr) objective_->ConvertOutput(out, out);
}

void GBDT::PredictLeafIndex(const double* x, double* out) const {
  const int st = start_iteration_for_pred_ * num_tree_per_iteration_;
  const int n = num_iteration_for_pred_ * num_tree_per_iteration_;
  for (int i = 0; i < n; ++i) out[i] = models_[st + i]->PredictLeafIndex(x);
}

void GBDT::PredictLeafIndexByMap(const std::unordered_map<int, double>& x, double* out) const {
  const int st = start_iteration_for_pred_ * num_tree_per_iteration_;
  const int n = num_iteration_for_pred_ * num_tree_per_iteration_;
  for (int i = 0; i < n; ++i) out[i] = models_[st + i]->PredictLeafIndexByMap(x);
}

void GBDT::PredictContrib(const double* x, double* out) const {
  const int nf = max_feature_idx_ + 1;
  std::memset(out, 0, sizeof(double) * num_tree_per_iteration_ * (nf + 1));
  const int end = start_iteration_for_pred_ + num_iteration_for_pred_;
  for (int i = start_iteration_for_pred_; i < end; ++i) {
    for (int k = 0; k < num_tree_per_iteration_; ++k) {
      models_[i * num_tree_per_iteration_ + k]->PredictContrib(x, nf, out + k * (nf + 1));
    }
  }
}

void GBDT::PredictContribByMap(const std::unordered_map<int, double>& x,
                               std::vector<std::unordered_map<int, double>>* out) const {
  const int nf = max_feature_idx_ + 1;
  const int end = start_iteration_for_pred_ + num_iteration_for_pred_;
  for (int i = start_iteration_for_pred_; i < end; ++i) {
    for (int k = 0; k < num_tree_per_iteration_; ++k) {
      models_[i * num_tree_per_iteration_ + k]->PredictContribByMap(x, nf, &(*out)[k]);
    }
  }
}

}  // namespace lgbm_amd
