// Command-line application: `lightgbm config=train.conf key=value ...`
// Tasks train / predict / convert_model / refit / save_binary with the reference's
// parameter precedence (command line over config file) and outputs
// (reference src/application/application.cpp:28-270, src/main.cpp).
#include <omp.h>

#include <chrono>
#include <cstdio>
#include <fstream>
#include <memory>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "lgbm_amd/boosting.h"
#include "lgbm_amd/common.h"
#include "lgbm_amd/config.h"
#include "lgbm_amd/dataset.h"
#include "lgbm_amd/dataset_loader.h"
#include "lgbm_amd/log.h"
#include "lgbm_amd/metric.h"
#include "lgbm_amd/network.h"
#include "lgbm_amd/objective.h"
#include "lgbm_amd/predictor.h"

using namespace lgbm_amd;

namespace {

class Application {
 public:
  Application(int argc, char** argv) {
    std::unordered_map<std::string, std::string> params;
    for (int i = 1; i < argc; ++i) Config::KV2Map(&params, argv[i]);
    Config::KeyAliasTransform(&params);
    if (params.count("config")) {
      std::ifstream f(params["config"]);
      if (!f) {
        Log::Warning("Config file %s doesn't exist, will ignore", params["config"].c_str());
      } else {
        std::string line;
        while (std::getline(f, line)) {
          auto pos = line.find_first_of('#');
          if (pos != std::string::npos) line.erase(pos);
          line = common::Trim(line);
          if (!line.empty()) Config::KV2Map(&params, line.c_str());
        }
      }
    }
    Config::KeyAliasTransform(&params);
    config_.Set(params);
    if (config_.num_threads > 0) omp_set_num_threads(config_.num_threads);
    if (config_.data.empty() && config_.task != "convert_model") Log::Fatal("No training/prediction data, application quit");
  }

  ~Application() {
    if (config_.is_parallel) Network::Dispose();
  }

  void Run() {
    const std::string& t = config_.task;
    if (t == "train") {
      InitTrain();
      Train();
    } else if (t == "predict") {
      Predict();
    } else if (t == "convert_model") {
      ConvertModel();
    } else if (t == "refit") {
      Refit();
    } else if (t == "save_binary") {
      DatasetLoader loader(config_, 1, 0);
      auto ds = loader.LoadFromFile(config_.data);
      ds->SaveBinaryFile(config_.data + ".bin");
    } else {
      Log::Fatal("Unknown task type %s", t.c_str());
    }
  }

 private:
  // raw scores of an existing model for every row of a text file (continued training)
  std::vector<double> PredictInitScore(const std::string& file, data_size_t expected_rows) {
    std::string tmp = file + ".init_score.tmp";
    Predictor pred(boosting_.get(), 0, -1, true, false, false, false, -1, -1);
    pred.PredictFile(file, tmp, config_.header, true);
    std::ifstream in(tmp);
    const int k = boosting_->NumModelPerIteration();
    std::vector<std::vector<double>> rows;
    std::string line;
    while (std::getline(in, line)) {
      if (line.empty()) continue;
      std::vector<double> v;
      for (auto& tok : common::Split(line.c_str(), '\t')) {
        double d = 0;
        common::Atof(tok.c_str(), &d);
        v.push_back(d);
      }
      rows.push_back(v);
    }
    in.close();
    std::remove(tmp.c_str());
    if (static_cast<data_size_t>(rows.size()) != expected_rows) {
      Log::Warning("Could not map continued-training predictions onto the loaded rows; ignoring input_model scores");
      return {};
    }
    std::vector<double> out(static_cast<size_t>(expected_rows) * k);
    for (data_size_t i = 0; i < expected_rows; ++i) {
      for (int j = 0; j < k; ++j) out[static_cast<size_t>(j) * expected_rows + i] = rows[i][j];
    }
    return out;
  }

  void InitTrain() {
    if (config_.is_parallel) {
      Network::Init(config_);
      Log::Info("Finished initializing network");
      config_.feature_fraction_seed = Network::GlobalSyncUpByMin(config_.feature_fraction_seed);
      config_.feature_fraction = Network::GlobalSyncUpByMin(config_.feature_fraction);
      config_.drop_seed = Network::GlobalSyncUpByMin(config_.drop_seed);
    }
    boosting_.reset(GBDT::CreateBoosting(config_.boosting, config_.input_model.c_str()));
    objective_.reset(ObjectiveFunction::CreateObjectiveFunction(config_.objective, config_));
    auto start = std::chrono::steady_clock::now();
    if (config_.is_data_based_parallel) config_.data_random_seed = Network::GlobalSyncUpByMin(config_.data_random_seed);
    const int nm = config_.is_data_based_parallel ? Network::num_machines() : 1;
    const int rk = config_.is_data_based_parallel ? Network::rank() : 0;
    DatasetLoader loader(config_, nm, rk);
    train_data_ = loader.LoadFromFile(config_.data);
    const bool continued = boosting_->NumberOfTotalModel() > 0;
    if (continued) {
      auto init = PredictInitScore(config_.data, train_data_->num_data());
      if (!init.empty()) train_data_->metadata().SetInitScore(init.data(), static_cast<int64_t>(init.size()));
    }
    if (config_.save_binary) train_data_->SaveBinaryFile(config_.data + ".bin");
    if (config_.is_provide_training_metric) {
      for (auto& m : config_.metric) {
        std::unique_ptr<Metric> mm(Metric::CreateMetric(m, config_));
        if (mm == nullptr) continue;
        mm->Init(train_data_->metadata(), train_data_->num_data());
        train_metric_.push_back(std::move(mm));
      }
    }
    if (!config_.metric.empty()) {
      for (auto& v : config_.valid) {
        valid_datas_.push_back(loader.LoadFromFileAlignWithOtherDataset(v, *train_data_));
        if (continued) {
          auto init = PredictInitScore(v, valid_datas_.back()->num_data());
          if (!init.empty()) valid_datas_.back()->metadata().SetInitScore(init.data(), static_cast<int64_t>(init.size()));
        }
        if (config_.save_binary) valid_datas_.back()->SaveBinaryFile(v + ".bin");
        valid_metrics_.emplace_back();
        for (auto& m : config_.metric) {
          std::unique_ptr<Metric> mm(Metric::CreateMetric(m, config_));
          if (mm == nullptr) continue;
          mm->Init(valid_datas_.back()->metadata(), valid_datas_.back()->num_data());
          valid_metrics_.back().push_back(std::move(mm));
        }
      }
    }
    Log::Info("Finished loading data in %f seconds",
              std::chrono::duration<double>(std::chrono::steady_clock::now() - start).count());
    if (objective_ != nullptr) objective_->Init(train_data_->metadata(), train_data_->num_data());
    std::vector<const Metric*> tm;
    for (auto& m : train_metric_) tm.push_back(m.get());
    boosting_->Init(&config_, train_data_.get(), objective_.get(), tm);
    for (size_t i = 0; i < valid_datas_.size(); ++i) {
      std::vector<const Metric*> vm;
      for (auto& m : valid_metrics_[i]) vm.push_back(m.get());
      boosting_->AddValidDataset(valid_datas_[i].get(), vm);
      Log::Debug("Number of data points in validation set #%zu: %d", i + 1, valid_datas_[i]->num_data());
    }
    Log::Info("Finished initializing training");
  }

  void Train() {
    Log::Info("Started training...");
    boosting_->Train(config_.snapshot_freq, config_.output_model);
    boosting_->SaveModelToFile(0, -1, config_.saved_feature_importance_type, config_.output_model.c_str());
    if (config_.convert_model_language == "cpp") boosting_->SaveModelToIfElse(-1, config_.convert_model.c_str());
    Log::Info("Finished training");
  }

  void Predict() {
    boosting_.reset(GBDT::CreateBoosting("gbdt", config_.input_model.c_str()));
    Predictor pred(boosting_.get(), config_.start_iteration_predict, config_.num_iteration_predict,
                   config_.predict_raw_score, config_.predict_leaf_index, config_.predict_contrib,
                   config_.pred_early_stop, config_.pred_early_stop_freq, config_.pred_early_stop_margin);
    pred.PredictFile(config_.data, config_.output_result, config_.header, config_.predict_disable_shape_check);
    Log::Info("Finished prediction");
  }

  void ConvertModel() {
    boosting_.reset(GBDT::CreateBoosting(config_.boosting, config_.input_model.c_str()));
    boosting_->SaveModelToIfElse(-1, config_.convert_model.c_str());
  }

  void Refit() {
    boosting_.reset(GBDT::CreateBoosting(config_.boosting, config_.input_model.c_str()));
    std::string leaf_file = config_.output_result + ".leaf.tmp";
    {
      Predictor pred(boosting_.get(), 0, -1, false, true, false, false, 1, 1e10);
      pred.PredictFile(config_.data, leaf_file, config_.header, config_.predict_disable_shape_check);
    }
    std::vector<std::vector<int>> leaf_preds;
    {
      std::ifstream in(leaf_file);
      std::string line;
      while (std::getline(in, line)) {
        if (line.empty()) continue;
        std::vector<int> v;
        for (auto& tok : common::Split(line.c_str(), '\t')) {
          double d = 0;
          common::Atof(tok.c_str(), &d);
          v.push_back(static_cast<int>(d));
        }
        leaf_preds.push_back(v);
      }
    }
    std::remove(leaf_file.c_str());
    DatasetLoader loader(config_, 1, 0);
    train_data_ = loader.LoadFromFile(config_.data);
    objective_.reset(ObjectiveFunction::CreateObjectiveFunction(config_.objective, config_));
    objective_->Init(train_data_->metadata(), train_data_->num_data());
    boosting_->Init(&config_, train_data_.get(), objective_.get(), {});
    boosting_->RefitTree(leaf_preds);
    boosting_->SaveModelToFile(0, -1, config_.saved_feature_importance_type, config_.output_model.c_str());
    Log::Info("Finished RefitTree");
  }

  Config config_;
  std::unique_ptr<GBDT> boosting_;
  std::unique_ptr<ObjectiveFunction> objective_;
  std::unique_ptr<Dataset> train_data_;
  std::vector<std::unique_ptr<Dataset>> valid_datas_;
  std::vector<std::unique_ptr<Metric>> train_metric_;
  std::vector<std::vector<std::unique_ptr<Metric>>> valid_metrics_;
};

}  // namespace

int main(int argc, char** argv) {
  bool success = false;
  try {
    Application app(argc, argv);
    app.Run();
    success = true;
  } catch (std::exception& ex) {
    fprintf(stderr, "Met Exceptions:\n%s\n", ex.what());
  } catch (...) {
    fprintf(stderr, "Unknown Exceptions\n");
  }
  if (!success) {
    Network::Dispose();
    MpiAbortIfStarted();
    return 1;
  }
  MpiFinalizeIfStarted();
  return 0;
}
