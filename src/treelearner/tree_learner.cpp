// Tree learner factory (reference src/treelearner/tree_learner.cpp:15-55).
// device_type=cpu  -> host learners (serial / feature / data / voting parallel over Network)
// device_type=gpu  -> the MI355X device learner; its data-parallel mode reduces histograms
//                     with RCCL (or the host Network when RCCL is not initialised).
#include "lgbm_amd/tree_learner.h"

#include "lgbm_amd/device_learner.h"
#include "lgbm_amd/log.h"
#include "parallel_tree_learner.h"
#include "serial_tree_learner.h"

namespace lgbm_amd {

TreeLearner* TreeLearner::CreateTreeLearner(const std::string& learner_type, const std::string& device_type,
                                            const Config* config) {
  if (device_type == "cpu") {
    if (learner_type == "serial") return new SerialTreeLearner(config);
    if (learner_type == "feature") return new FeatureParallelTreeLearner(config);
    if (learner_type == "data") return new DataParallelTreeLearner(config);
    if (learner_type == "voting") return new VotingParallelTreeLearner<SerialTreeLearner>(config);
  } else if (device_type == "gpu") {
    return CreateDeviceTreeLearner(learner_type, config);
  }
  Log::Fatal("Unknown tree learner type %s for device %s", learner_type.c_str(), device_type.c_str());
  return nullptr;
}

}  // namespace lgbm_amd
