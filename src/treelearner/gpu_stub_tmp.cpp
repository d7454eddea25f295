#include "lgbm_amd/device_learner.h"
#include "lgbm_amd/log.h"
namespace lgbm_amd {
TreeLearner* CreateDeviceTreeLearner(const std::string&, const Config*) { Log::Fatal("device learner not built"); return nullptr; }
}
