// Stand-alone device ops over caller-owned device buffers (torch tensors on cuda), exposed
// for lightgbmv1_amd.ops: the same HIP kernels the device learner runs each iteration --
// point-wise objective gradients (src/device/objective_kernels.hip), validation metrics
// (src/device/metric_kernels.hip) and the bagging / GOSS row sampler
// (src/device/sample_kernels.hip) -- callable one at a time so that their numerics can be
// checked against plain PyTorch references (tests/test_ops.py).
//
// Objectives and metrics are created from a parameter string exactly as training creates
// them (reference objective_function.cpp:16-56, metric.cpp:16-63), so the kernels see the
// same DeviceGradSpec / DeviceMetricSpec.  Every op runs on the null stream and returns
// after it finished (the caller synchronises its own stream before the call).
#include <hip/hip_runtime_api.h>

#include <cmath>
#include <memory>
#include <string>
#include <vector>

#include "../device/kernels.h"
#include "lgbm_amd/c_api.h"
#include "lgbm_amd/config.h"
#include "lgbm_amd/dataset.h"
#include "lgbm_amd/log.h"
#include "lgbm_amd/tuning.h"
#include "lgbm_amd/metric.h"
#include "lgbm_amd/objective.h"

using namespace lgbm_amd;

namespace {

thread_local std::string g_op_error = "Everything is fine";

#define OPCHECK(x)                                                                                  \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) Log::Fatal("HIP error %s at %s:%d: %s", #x, __FILE__, __LINE__, hipGetErrorString(e_)); \
  } while (0)

template <typename F>
int Guard(F&& f) {
  try {
    f();
    return 0;
  } catch (std::exception& e) {
    g_op_error = e.what();
  } catch (...) {
    g_op_error = "unknown exception";
  }
  return -1;
}

// device scratch freed at scope exit
struct Scratch {
  std::vector<void*> ptrs;
  ~Scratch() {
    for (void* p : ptrs) (void)hipFree(p);
  }
  template <typename T>
  T* Upload(const T* host, size_t n) {
    if (host == nullptr) return nullptr;
    T* p = Alloc<T>(n);
    OPCHECK(hipMemcpy(p, host, n * sizeof(T), hipMemcpyHostToDevice));
    return p;
  }
  template <typename T>
  T* Alloc(size_t n) {
    void* p = nullptr;
    OPCHECK(hipMalloc(&p, std::max<size_t>(1, n) * sizeof(T)));
    ptrs.push_back(p);
    return static_cast<T*>(p);
  }
};

Config ParseConfig(const char* params) {
  Config c;
  c.Set(Config::Str2Map(params ? params : ""));
  return c;
}

void FillMetadata(Metadata* md, const float* label, const float* weight, int32_t n) {
  md->Init(n, weight != nullptr, false);
  md->SetLabel(label, n);
  if (weight != nullptr) md->SetWeights(weight, n);
}

}  // namespace

LIGHTGBM_C_EXPORT const char* LGBMAMD_OpLastError() { return g_op_error.c_str(); }

// gradients / hessians of a point-wise objective: score [num_class][n] (device, float64),
// grad / hess [num_class][n] (device, float32); label / weight are host arrays (the objective's
// Init reads them: label checks, MAPE weights, class counts)
LIGHTGBM_C_EXPORT int LGBMAMD_OpGradients(const char* params, const float* label, const float* weight, int32_t n,
                                          const double* d_score, float* d_grad, float* d_hess) {
  return Guard([&] {
    Config c = ParseConfig(params);
    std::unique_ptr<ObjectiveFunction> obj(ObjectiveFunction::CreateObjectiveFunction(c.objective, c));
    if (!obj) Log::Fatal("op gradients: no objective '%s'", c.objective.c_str());
    Metadata md;
    FillMetadata(&md, label, weight, n);
    obj->Init(md, n);
    const DeviceGradSpec spec = obj->DeviceSpec();
    if (spec.kind == DeviceGradKind::None || spec.kind == DeviceGradKind::Lambdarank ||
        spec.kind == DeviceGradKind::RankXendcg || spec.kind == DeviceGradKind::MulticlassOVA) {
      Log::Fatal("op gradients: objective '%s' has no point-wise device kernel", c.objective.c_str());
    }
    Scratch sc;
    dev::GradArgs g{};
    tuning::PoisonArgs(&g);  // (every field set below)
    g.kind = static_cast<int32_t>(spec.kind);
    g.num_class = spec.kind == DeviceGradKind::MulticlassSoftmax ? obj->NumModelPerIteration() : 1;
    g.num_data = n;
    g.p0 = spec.p0;
    g.p1 = spec.p1;
    g.p2 = spec.p2;
    g.lw0 = spec.label_weight[0];
    g.lw1 = spec.label_weight[1];
    g.label = sc.Upload(spec.label, n);
    g.weights = sc.Upload(spec.weights, n);
    g.label_weight = sc.Upload(spec.label_weight_arr, n);
    g.score = d_score;
    g.grad = d_grad;
    g.hess = d_hess;
    g.write_split = 1;
    g.gh = nullptr;
    g.gh_stride = 1;
    g.max_parts = nullptr;
    g.root_parts = nullptr;
    dev::Gradients(g, nullptr);
    OPCHECK(hipGetLastError());
    OPCHECK(hipDeviceSynchronize());
  });
}

// a validation metric of raw scores (device, float64, one model per iteration); params
// name the metric and the objective whose output transform applies
LIGHTGBM_C_EXPORT int LGBMAMD_OpMetric(const char* params, const float* label, const float* weight, int32_t n,
                                       const double* d_score, double* out) {
  return Guard([&] {
    Config c = ParseConfig(params);
    if (c.metric.empty()) Log::Fatal("op metric: no metric given");
    std::unique_ptr<Metric> m(Metric::CreateMetric(c.metric[0], c));
    if (!m) Log::Fatal("op metric: unknown metric '%s'", c.metric[0].c_str());
    std::unique_ptr<ObjectiveFunction> obj;
    if (!c.objective.empty() && c.objective != "none") {
      obj.reset(ObjectiveFunction::CreateObjectiveFunction(c.objective, c));
    }
    Metadata md;
    FillMetadata(&md, label, weight, n);
    m->Init(md, n);
    if (obj) obj->Init(md, n);
    const DeviceMetricSpec spec = m->DeviceSpec(obj.get());
    if (spec.kind == 0) Log::Fatal("op metric: '%s' has no device kernel for this objective", c.metric[0].c_str());
    bool negative_weight = false;
    for (int32_t i = 0; weight != nullptr && i < n && !negative_weight; ++i) negative_weight = weight[i] < 0.0f;
    if (spec.kind == dev::kMetricAUC && negative_weight) {
      // the device AUC carries the class in the weight's sign: evaluate these rows on the host
      std::vector<double> hs(static_cast<size_t>(std::max(0, n)));
      OPCHECK(hipMemcpy(hs.data(), d_score, sizeof(double) * hs.size(), hipMemcpyDeviceToHost));
      *out = m->Eval(hs.data(), obj.get())[0];
      return;
    }
    Scratch sc;
    dev::MetricArgs a{};
    a.kind = spec.kind;
    a.convert = spec.convert;
    a.sigmoid = spec.sigmoid;
    a.param = spec.param;
    a.num_class = spec.num_class;
    a.top_k = spec.top_k;
    a.n = n;
    a.score = d_score;
    a.label = sc.Upload(spec.label, n);
    a.weights = sc.Upload(spec.weights, n);
    a.scratch = sc.Alloc<char>(dev::MetricScratchBytes(n));
    if (spec.kind == dev::kMetricNDCG || spec.kind == dev::kMetricMAP) Log::Fatal("op metric: query metrics need queries");
    a.out = sc.Alloc<double>(2);
    dev::EvalMetric(a, nullptr);
    OPCHECK(hipGetLastError());
    std::vector<double> h(2, 0.0);
    OPCHECK(hipMemcpy(h.data(), a.out, sizeof(double) * 2, hipMemcpyDeviceToHost));
    *out = m->FinishDevice(h)[0];
  });
}

// one bagging (goss = 0) or GOSS (goss = 1) draw with fresh generators Random(seed + block):
// d_bag receives the in-bag rows ascending, d_oob the others; GOSS rescales the sampled
// small-gradient rows of d_grad / d_hess ([num_class][n]) in place
LIGHTGBM_C_EXPORT int LGBMAMD_OpSampleRows(int64_t n, int32_t seed, int32_t goss, int32_t num_class,
                                           double fraction, double top_rate, double other_rate, float* d_grad,
                                           float* d_hess, int32_t* d_bag, int32_t* d_oob, int32_t* out_count) {
  return Guard([&] {
    Scratch sc;
    const int64_t nb = dev::SampleBlocks(n);
    std::vector<uint32_t> st(nb);
    for (int64_t b = 0; b < nb; ++b) st[b] = static_cast<uint32_t>(seed + static_cast<int>(b));
    dev::SampleArgs s{};
    tuning::PoisonArgs(&s);
    s.num_data = n;
    s.num_blocks = nb;
    s.goss = goss;
    s.balanced = 0;
    s.num_class = num_class;
    s.fraction = fraction;
    s.pos_fraction = s.neg_fraction = 1.0;
    s.top_rate = top_rate;
    s.other_rate = other_rate;
    s.label = nullptr;
    s.grad = d_grad;
    s.hess = d_hess;
    s.rng = sc.Upload(st.data(), st.size());
    s.codes = sc.Alloc<uint8_t>(n);
    s.block_cnt = sc.Alloc<int32_t>(nb);
    s.block_off = sc.Alloc<int32_t>(nb);
    s.bag = d_bag;
    s.oob = d_oob;
    s.bag_count = sc.Alloc<int32_t>(1);
    dev::SampleRows(s, nullptr);
    OPCHECK(hipGetLastError());
    OPCHECK(hipMemcpy(out_count, s.bag_count, sizeof(int32_t), hipMemcpyDeviceToHost));
  });
}
