// Dense-matrix prediction on the MI355X (the C API's LGBM_BoosterPredictForMat path for a
// booster trained with device_type=gpu, or predicted with device_type=gpu): the forest is
// flattened into node arrays and evaluated by src/device/predict_kernels.hip, one row per
// thread, with the host predictor's semantics (reference GBDT::PredictRaw / Predict,
// src/boosting/gbdt_prediction.cpp:13-64); output transforms stay on the host.
#include <hip/hip_runtime_api.h>
#include <omp.h>

#include <cstring>
#include <vector>

#include "../device/kernels.h"
#include "lgbm_amd/boosting.h"
#include "lgbm_amd/log.h"

namespace lgbm_amd {

namespace {

#define HIPCHECK(x)                                                                                 \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) Log::Fatal("HIP error %s at %s:%d: %s", #x, __FILE__, __LINE__, hipGetErrorString(e_)); \
  } while (0)

// device copies of host vectors, freed together
struct DeviceBuffers {
  std::vector<void*> ptrs;
  ~DeviceBuffers() {
    for (void* p : ptrs) (void)hipFree(p);
  }
  template <typename T>
  T* Upload(const std::vector<T>& v, hipStream_t s) {
    void* p = nullptr;
    HIPCHECK(hipMalloc(&p, std::max<size_t>(1, v.size()) * sizeof(T)));
    ptrs.push_back(p);
    if (!v.empty()) HIPCHECK(hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
    return static_cast<T*>(p);
  }
  void* Alloc(size_t bytes) {
    void* p = nullptr;
    HIPCHECK(hipMalloc(&p, std::max<size_t>(1, bytes)));
    ptrs.push_back(p);
    return p;
  }
};

}  // namespace

bool GBDT::PredictDenseOnDevice(const void* data, bool is_double, int64_t nrow, int ncol, bool row_major,
                                int start_iteration, int num_iteration, bool raw, double* out) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return false;
  if (num_tree_per_iteration_ > dev::kMaxPredClasses || nrow <= 0) return false;
  InitPredict(start_iteration, num_iteration, false);
  const int ntpi = num_tree_per_iteration_;
  const int t0 = start_iteration_for_pred_ * ntpi;
  const int nt = num_iteration_for_pred_ * ntpi;
  // flatten the forest (rebuilt per call: trees may have been edited in place)
  std::vector<int32_t> node_off(nt + 1, 0), leaf_off(nt, 0), feature, left, right;
  std::vector<int32_t> cat_bound_off(nt, 0), cat_bound, cat_bits_off(nt, 0);
  std::vector<double> thr, leafv;
  std::vector<int8_t> dtype;
  std::vector<uint32_t> cat_bits;
  for (int i = 0; i < nt; ++i) {
    const Tree* tr = models_[t0 + i].get();
    node_off[i] = static_cast<int32_t>(feature.size());
    leaf_off[i] = static_cast<int32_t>(leafv.size());
    cat_bound_off[i] = static_cast<int32_t>(cat_bound.size());
    cat_bits_off[i] = static_cast<int32_t>(cat_bits.size());
    const int nl = tr->num_leaves();
    for (int j = 0; j + 1 < nl; ++j) {
      feature.push_back(tr->split_feature(j));
      thr.push_back(tr->threshold(j));
      dtype.push_back(tr->decision_type(j));
      left.push_back(tr->left_child(j));
      right.push_back(tr->right_child(j));
    }
    for (int j = 0; j < nl; ++j) leafv.push_back(tr->LeafOutput(j));
    cat_bound.insert(cat_bound.end(), tr->cat_boundaries().begin(), tr->cat_boundaries().end());
    cat_bits.insert(cat_bits.end(), tr->cat_threshold().begin(), tr->cat_threshold().end());
  }
  node_off[nt] = static_cast<int32_t>(feature.size());
  hipStream_t s;
  HIPCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::vector<double> raw_out(static_cast<size_t>(nrow) * ntpi);
  {
    DeviceBuffers b;
    dev::ForestArgs f{};
    f.num_trees = nt;
    f.num_class = ntpi;
    f.num_cols = ncol;
    f.is_double = is_double ? 1 : 0;
    f.row_major = row_major ? 1 : 0;
    f.num_rows = nrow;
    const size_t data_bytes = static_cast<size_t>(nrow) * ncol * (is_double ? 8 : 4);
    void* d_data = b.Alloc(data_bytes);
    HIPCHECK(hipMemcpyAsync(d_data, data, data_bytes, hipMemcpyHostToDevice, s));
    f.data = d_data;
    f.node_off = b.Upload(node_off, s);
    f.leaf_off = b.Upload(leaf_off, s);
    f.feature = b.Upload(feature, s);
    f.threshold = b.Upload(thr, s);
    f.dtype = b.Upload(dtype, s);
    f.left = b.Upload(left, s);
    f.right = b.Upload(right, s);
    f.leaf_value = b.Upload(leafv, s);
    f.cat_bound_off = b.Upload(cat_bound_off, s);
    f.cat_bound = b.Upload(cat_bound, s);
    f.cat_bits_off = b.Upload(cat_bits_off, s);
    f.cat_bits = b.Upload(cat_bits, s);
    f.out = static_cast<double*>(b.Alloc(raw_out.size() * sizeof(double)));
    dev::PredictForest(f, s);
    HIPCHECK(hipMemcpyAsync(raw_out.data(), f.out, raw_out.size() * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHECK(hipStreamSynchronize(s));
  }
  HIPCHECK(hipStreamDestroy(s));
  if (raw) {
    std::memcpy(out, raw_out.data(), raw_out.size() * sizeof(double));
    return true;
  }
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < nrow; ++r) {
    double* o = out + r * ntpi;
    std::memcpy(o, raw_out.data() + r * ntpi, sizeof(double) * ntpi);
    if (average_output_) {
      for (int k = 0; k < ntpi; ++k) o[k] /= num_iteration_for_pred_;
    }
    if (objective_ != nullptr) objective_->ConvertOutput(o, o);
  }
  return true;
}

}  // namespace lgbm_amd
