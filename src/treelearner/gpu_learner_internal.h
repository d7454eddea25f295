// Shared by the MI355X tree learner's host sources (gpu_tree_learner.cpp, gpu_learner_*.cpp).
#pragma once

#include "gpu_tree_learner.h"

#include "parallel_tree_learner.h"

#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>

#include "lgbm_amd/common.h"
#include "lgbm_amd/dcg.h"
#include "lgbm_amd/log.h"
#include "lgbm_amd/network.h"

#define HIPCHECK(x)                                                                               \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) Log::Fatal("HIP error %s at %s:%d: %s", #x, __FILE__, __LINE__, hipGetErrorString(e_)); \
  } while (0)

namespace lgbm_amd {

// device buffers live until FreeBuffers (every allocation is recorded)
template <typename T>
T* GPUTreeLearner::Alloc(size_t n) {
  void* p = nullptr;
  HIPCHECK(hipMalloc(&p, std::max<size_t>(1, n) * sizeof(T)));
  allocs_.push_back(p);
  return static_cast<T*>(p);
}

}  // namespace lgbm_amd
