// Batch prediction of a forest on raw feature values (reference Tree::GetLeaf /
// NumericalDecision / CategoricalDecision, include/LightGBM/tree.h:265-337,578-598, and
// GBDT::PredictRaw, src/boosting/gbdt_prediction.cpp:13-40).
//
// One thread per row walks every tree in model order, accumulating the raw score of each
// class in registers in the same order as the host predictor (bit-identical sums).  The
// flattened forest (a few hundred KB for 500 x 63-leaf trees) stays L2-resident and every
// wave reads the same node at the same time; dense rows follow the C API's convention of
// treating |v| <= kZeroThreshold as 0.
#include "device_common.h"

namespace lgbm_amd {
namespace dev {

namespace {

constexpr double kPredZero = 1e-35f;  // kZeroThreshold

template <typename T, bool ROW_MAJOR>
__global__ __launch_bounds__(256) void k_predict_forest(ForestArgs f) {
  const int64_t row = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (row >= f.num_rows) return;
  double acc[kMaxPredClasses];
#pragma unroll
  for (int k = 0; k < kMaxPredClasses; ++k) acc[k] = 0.0;
  const T* x = static_cast<const T*>(f.data);
  for (int t = 0; t < f.num_trees; ++t) {
    const int n0 = f.node_off[t], n1 = f.node_off[t + 1];
    int leaf = 0;
    if (n1 > n0) {
      int node = 0;
      while (node >= 0) {
        const int gi = n0 + node;
        const int feat = f.feature[gi];
        double v = ROW_MAJOR ? static_cast<double>(x[row * f.num_cols + feat])
                             : static_cast<double>(x[static_cast<int64_t>(feat) * f.num_rows + row]);
        if (fabs(v) <= kPredZero) v = 0.0;
        const int8_t dt = f.dtype[gi];
        const int mt = (dt >> 2) & 3;
        bool left;
        if (dt & 1) {  // categorical
          int iv = static_cast<int>(v);
          if (iv < 0) {
            left = false;
          } else if (v != v && mt == 2) {
            left = false;
          } else {
            if (v != v) iv = 0;
            const int32_t* bound = f.cat_bound + f.cat_bound_off[t];
            const uint32_t* bits = f.cat_bits + f.cat_bits_off[t];
            const int ci = static_cast<int>(f.threshold[gi]);
            const int lo = bound[ci], nw = bound[ci + 1] - lo;
            const int w = iv >> 5;
            left = w < nw && ((bits[lo + w] >> (iv & 31)) & 1u);
          }
        } else {
          if (v != v && mt != 2) v = 0.0;
          if ((mt == 1 && fabs(v) <= kPredZero) || (mt == 2 && v != v)) {
            left = (dt & 2) != 0;
          } else {
            left = v <= f.threshold[gi];
          }
        }
        node = left ? f.left[gi] : f.right[gi];
      }
      leaf = ~node;
    }
    const double lv = f.leaf_value[f.leaf_off[t] + leaf];
    const int k = t % f.num_class;
#pragma unroll
    for (int c = 0; c < kMaxPredClasses; ++c) {
      if (c == k) acc[c] += lv;
    }
  }
  for (int c = 0; c < f.num_class; ++c) f.out[row * f.num_class + c] = acc[c];
}

}  // namespace

void PredictForest(const ForestArgs& f, hipStream_t s) {
  if (f.num_rows <= 0) return;
  const dim3 grid(static_cast<unsigned>((f.num_rows + 255) / 256));
  if (f.is_double) {
    if (f.row_major) hipLaunchKernelGGL((k_predict_forest<double, true>), grid, dim3(256), 0, s, f);
    else hipLaunchKernelGGL((k_predict_forest<double, false>), grid, dim3(256), 0, s, f);
  } else {
    if (f.row_major) hipLaunchKernelGGL((k_predict_forest<float, true>), grid, dim3(256), 0, s, f);
    else hipLaunchKernelGGL((k_predict_forest<float, false>), grid, dim3(256), 0, s, f);
  }
}

}  // namespace dev
}  // namespace lgbm_amd
