// Cost-effective gradient boosting, lazy feature penalties, on the device (reference
// src/treelearner/cost_effective_gradient_boosting.hpp:29-60, 120-156; host
// src/treelearner/cegb.cpp).  A split on feature f in leaf l costs tradeoff * penalty_lazy[f]
// for every row of l that has not yet "paid" for f; once a leaf is split on f, all of its rows
// have.  The device keeps the paid (row, feature) pairs as a row-major bitset and every leaf's
// unpaid-row count per feature:
//   * root: counts over the root's rows (k_cegb_root);
//   * each step, after the partition (k_cegb_step): f is paid on every row of the split leaf
//     (one atomicOr per row), and the histogrammed child's counts are summed -- per wave, one
//     ballot per feature over 64 rows; the other child's are the split leaf's snapshot minus
//     those, and f's are 0 (the split scans derive and store both, split_kernels.hip).
#include "device_common.h"

namespace lgbm_amd {
namespace dev {

namespace {

constexpr int kCegbThreads = 256;
constexpr int kCegbMaxLdsFeatures = 8192;

// unpaid counts of `n` rows (rows[i], or i itself when rows is null) into out[f] (atomics)
__device__ void CegbCountRows(const KArgs& a, const int32_t* rows, int n, int32_t* out, int* cnt_lds) {
  const int F = a.p.num_features, pw = a.cegb_paid_words;
  const int lane = threadIdx.x & 63;
  for (int f = threadIdx.x; f < F; f += kCegbThreads) cnt_lds[f] = 0;
  __syncthreads();
  const int stride = gridDim.x * kCegbThreads;
  // whole waves step together over the rows (ballots need every lane)
  for (int i0 = blockIdx.x * kCegbThreads + (threadIdx.x & ~63); i0 < n; i0 += stride) {
    const int i = i0 + lane;
    const bool live = i < n;
    const int row = live ? (rows != nullptr ? rows[i] : i) : 0;
    const uint32_t* pr = a.cegb_paid + static_cast<int64_t>(row) * pw;
    for (int w = 0; w < pw; ++w) {
      const uint32_t bits = live ? pr[w] : 0xffffffffu;
      const int fmax = min(32, F - 32 * w);
      for (int b = 0; b < fmax; ++b) {
        const unsigned long long m = __ballot(((bits >> b) & 1u) == 0u);
        if (lane == 0 && m != 0ull) atomicAdd(&cnt_lds[32 * w + b], __popcll(m));
      }
    }
  }
  __syncthreads();
  for (int f = threadIdx.x; f < F; f += kCegbThreads) {
    if (cnt_lds[f] != 0) atomicAdd(&out[f], cnt_lds[f]);
  }
}

__global__ __launch_bounds__(kCegbThreads) void k_cegb_root(KArgs a) {
  extern __shared__ int cnt_lds[];
  const int n = RootRows(a);
  CegbCountRows(a, a.root_identity ? nullptr : a.idx, n, a.cegb_cnt, cnt_lds);
}

__global__ __launch_bounds__(kCegbThreads) void k_cegb_step(KArgs a) {
  extern __shared__ int cnt_lds[];
  const Step* st = a.st;
  if (st->done) return;
  const CurSplit& cs = st->cs;
  const int F = a.p.num_features, par = cs.s & 1;
  const int pb = cs.part_begin, pc = cs.part_count, fstar = cs.split.feature;
  int32_t* scratch = a.cegb_scratch + static_cast<size_t>(par) * F;
  if (blockIdx.x == 0) {
    // the split leaf's counts before its children replace them; the other parity's scratch
    // (read by the previous step's scans) is cleared for the next step
    int32_t* snap = a.cegb_snap + static_cast<size_t>(par) * F;
    int32_t* other = a.cegb_scratch + static_cast<size_t>(par ^ 1) * F;
    for (int f = threadIdx.x; f < F; f += kCegbThreads) {
      snap[f] = a.cegb_cnt[static_cast<size_t>(cs.leaf) * F + f];
      other[f] = 0;
    }
  }
  // the split feature is paid on every row of the leaf
  if (fstar >= 0) {
    const int32_t* src = RowBuf(a, cs.src_buf);
    const uint32_t bit = 1u << (fstar & 31);
    for (int i = blockIdx.x * kCegbThreads + threadIdx.x; i < pc; i += gridDim.x * kCegbThreads) {
      const int row = src[pb + i];
      atomicOr(&a.cegb_paid[static_cast<int64_t>(row) * a.cegb_paid_words + (fstar >> 5)], bit);
    }
  }
  // the histogrammed child's rows: [pb, pb + left) or the rest, in the other index buffer
  const int32_t* dst = RowBuf(a, cs.src_buf ? 0 : 1);
  const int left = st->cur_left;
  const int hb = st->hist_left ? pb : pb + left, hn = st->hist_left ? left : pc - left;
  CegbCountRows(a, dst + hb, hn, scratch, cnt_lds);
}

int CegbGrid(int64_t rows) { return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>((rows + 1023) / 1024, 2 * NumCUs()))); }

}  // namespace

void CegbRoot(const KArgs& a, hipStream_t s) {
  const size_t lds = sizeof(int) * std::min(a.p.num_features, kCegbMaxLdsFeatures);
  hipLaunchKernelGGL(k_cegb_root, dim3(CegbGrid(a.num_rows)), dim3(kCegbThreads), lds, s, a);
}

void CegbStep(const KArgs& a, hipStream_t s) {
  const size_t lds = sizeof(int) * std::min(a.p.num_features, kCegbMaxLdsFeatures);
  hipLaunchKernelGGL(k_cegb_step, dim3(CegbGrid(a.num_rows)), dim3(kCegbThreads), lds, s, a);
}

}  // namespace dev
}  // namespace lgbm_amd
