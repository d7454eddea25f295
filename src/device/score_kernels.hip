// Training-score updates with a finished tree (reference ScoreUpdater::AddScore /
// Tree::AddPredictionToScore, src/boosting/score_updater.hpp, src/io/tree.cpp).
//
// k_add_tree_score walks the tree for every (or every listed) row of the binned matrix:
// the tree's nodes -- with each split feature's decode parameters -- are staged in LDS and
// each thread stages its row's bin words in LDS, so a level costs two LDS reads.  Rows and
// scores are streamed in order (coalesced), which beats scattering leaf values through
// the partition order.
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "objective_common.h"
#include "lgbm_amd/tuning.h"

namespace lgbm_amd {
namespace dev {

__global__ void k_add_leaf_score(KArgs a, const double* __restrict__ vals, int num_leaves, double* __restrict__ score) {
  const int leaf = blockIdx.y;
  if (leaf >= num_leaves) return;
  const Leaf lf = a.leaves[leaf];
  const double v = vals[leaf];
  const int32_t* ids = RowBuf(a, lf.buf);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < lf.count; i += gridDim.x * blockDim.x) {
    score[ids[lf.begin + i]] += v;
  }
}

void AddLeafScore(const KArgs& a, const double* leaf_values, int num_leaves, double* score, hipStream_t s) {
  const int bx = std::max(1, std::min(64, (a.num_rows / std::max(1, num_leaves) + 255) / 256));
  hipLaunchKernelGGL(k_add_leaf_score, dim3(bx, num_leaves), dim3(256), 0, s, a, leaf_values, num_leaves, score);
}

namespace {
constexpr int kMaxNodes = 255;
constexpr int kMaxRowWords = 16;

struct NodeInfo {
  int32_t gbyte;                   // the split group's byte offset in a row (Feature::gbyte)
  int16_t gwide, left_is_default;  // 16-bit group; default direction for missing values
  int16_t missing_type, is_cat;
  int32_t sub_lo, sub_hi, offset, mfb, default_bin, max_bin;
  uint32_t threshold;
  int32_t left, right;
  int64_t col_off;                 // the group's column (row-sparse training storage)
};
}  // namespace

__device__ __forceinline__ NodeInfo MakeNode(const KArgs& a, const DevTree& t, int i) {
    const int f = t.split_feature_inner[i];
    const Feature F = a.feat[f];
    const int8_t dt = t.decision_type[i];
    NodeInfo nd;
    nd.gbyte = F.gbyte;
    nd.gwide = static_cast<int16_t>(F.gwide);
    nd.col_off = F.col_off;
    nd.left_is_default = (dt & 2) ? 1 : 0;
    nd.missing_type = static_cast<int16_t>((dt >> 2) & 3);
    nd.is_cat = (dt & 1) ? 1 : 0;
    nd.sub_lo = F.sub_lo;
    nd.sub_hi = F.sub_hi;
    nd.offset = F.offset;
    nd.mfb = F.mfb;
    nd.default_bin = F.default_bin;
    nd.max_bin = F.num_bin - 1;
    nd.threshold = t.threshold_in_bin[i];
    nd.left = t.left_child[i];
    nd.right = t.right_child[i];
    return nd;
}

// STAGED: tree (<= kMaxNodes internal nodes) cached in LDS; otherwise read from HBM
template <bool STAGED>
__global__ __launch_bounds__(256) void k_add_tree_score(KArgs a, DevTree t, const int32_t* __restrict__ rows,
                                                        int64_t n, double* __restrict__ score) {
  __shared__ NodeInfo s_node[STAGED ? kMaxNodes : 1];
  __shared__ double s_val[STAGED ? kMaxNodes + 1 : 1];
  __shared__ uint32_t s_row[256 * kMaxRowWords];
  const int ni = t.num_leaves - 1;
  if (STAGED) {
    for (int i = threadIdx.x; i < ni; i += blockDim.x) s_node[i] = MakeNode(a, t, i);
    for (int i = threadIdx.x; i < t.num_leaves; i += blockDim.x) s_val[i] = t.leaf_value[i];
  }
  __syncthreads();
  const int wpr = a.words_per_row;
  const int64_t stride = a.row_words;
  const bool words = a.bins != nullptr;  // else row-sparse training storage: the column copy
  const bool stage_row = words && wpr <= kMaxRowWords;
  const uint32_t* bins32 = static_cast<const uint32_t*>(a.bins);
  uint32_t* my = s_row + threadIdx.x * kMaxRowWords;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int row = rows ? rows[i] : static_cast<int>(i);
    int node = 0;
    if (t.num_leaves > 1) {
      if (stage_row) {
        for (int k = 0; k < wpr; ++k) my[k] = bins32[static_cast<int64_t>(row) * stride + k];
      }
      while (node >= 0) {
        const NodeInfo nd = STAGED ? s_node[node] : MakeNode(a, t, node);
        uint32_t gb;
        if (stage_row) {
          gb = GroupBinAt(reinterpret_cast<const uint8_t*>(my) + nd.gbyte, nd.gwide);
        } else {
          gb = words ? RowBin(a, row, nd.gbyte, nd.gwide) : ColBin(a, row, nd.gbyte, nd.gwide, nd.col_off);
        }
        const uint32_t bin = (gb < static_cast<uint32_t>(nd.sub_lo) || gb >= static_cast<uint32_t>(nd.sub_hi))
                                 ? static_cast<uint32_t>(nd.mfb)
                                 : gb - nd.sub_lo + nd.offset;
        bool left;
        if (nd.is_cat) {
          const int ci = static_cast<int>(nd.threshold);
          const int lo = t.cat_boundaries_inner[ci], hi = t.cat_boundaries_inner[ci + 1];
          const int word = static_cast<int>(bin >> 5);
          left = word < hi - lo && ((t.cat_threshold_inner[lo + word] >> (bin & 31u)) & 1u);
        } else if ((nd.missing_type == 1 && bin == static_cast<uint32_t>(nd.default_bin)) ||
                   (nd.missing_type == 2 && bin == static_cast<uint32_t>(nd.max_bin))) {
          left = nd.left_is_default != 0;
        } else {
          left = bin <= nd.threshold;
        }
        node = left ? nd.left : nd.right;
      }
      node = ~node;
    }
    score[row] += STAGED ? s_val[node] : t.leaf_value[node];
  }
}

// ---------------------------------------------------------------- bitmap traversal
// For 8-bit storage columns every decision of a node (numerical threshold, missing-value
// routing, categorical set, the group-bin -> feature-bin mapping of bundles) collapses into
// one 256-bit "goes left" set over the raw group bin: a level of the walk is then a byte
// read of the row, a bit test and a child index, all from LDS.
__global__ __launch_bounds__(256) void k_tree_bitmaps(KArgs a, DevTree t) {
  const int node = blockIdx.x;
  const NodeInfo nd = MakeNode(a, t, node);
  // raw byte 0..255 of the row at the group's offset: its bin (4-bit groups: one half of it)
  const uint32_t gb = nd.gwide >= 2 ? (threadIdx.x >> ((nd.gwide & 1) * 4)) & 15u : threadIdx.x;
  const uint32_t bin = (gb < static_cast<uint32_t>(nd.sub_lo) || gb >= static_cast<uint32_t>(nd.sub_hi))
                           ? static_cast<uint32_t>(nd.mfb)
                           : gb - nd.sub_lo + nd.offset;
  bool left;
  if (nd.is_cat) {
    const int ci = static_cast<int>(nd.threshold);
    const int lo = t.cat_boundaries_inner[ci], hi = t.cat_boundaries_inner[ci + 1];
    const int word = static_cast<int>(bin >> 5);
    left = word < hi - lo && ((t.cat_threshold_inner[lo + word] >> (bin & 31u)) & 1u);
  } else if ((nd.missing_type == 1 && bin == static_cast<uint32_t>(nd.default_bin)) ||
             (nd.missing_type == 2 && bin == static_cast<uint32_t>(nd.max_bin))) {
    left = nd.left_is_default != 0;
  } else {
    left = bin <= nd.threshold;
  }
  const unsigned long long m = __ballot(left);
  if ((threadIdx.x & 63) == 0) t.bm_work[node * 4 + (threadIdx.x >> 6)] = m;
  if (threadIdx.x == 0) {
    // group byte offset | left child (16 bits, two's complement leaves) | right child
    t.bm_meta[node * 3 + 0] = nd.gbyte;
    t.bm_meta[node * 3 + 1] = nd.left;
    t.bm_meta[node * 3 + 2] = nd.right;
  }
}

constexpr int kBmRowsPerBlock = 256;
constexpr int kBmMaxRowBytes = 64;

__global__ __launch_bounds__(kBmRowsPerBlock) void k_add_tree_score_bm(KArgs a, DevTree t, int64_t n,
                                                                        double* __restrict__ score) {
  __shared__ unsigned long long s_bm[kMaxNodes * 4];
  __shared__ int16_t s_group[kMaxNodes], s_left[kMaxNodes], s_right[kMaxNodes];
  __shared__ double s_val[kMaxNodes + 1];
  extern __shared__ uint32_t s_rows[];  // [kBmRowsPerBlock][words_per_row]
  const int ni = t.num_leaves - 1;
  for (int i = threadIdx.x; i < ni * 4; i += blockDim.x) s_bm[i] = t.bm_work[i];
  for (int i = threadIdx.x; i < ni; i += blockDim.x) {
    s_group[i] = static_cast<int16_t>(t.bm_meta[i * 3 + 0]);
    s_left[i] = static_cast<int16_t>(t.bm_meta[i * 3 + 1]);
    s_right[i] = static_cast<int16_t>(t.bm_meta[i * 3 + 2]);
  }
  for (int i = threadIdx.x; i < t.num_leaves; i += blockDim.x) s_val[i] = t.leaf_value[i];
  const int wpr = a.row_words;  // (whole rows, (g, h) of interleaved rows included)
  const uint32_t* bins32 = static_cast<const uint32_t*>(a.bins);
  const uint8_t* rows8 = reinterpret_cast<const uint8_t*>(s_rows);
  // a workgroup walks several chunks: the next chunk's row words (one contiguous run of the
  // row-major matrix, coalesced) and scores are loaded into registers while this one is walked
  constexpr int kW = kBmMaxRowBytes / 4;  // words per thread and chunk, at most
  const int64_t step = static_cast<int64_t>(gridDim.x) * kBmRowsPerBlock;
  uint32_t pre[kW];
  double sc = 0.0;
  auto load = [&](int64_t r0) {
    const int nr = static_cast<int>(min<int64_t>(kBmRowsPerBlock, n - r0));
    const uint32_t* src = bins32 + r0 * wpr;
#pragma unroll
    for (int k = 0; k < kW; ++k) {
      const int i = threadIdx.x + k * kBmRowsPerBlock;
      pre[k] = (k < wpr && i < nr * wpr) ? src[i] : 0u;
    }
    sc = threadIdx.x < nr ? score[r0 + threadIdx.x] : 0.0;
  };
  int64_t r0 = static_cast<int64_t>(blockIdx.x) * kBmRowsPerBlock;
  if (r0 < n) load(r0);
  for (; r0 < n; r0 += step) {
    const int nr = static_cast<int>(min<int64_t>(kBmRowsPerBlock, n - r0));
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kW; ++k) {
      const int i = threadIdx.x + k * kBmRowsPerBlock;
      if (k < wpr && i < nr * wpr) s_rows[i] = pre[k];
    }
    const double my = sc;
    __syncthreads();
    if (r0 + step < n) load(r0 + step);
    if (threadIdx.x < nr) {
      const uint8_t* row = rows8 + threadIdx.x * wpr * 4;
      int node = 0;
      while (node >= 0) {
        const uint32_t gb = row[s_group[node]];
        const bool left = (s_bm[node * 4 + (gb >> 6)] >> (gb & 63u)) & 1ull;
        node = left ? s_left[node] : s_right[node];
      }
      score[r0 + threadIdx.x] = my + s_val[~node];
    }
  }
}

// The bitmap walk that also computes the next iteration's gradients from the updated score
// (point-wise objectives, one model per iteration): the next gradient kernel would re-read
// every row's score and label right after this pass wrote them.  Writes the interleaved
// (g, h) and the per-workgroup max |g| / max h and (sum g, sum h) partials of k_gradients
// (reduced in a fixed order by k_reduce_parts); grad / hess are not written.
#ifndef LGBM_BMG_WAVES
#define LGBM_BMG_WAVES 5
#endif
// KIND: the objective (GradArgs::kind), a compile-time constant so that only its math is
// inlined (every kind inlined takes 171 VGPRs: 2 waves per SIMD against the walk's 7)
// W: row words prefetched per thread and chunk (>= row_words; 8 or 16)
template <int KIND, int W>
__global__ __launch_bounds__(kBmRowsPerBlock) __attribute__((amdgpu_waves_per_eu(LGBM_BMG_WAVES))) void k_add_tree_score_bm_grad(KArgs a, DevTree t, int64_t n,
                                                                             double* __restrict__ score, GradArgs ga) {
  ga.kind = KIND;
  __shared__ unsigned long long s_bm[kMaxNodes * 4];
  __shared__ int16_t s_group[kMaxNodes], s_left[kMaxNodes], s_right[kMaxNodes];
  __shared__ double s_val[kMaxNodes + 1];
  __shared__ float smg[kBmRowsPerBlock / kWave], smh[kBmRowsPerBlock / kWave];
  __shared__ double ssg[kBmRowsPerBlock / kWave], ssh[kBmRowsPerBlock / kWave];
  extern __shared__ uint32_t s_rows[];  // [kBmRowsPerBlock][row_words]
  const int ni = t.num_leaves - 1;
  for (int i = threadIdx.x; i < ni * 4; i += blockDim.x) s_bm[i] = t.bm_work[i];
  for (int i = threadIdx.x; i < ni; i += blockDim.x) {
    s_group[i] = static_cast<int16_t>(t.bm_meta[i * 3 + 0]);
    s_left[i] = static_cast<int16_t>(t.bm_meta[i * 3 + 1]);
    s_right[i] = static_cast<int16_t>(t.bm_meta[i * 3 + 2]);
  }
  for (int i = threadIdx.x; i < t.num_leaves; i += blockDim.x) s_val[i] = t.leaf_value[i];
  const int wpr = a.row_words;
  const uint32_t* bins32 = static_cast<const uint32_t*>(a.bins);
  const uint8_t* rows8 = reinterpret_cast<const uint8_t*>(s_rows);
  constexpr int kW = W;
  const int64_t step = static_cast<int64_t>(gridDim.x) * kBmRowsPerBlock;
  uint32_t pre[kW];
  double sc = 0.0, yv = 0.0, wv = 1.0;
  auto load = [&](int64_t r0) {
    const int nr = static_cast<int>(min<int64_t>(kBmRowsPerBlock, n - r0));
    const uint32_t* src = bins32 + r0 * wpr;
#pragma unroll
    for (int k = 0; k < kW; ++k) {
      const int i = threadIdx.x + k * kBmRowsPerBlock;
      pre[k] = (k < wpr && i < nr * wpr) ? src[i] : 0u;
    }
    const bool ok = threadIdx.x < nr;
    sc = ok ? score[r0 + threadIdx.x] : 0.0;
    yv = ok ? static_cast<double>(ga.label[r0 + threadIdx.x]) : 0.0;
    wv = ok && ga.weights != nullptr ? static_cast<double>(ga.weights[r0 + threadIdx.x]) : 1.0;
  };
  float mg = 0.f, mh = 0.f;
  double sg = 0.0, shh = 0.0;
  int64_t r0 = static_cast<int64_t>(blockIdx.x) * kBmRowsPerBlock;
  if (r0 < n) load(r0);
  for (; r0 < n; r0 += step) {
    const int nr = static_cast<int>(min<int64_t>(kBmRowsPerBlock, n - r0));
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kW; ++k) {
      const int i = threadIdx.x + k * kBmRowsPerBlock;
      if (k < wpr && i < nr * wpr) s_rows[i] = pre[k];
    }
    const double my = sc, y = yv, w = wv;
    __syncthreads();
    if (r0 + step < n) load(r0 + step);
    if (threadIdx.x < nr) {
      const uint8_t* row = rows8 + threadIdx.x * wpr * 4;
      int node = 0;
      while (node >= 0) {
        const uint32_t gb = row[s_group[node]];
        const bool left = (s_bm[node * 4 + (gb >> 6)] >> (gb & 63u)) & 1ull;
        node = left ? s_left[node] : s_right[node];
      }
      const int64_t i = r0 + threadIdx.x;
      const double s1 = my + s_val[~node];
      score[i] = s1;
      double g, h;
      RowGrad(ga, i, n, y, s1, w, g, h);
      const float gf = static_cast<float>(g), hf = static_cast<float>(h);
      reinterpret_cast<float2*>(ga.gh)[i * ga.gh_stride] = make_float2(gf, hf);
      mg = fmaxf(mg, fabsf(gf));
      mh = HessMax(mh, hf);
      sg += gf;
      shh += hf;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    mg = fmaxf(mg, __shfl_xor(mg, o, kWave));
    mh = HessMax(mh, __shfl_xor(mh, o, kWave));
    sg += __shfl_xor(sg, o, kWave);
    shh += __shfl_xor(shh, o, kWave);
  }
  const int wv_ = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    smg[wv_] = mg;
    smh[wv_] = mh;
    ssg[wv_] = sg;
    ssh[wv_] = shh;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double tg = 0.0, th = 0.0;
    for (int i = 0; i < kBmRowsPerBlock / kWave; ++i) {
      mg = fmaxf(mg, smg[i]);
      mh = HessMax(mh, smh[i]);
      tg += ssg[i];
      th += ssh[i];
    }
    ga.max_parts[2 * blockIdx.x] = mg;
    ga.max_parts[2 * blockIdx.x + 1] = mh;
    ga.root_parts[2 * blockIdx.x] = tg;
    ga.root_parts[2 * blockIdx.x + 1] = th;
  }
}

// ---------------------------------------------------------------- tree from split records
namespace {
struct TreeBlob {
  int32_t* split_feature_inner;
  int32_t* left_child;
  int32_t* right_child;
  int32_t* cat_boundaries_inner;
  uint32_t* threshold_in_bin;
  uint32_t* cat_threshold_inner;
  double* leaf_value;
  int8_t* decision_type;
};
TreeBlob BlobLayout(char* blob, int max_leaves) {
  const size_t ni = static_cast<size_t>(std::max(1, max_leaves - 1));
  auto up8 = [](size_t x) { return (x + 7) & ~static_cast<size_t>(7); };
  TreeBlob b;
  size_t o = 0;
  b.leaf_value = reinterpret_cast<double*>(blob + o);
  o += up8(sizeof(double) * (ni + 1));
  b.split_feature_inner = reinterpret_cast<int32_t*>(blob + o);
  o += up8(4 * ni);
  b.left_child = reinterpret_cast<int32_t*>(blob + o);
  o += up8(4 * ni);
  b.right_child = reinterpret_cast<int32_t*>(blob + o);
  o += up8(4 * ni);
  b.cat_boundaries_inner = reinterpret_cast<int32_t*>(blob + o);
  o += up8(4 * (ni + 1));
  b.threshold_in_bin = reinterpret_cast<uint32_t*>(blob + o);
  o += up8(4 * ni);
  b.decision_type = reinterpret_cast<int8_t*>(blob + o);
  o += up8(ni);
  b.cat_threshold_inner = reinterpret_cast<uint32_t*>(blob + o);
  return b;
}
}  // namespace

// One workgroup.  Split s is internal node s; its left child starts as its leaf and its right
// child as the new leaf s + 1 (Tree::SplitCommon), and the node takes the place of its leaf in
// the parent -- the last earlier split that split that leaf or created it.  A leaf's value is
// the output the last split touching it gave it (NaN -> 0), times the shrinkage, rounded to
// zero below kZeroThreshold (Tree::Shrinkage).
__global__ __launch_bounds__(256) void k_tree_from_records(KArgs a, int ns, double shrink, TreeBlob o) {
  __shared__ int s_leaf[kMaxNodes];
  __shared__ int s_cat[kMaxNodes];
  for (int s = threadIdx.x; s < ns; s += blockDim.x) {
    s_leaf[s] = a.rec[s].leaf;
    s_cat[s] = a.rec[s].split.is_categorical ? 1 : 0;
  }
  __syncthreads();
  for (int s = threadIdx.x; s < ns; s += blockDim.x) {
    const DeviceSplit& d = a.rec[s].split;
    const int f = d.feature;
    const int missing = a.feat[f].missing_type;
    o.split_feature_inner[s] = f;
    o.left_child[s] = ~s_leaf[s];
    o.right_child[s] = ~(s + 1);
    if (s_cat[s]) {
      int ci = 0;
      for (int k = 0; k < s; ++k) ci += s_cat[k];
      o.threshold_in_bin[s] = static_cast<uint32_t>(ci);
      o.decision_type[s] = static_cast<int8_t>(1 | (missing << 2));
      for (int w = 0; w < kMaxCatWords; ++w) o.cat_threshold_inner[static_cast<size_t>(ci) * kMaxCatWords + w] = d.cat_bits[w];
    } else {
      o.threshold_in_bin[s] = static_cast<uint32_t>(d.threshold);
      o.decision_type[s] = static_cast<int8_t>((d.default_left ? 2 : 0) | (missing << 2));
    }
  }
  for (int k = threadIdx.x; k <= ns; k += blockDim.x) o.cat_boundaries_inner[k] = k * kMaxCatWords;
  __syncthreads();  // (the default children are written: the parents' slots are replaced below)
  for (int s = 1 + static_cast<int>(threadIdx.x); s < ns; s += blockDim.x) {
    const int l = s_leaf[s];
    int p = s - 1;
    while (s_leaf[p] != l && p != l - 1) --p;  // (split 0 split leaf 0: every leaf has one)
    if (s_leaf[p] == l) o.left_child[p] = s;
    else o.right_child[p] = s;
  }
  for (int l = threadIdx.x; l <= ns; l += blockDim.x) {
    int p = ns - 1;
    while (s_leaf[p] != l && p != l - 1) --p;
    const DeviceSplit& d = a.rec[p].split;
    double v = s_leaf[p] == l ? d.left_output : d.right_output;
    if (isnan(v)) v = 0.0;
    v *= shrink;
    o.leaf_value[l] = (v >= -kZeroThreshold && v <= kZeroThreshold) ? 0.0 : v;
  }
}

// k_tree_from_records and k_tree_bitmaps in one launch (one workgroup per internal node; the
// score walk's two single-purpose launches were ~4.5 us each on the tree's critical path).
// Node s's children: the first later split of its leaf (left) or of its new leaf s + 1 (right),
// else those leaves -- the same links as k_tree_from_records' parent search (a split's parent is
// the last earlier split of its leaf, and no split between s and that first one touches it).
// Workgroup 0 also writes the leaf values and the category boundaries.
__global__ __launch_bounds__(256) void k_tree_from_records_bm(KArgs a, int ns, double shrink, TreeBlob o,
                                                              unsigned long long* bm_work, int32_t* bm_meta) {
  __shared__ int s_leaf[kMaxNodes];
  __shared__ int s_cat[kMaxNodes];
  __shared__ int s_lr[2];
  const int s = blockIdx.x;
  for (int k = threadIdx.x; k < ns; k += blockDim.x) {
    s_leaf[k] = a.rec[k].leaf;
    s_cat[k] = a.rec[k].split.is_categorical ? 1 : 0;
  }
  if (threadIdx.x == 0) s_lr[0] = s_lr[1] = 0x7fffffff;
  __syncthreads();
  const int l = s_leaf[s];
  for (int k = s + 1 + static_cast<int>(threadIdx.x); k < ns; k += blockDim.x) {
    if (s_leaf[k] == l) atomicMin(&s_lr[0], k);
    if (s_leaf[k] == s + 1) atomicMin(&s_lr[1], k);
  }
  if (s == 0) {
    for (int k = threadIdx.x; k <= ns; k += blockDim.x) o.cat_boundaries_inner[k] = k * kMaxCatWords;
    for (int lf = threadIdx.x; lf <= ns; lf += blockDim.x) {
      int p = ns - 1;
      while (s_leaf[p] != lf && p != lf - 1) --p;
      const DeviceSplit& d = a.rec[p].split;
      double v = s_leaf[p] == lf ? d.left_output : d.right_output;
      if (isnan(v)) v = 0.0;
      v *= shrink;
      o.leaf_value[lf] = (v >= -kZeroThreshold && v <= kZeroThreshold) ? 0.0 : v;
    }
  }
  __syncthreads();
  const DeviceSplit& d = a.rec[s].split;
  const int f = d.feature;
  const Feature F = a.feat[f];
  const bool cat = s_cat[s] != 0;
  int ci = 0;
  if (cat) {
    for (int k = 0; k < s; ++k) ci += s_cat[k];
  }
  NodeInfo nd;
  nd.gbyte = F.gbyte;
  nd.gwide = static_cast<int16_t>(F.gwide);
  nd.col_off = F.col_off;
  nd.left_is_default = (!cat && d.default_left) ? 1 : 0;
  nd.missing_type = static_cast<int16_t>(F.missing_type);
  nd.is_cat = cat ? 1 : 0;
  nd.sub_lo = F.sub_lo;
  nd.sub_hi = F.sub_hi;
  nd.offset = F.offset;
  nd.mfb = F.mfb;
  nd.default_bin = F.default_bin;
  nd.max_bin = F.num_bin - 1;
  nd.threshold = cat ? static_cast<uint32_t>(ci) : static_cast<uint32_t>(d.threshold);
  nd.left = s_lr[0] != 0x7fffffff ? s_lr[0] : ~l;
  nd.right = s_lr[1] != 0x7fffffff ? s_lr[1] : ~(s + 1);
  if (threadIdx.x == 0) {
    o.split_feature_inner[s] = f;
    o.left_child[s] = nd.left;
    o.right_child[s] = nd.right;
    o.threshold_in_bin[s] = nd.threshold;
    o.decision_type[s] = static_cast<int8_t>((cat ? 1 : (d.default_left ? 2 : 0)) | (F.missing_type << 2));
    bm_meta[s * 3 + 0] = nd.gbyte;
    bm_meta[s * 3 + 1] = nd.left;
    bm_meta[s * 3 + 2] = nd.right;
  }
  if (cat) {
    for (int w = threadIdx.x; w < kMaxCatWords; w += blockDim.x) {
      o.cat_threshold_inner[static_cast<size_t>(ci) * kMaxCatWords + w] = d.cat_bits[w];
    }
  }
  // the node's "goes left" set over the raw group byte (k_tree_bitmaps)
  const uint32_t gb = nd.gwide >= 2 ? (threadIdx.x >> ((nd.gwide & 1) * 4)) & 15u : threadIdx.x;
  const uint32_t bin = (gb < static_cast<uint32_t>(nd.sub_lo) || gb >= static_cast<uint32_t>(nd.sub_hi))
                           ? static_cast<uint32_t>(nd.mfb)
                           : gb - nd.sub_lo + nd.offset;
  bool left;
  if (cat) {
    const int word = static_cast<int>(bin >> 5);
    left = word < kMaxCatWords && ((d.cat_bits[word] >> (bin & 31u)) & 1u);
  } else if ((nd.missing_type == 1 && bin == static_cast<uint32_t>(nd.default_bin)) ||
             (nd.missing_type == 2 && bin == static_cast<uint32_t>(nd.max_bin))) {
    left = nd.left_is_default != 0;
  } else {
    left = bin <= nd.threshold;
  }
  const unsigned long long m = __ballot(left);
  if ((threadIdx.x & 63) == 0) bm_work[s * 4 + (threadIdx.x >> 6)] = m;
}

size_t TreeFromRecordsBytes(int max_leaves) {
  const size_t ni = static_cast<size_t>(std::max(1, max_leaves - 1));
  char* base = nullptr;
  const TreeBlob b = BlobLayout(base, max_leaves);
  return static_cast<size_t>(reinterpret_cast<char*>(b.cat_threshold_inner) - base) + 4 * ni * kMaxCatWords;
}

DevTree TreeFromRecords(const KArgs& a, int nsplit, int max_leaves, double shrinkage, char* blob, hipStream_t s,
                        unsigned long long* bm_work, int32_t* bm_meta) {
  if (nsplit < 1 || nsplit > kMaxNodes || nsplit > max_leaves - 1) {
    throw std::runtime_error("TreeFromRecords: split count out of range");
  }
  const TreeBlob b = BlobLayout(blob, max_leaves);
  DevTree t{};
  if (bm_work != nullptr && bm_meta != nullptr && TreeBitmapsApply(a, nsplit + 1)) {
    hipLaunchKernelGGL(k_tree_from_records_bm, dim3(nsplit), dim3(256), 0, s, a, nsplit, shrinkage, b, bm_work, bm_meta);
    t.bm_work = bm_work;
    t.bm_meta = bm_meta;
    t.bm_ready = 1;
  } else {
    hipLaunchKernelGGL(k_tree_from_records, dim3(1), dim3(256), 0, s, a, nsplit, shrinkage, b);
  }
  t.num_leaves = nsplit + 1;
  t.split_feature_inner = b.split_feature_inner;
  t.threshold_in_bin = b.threshold_in_bin;
  t.decision_type = b.decision_type;
  t.left_child = b.left_child;
  t.right_child = b.right_child;
  t.leaf_value = b.leaf_value;
  t.cat_boundaries_inner = b.cat_boundaries_inner;
  t.cat_threshold_inner = b.cat_threshold_inner;
  return t;
}

bool TreeBitmapsApply(const KArgs& a, int num_leaves) {
  const int ni = num_leaves - 1;
  return a.bins != nullptr && a.bin_bytes == 1 && ni >= 1 && ni <= kMaxNodes && a.row_words * 4 <= kBmMaxRowBytes;
}

namespace {
int BmBlocks(int64_t num_rows) {
  // 32 workgroups per CU walk the chunks (LGBM_AMD_BM_WG_PER_CU; 0: one chunk per
  // workgroup).  Headline A/B at 0/4/8/16/32: 4.146/4.135/4.133/4.120/4.109 ms/iter
  static const int per_cu = [] {
    const char* e = tuning::Get(tuning::Knob::BmWgPerCu);
    return e != nullptr ? std::atoi(e) : tuning::kScoreWalkWgPerCu;
  }();
  int64_t blocks64 = (num_rows + kBmRowsPerBlock - 1) / kBmRowsPerBlock;
  if (per_cu > 0) blocks64 = std::min<int64_t>(blocks64, static_cast<int64_t>(per_cu) * NumCUs());
  return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(blocks64, 1 << 30)));
}
}  // namespace

int AddTreeScoreGradParts(int64_t num_rows) { return BmBlocks(num_rows); }

// the objectives whose gradients the score walk computes: L2, L1, Huber, quantile, binary,
// cross-entropy (the others keep the separate gradient kernel)
bool AddTreeScoreGradKind(int kind) {
  return kind == 1 || kind == 2 || kind == 3 || kind == 6 || kind == 10 || kind == 11;
}

void AddTreeScoreGrad(const KArgs& a, const DevTree& t, int64_t num_rows, double* score, const GradArgs& ga,
                      hipStream_t s) {
  const int ni = t.num_leaves - 1;
  if (!t.bm_ready) hipLaunchKernelGGL(k_tree_bitmaps, dim3(ni), dim3(256), 0, s, a, t);
  const size_t lds = sizeof(uint32_t) * kBmRowsPerBlock * a.row_words;
  const dim3 grid(BmBlocks(num_rows)), block(kBmRowsPerBlock);
  auto go = [&](auto kind) {
    constexpr int K = decltype(kind)::value;
    if (a.row_words <= 8) hipLaunchKernelGGL((k_add_tree_score_bm_grad<K, 8>), grid, block, lds, s, a, t, num_rows, score, ga);
    else hipLaunchKernelGGL((k_add_tree_score_bm_grad<K, 16>), grid, block, lds, s, a, t, num_rows, score, ga);
  };
  switch (ga.kind) {
    case 1: go(std::integral_constant<int, 1>()); break;
    case 2: go(std::integral_constant<int, 2>()); break;
    case 3: go(std::integral_constant<int, 3>()); break;
    case 6: go(std::integral_constant<int, 6>()); break;
    case 10: go(std::integral_constant<int, 10>()); break;
    default: go(std::integral_constant<int, 11>()); break;
  }
}

void AddTreeScore(const KArgs& a, const DevTree& t, const int32_t* rows, int64_t num_rows, double* score,
                  hipStream_t s) {
  if (num_rows <= 0) return;
  const int ni = t.num_leaves - 1;
  if (rows == nullptr && TreeBitmapsApply(a, t.num_leaves) && t.bm_work != nullptr) {
    hipLaunchKernelGGL(k_tree_bitmaps, dim3(ni), dim3(256), 0, s, a, t);
    const size_t lds = sizeof(uint32_t) * kBmRowsPerBlock * a.row_words;
    hipLaunchKernelGGL(k_add_tree_score_bm, dim3(BmBlocks(num_rows)), dim3(kBmRowsPerBlock), lds, s, a, t, num_rows,
                       score);
    return;
  }
  // one row per thread: many rows in flight hide the per-row load latency
  const int blocks = static_cast<int>(std::min<int64_t>((num_rows + 255) / 256, 1 << 20));
  if (t.num_leaves - 1 <= kMaxNodes) {
    hipLaunchKernelGGL(k_add_tree_score<true>, dim3(blocks), dim3(256), 0, s, a, t, rows, num_rows, score);
  } else {
    hipLaunchKernelGGL(k_add_tree_score<false>, dim3(blocks), dim3(256), 0, s, a, t, rows, num_rows, score);
  }
}

}  // namespace dev
}  // namespace lgbm_amd
