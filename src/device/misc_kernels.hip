// Small per-tree kernels of the MI355X learner: gradient packing + fixed-point scale
// selection, tree reset, root statistics and score arithmetic.
#include <algorithm>
#include <stdexcept>

#include "device_common.h"
#include "lgbm_amd/tuning.h"

namespace lgbm_amd {
namespace dev {

namespace {
int g_num_cus = 256;
}  // namespace

int NumCUs() { return g_num_cus; }

void SetNumCUs(int n) { g_num_cus = n > 0 ? n : 256; }
int HistGridBlocks() {
  static const int per_cu = [] {  // LGBM_AMD_ROOT_WG_PER_CU (A/B knob; default 2)
    const char* e = tuning::Get(tuning::Knob::RootWgPerCu);
    return e != nullptr && std::atoi(e) > 0 ? std::atoi(e) : tuning::kRootWgPerCu;
  }();
  return per_cu * g_num_cus;
}

// ---------------------------------------------------------------- gradient packing
// (g, h) interleaved so a gathered row costs one 8-byte load; also the per-workgroup max|g|
// / max h of the tree (reduced by k_reduce_parts: no contended atomics)
__global__ __launch_bounds__(256) void k_pack_gh(const float* __restrict__ g, const float* __restrict__ h,
                                                 float2* __restrict__ gh, int64_t stride, int64_t n, float* max_parts) {
  float mg = 0.f, mh = 0.f;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const float a = g[i], b = h[i];
    gh[i * stride] = make_float2(a, b);
    mg = fmaxf(mg, fabsf(a));
    mh = HessMax(mh, b);
  }
  for (int o = 32; o > 0; o >>= 1) {
    mg = fmaxf(mg, __shfl_xor(mg, o, kWave));
    mh = HessMax(mh, __shfl_xor(mh, o, kWave));
  }
  __shared__ float smg[4], smh[4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    smg[w] = mg;
    smh[w] = mh;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < static_cast<int>(blockDim.x >> 6); ++i) {
      mg = fmaxf(mg, smg[i]);
      mh = HessMax(mh, smh[i]);
    }
    max_parts[2 * blockIdx.x] = mg;
    max_parts[2 * blockIdx.x + 1] = mh;
  }
}

int PackBlocks(int64_t n) {
  return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4 * NumCUs())));
}

void PackGH(const float* g, const float* h, GH* gh, int64_t gh_stride, int64_t n, float* max_parts, hipStream_t s) {
  hipLaunchKernelGGL(k_pack_gh, dim3(PackBlocks(n)), dim3(256), 0, s, g, h, reinterpret_cast<float2*>(gh), gh_stride, n,
                     max_parts);
}

// scale = 2^k per component.  Packed (units 1): rows_cap * max * scale <= 2^30 (g: signed
// high half of the packed word) and <= 2^31 (h: low half; 2^30 when absmax[3] flags a negative
// hessian, see UnpackPartial) -- a row block never holds more than rows_cap rows.  Wide (units 2): max * scale <= 2^31, so each row keeps 31 bits of
// max |g| (every fp32 gradient within 2^-7 of the maximum exactly) and sums over up to 2^31
// rows stay inside int64.  absmax[2] (if set) carries the row cap of all ranks.
__global__ void k_scales(const uint32_t* absmax, int rows_cap, int units, double* scales) {
  if (threadIdx.x != 0) return;
  const uint32_t am[4] = {absmax[0], absmax[1], absmax[2], absmax[3]};
  ScalesFromAbsmax(am, rows_cap, units, scales);
}

void ComputeScales(const uint32_t* absmax, int rows_cap, int units, double* scales, hipStream_t s) {
  hipLaunchKernelGGL(k_scales, dim3(1), dim3(64), 0, s, absmax, rows_cap, units, scales);
}

// ---------------------------------------------------------------- tree reset
// Every workgroup zeroes its share of `zero` (the histogram scratch of the tree's first step or
// round) and block 0 also copies the tree's feature mask from fine-grained host memory:
// kernel work instead of memset / memcpy graph nodes, whose boundaries stalled the graph
// (~10-30 us each, profiles/r05_round_latency_ab.md).
__global__ void k_tree_begin(KArgs a, unsigned long long* zero, int64_t zero_words, const int8_t* mask_host, int nmask) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < zero_words;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    zero[i] = 0ull;
  }
  if (blockIdx.x != 0) return;
  for (int f = threadIdx.x; mask_host != nullptr && f < nmask; f += blockDim.x) {
    const_cast<int8_t*>(a.tree_mask)[f] = mask_host[f];
  }
  const int L = a.p.num_leaves;
  for (int l = threadIdx.x; l < L; l += blockDim.x) {
    Leaf lf;
    // splittable rows persist across trees; round growth hands out fresh rows from 0 (the root)
    lf.frow = a.rd != nullptr ? (l == 0 ? 0 : -1) : a.leaves[l].frow;
    lf.pad = 0;
    lf.begin = 0;
    lf.count = l == 0 ? RootRows(a) : 0;
    lf.global_count = lf.count;
    lf.depth = 0;
    lf.slot = l;
    lf.buf = 0;
    lf.sum_g = lf.sum_h = lf.output = 0.0;
    lf.lsum_g = lf.lsum_h = 0.0;
    lf.cmin = -DBL_MAX;
    lf.cmax = DBL_MAX;
    lf.icmask = kIcAll;  // the root may use every constraint
    a.leaves[l] = lf;
    a.best[l].gain = -INFINITY;
    a.best[l].feature = -1;
    a.best[l].real_feature = -1;
  }
  if (threadIdx.x == 0) {
    Step* st = a.st;
    st->done = 0;
    st->nsplit = 0;
    st->fresh = 1;  // the root's per-feature results (k_find<true>) are the first pick's input
    st->bynode_base = 0;
    st->bynode_next = 1;  // mask 0: the root
    st->smaller = 0;
    st->larger = -1;
    st->hist_left = 1;
    st->find_count = 0u;
    for (int i = 0; i < kFindSub; ++i) a.find_sub[i * kFindSubStride] = 0u;
    st->loc_acc[0] = st->loc_acc[1] = 0ull;
    st->root_count = 0;
    st->cur_left = st->cur_right = 0;
    st->forced_abort = 0;
    if (a.rd != nullptr) {
      Round* rd = a.rd;
      rd->done = 0;
      rd->nsplit = 0;
      rd->nexp = 0;
      rd->round = 0;
      rd->rpb = 0;
      rd->nblk = 0;
      rd->next_slot = 1;  // slot 0: the root
      rd->next_frow = 1;  // row 0: the root
      rd->rounds = 0;
      rd->accepted_max = 0;
      rd->child_done = 0u;
      rd->bynode_next = 1;  // (per-node sampling on round growth: draw 0 is the root's)
    }
  }
  for (int k = threadIdx.x; k < a.forced_n; k += blockDim.x) {  // no stale forced results
    a.forced_best[k].gain = -INFINITY;
    a.forced_best[k].feature = -1;
  }
}

void TreeBegin(const KArgs& a, hipStream_t s, void* zero, size_t zero_bytes, const int8_t* mask_host, int nmask) {
  const int64_t words = static_cast<int64_t>(zero_bytes / 8);
  if (zero_bytes % 8 != 0) throw std::runtime_error("TreeBegin: the zeroed range is not in 8-byte words");
  const int blocks = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(2 * NumCUs(), (words + 2047) / 2048)));
  hipLaunchKernelGGL(k_tree_begin, dim3(blocks), dim3(256), 0, s, a, static_cast<unsigned long long*>(zero), words,
                     mask_host, nmask);
}

__global__ __launch_bounds__(256) void k_root_sum(KArgs a) {
  __shared__ double sh[8];
  double sg = 0.0, shh = 0.0;
  const int n = RootRows(a);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int r = a.root_identity ? i : a.idx[i];
    const float2 v = GhAt(a, r);
    sg += v.x;
    shh += v.y;
  }
  sg = BlockSum(sg, sh);
  shh = BlockSum(shh, sh);
  if (threadIdx.x == 0) {
    a.root_blk[2 * blockIdx.x] = sg;
    a.root_blk[2 * blockIdx.x + 1] = shh;
  }
}

// the workgroups' partials summed in a fixed order: the same sums on every run (float atomics
// across workgroups would add in arrival order)
__global__ __launch_bounds__(256) void k_root_finish(KArgs a, int nblk) {
  __shared__ double sh[8];
  double sg = 0.0, shh = 0.0;
  for (int b = threadIdx.x; b < nblk; b += blockDim.x) {
    sg += a.root_blk[2 * b];
    shh += a.root_blk[2 * b + 1];
  }
  sg = BlockSum(sg, sh);
  shh = BlockSum(shh, sh);
  if (threadIdx.x == 0) {
    a.root[0] = sg;
    a.root[1] = shh;
    a.root[2] = static_cast<double>(RootRows(a));
  }
}

int RootSumBlocks() { return 2 * NumCUs(); }

void RootSum(const KArgs& a, hipStream_t s) {
  const int blocks = std::max(1, std::min((a.num_rows + 255) / 256, RootSumBlocks()));
  hipLaunchKernelGGL(k_root_sum, dim3(blocks), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_root_finish, dim3(1), dim3(256), 0, s, a, blocks);
}

// ---------------------------------------------------------------- elementwise
__global__ void k_add_const(double* s, int64_t n, double v) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    s[i] += v;
}
__global__ void k_mul_const(double* s, int64_t n, double v) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    s[i] *= v;
}
__global__ void k_iota(int32_t* p, int64_t n) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    p[i] = static_cast<int32_t>(i);
}

template <typename T, int OP>
__global__ void k_reduce_peers(PeerBufs src, int n, size_t offset, T* out, size_t count) {
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < count;
       i += static_cast<size_t>(gridDim.x) * blockDim.x) {
    T v = static_cast<const T*>(src.p[0])[offset + i];
    for (int r = 1; r < n; ++r) {
      const T x = static_cast<const T*>(src.p[r])[offset + i];
      v = OP == 3 ? (x > v ? x : v) : v + x;
    }
    out[i] = v;
  }
}

void ReducePeers(const PeerBufs& src, int n, size_t offset, void* out, size_t count, int op, hipStream_t s) {
  const int grid = GridFor(static_cast<int64_t>(count));
  switch (op) {
    case kPeerSumF64:
      hipLaunchKernelGGL((k_reduce_peers<double, 0>), dim3(grid), dim3(256), 0, s, src, n, offset,
                         static_cast<double*>(out), count);
      break;
    case kPeerSumF32:
      hipLaunchKernelGGL((k_reduce_peers<float, 0>), dim3(grid), dim3(256), 0, s, src, n, offset,
                         static_cast<float*>(out), count);
      break;
    case kPeerSumI64:
      hipLaunchKernelGGL((k_reduce_peers<long long, 0>), dim3(grid), dim3(256), 0, s, src, n, offset,
                         static_cast<long long*>(out), count);
      break;
    default:
      hipLaunchKernelGGL((k_reduce_peers<uint32_t, 3>), dim3(grid), dim3(256), 0, s, src, n, offset,
                         static_cast<uint32_t*>(out), count);
      break;
  }
}

void Iota(int32_t* p, int64_t n, hipStream_t s) { hipLaunchKernelGGL(k_iota, dim3(GridFor(n)), dim3(256), 0, s, p, n); }
void AddConst(double* score, int64_t n, double v, hipStream_t s) {
  hipLaunchKernelGGL(k_add_const, dim3(GridFor(n)), dim3(256), 0, s, score, n, v);
}
void MulConst(double* score, int64_t n, double v, hipStream_t s) {
  hipLaunchKernelGGL(k_mul_const, dim3(GridFor(n)), dim3(256), 0, s, score, n, v);
}

}  // namespace dev
}  // namespace lgbm_amd
