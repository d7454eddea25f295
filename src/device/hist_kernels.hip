// Histogram construction (reference: the GPU learner's histogram256 OpenCL kernel and
// DenseBin::ConstructHistogram, src/treelearner/ocl/histogram256.cl, src/io/dense_bin.hpp).
//
// Layout: row-major bin matrix (one 32-bit word = 4 uint8 or 2 uint16 storage columns).
// Grid: (row blocks, column tiles) of 1024-thread workgroups.  A workgroup accumulates a
// LDS-private histogram of its tile's columns over its block of the leaf's rows and stores
// it whole as a partial histogram -- no global atomics (on gfx950 those execute at the
// memory side; a per-workgroup atomic flush of a 7K-bin tile took ~22 us).  k_hist_reduce
// then sums the partials of every bin into the step's int64 histogram.
//
// Accumulation is fixed point: (g * scale_g, h * scale_h) rounded to integers and packed
// into one uint64 (g in the signed high half, h in the low half) -> one ds_add_u64 per
// row and feature.  ds_add_f32 runs at ~0.33 lane-ops/CU/clk on gfx950, ds_add_u64 at ~5
// (tools/microbench/lds_atomics.hip); the scale (k_scales) leaves headroom for the largest
// per-workgroup row count so the 32-bit halves never overflow, and global sums are int64
// (exact, deterministic regardless of the row order, and summable across ranks with RCCL).
#include "device_common.h"

namespace lgbm_amd {
namespace dev {

namespace {

constexpr int kRowsInFlight = 8;  // independent row gathers per thread

__device__ __forceinline__ unsigned long long PackFixed(float2 v, float sg, float sh) {
  const long long gq = __float2ll_rn(v.x * sg);
  const long long hq = __float2ll_rn(v.y * sh);
  return (static_cast<unsigned long long>(gq) << 32) + static_cast<unsigned long long>(hq);
}

// Group bin 0 holds every row whose features all sit in their most frequent bin: it is
// outside every feature's histogram range (bin_offsets start at 1) and is restored by
// FixHistogram, so it is never accumulated (this also skips most rows of sparse columns).
template <int GPW>
__device__ __forceinline__ void AddRow(unsigned long long* lds, const int* goff, uint32_t w, unsigned long long pk) {
#pragma unroll
  for (int j = 0; j < GPW; ++j) {
    const uint32_t b = GPW == 4 ? ((w >> (8 * j)) & 0xffu) : ((w >> (16 * j)) & 0xffffu);
    if (goff[j] >= 0 && b != 0u) atomicAdd(&lds[goff[j] + b], pk);
  }
}

// rows of the histogram: MODE 0 root, 1 smaller child of the step, 2 explicit range.
// MODE 1 derives them from the partition's result (StepChildren); the reduce kernel (MODE
// 1, after the histogram kernel's bookkeeping) passes from_step to read the stored copy.
template <int MODE>
__device__ __forceinline__ bool HistRows(const KArgs& a, bool from_step, int* begin, int* count,
                                         const int32_t** src) {
  if (MODE == 0) {
    *begin = 0;
    *count = RootRows(a);
    *src = a.root_identity ? nullptr : a.idx;
  } else if (MODE == 2) {
    *begin = a.range_begin;
    *count = a.num_rows;
    *src = a.idx;
  } else {
    const Step* st = a.st;
    if (st->done) return false;
    if (from_step) {
      if (st->skip_find) return false;
      *begin = st->s_begin;
      *count = st->s_count;
      *src = st->s_buf ? a.tmp : a.idx;
    } else {
      const ChildInfo c = StepChildren(a, st);
      if (c.skip) return false;
      *begin = c.s_begin;
      *count = c.s_count;
      *src = c.buf ? a.tmp : a.idx;
    }
  }
  return *count > 0;
}

// the step's bookkeeping (one thread of the histogram kernel): children ranges and counts,
// histogram-slot hand-over to the larger child, split records, best[] reset, and the
// smaller / larger children's records for the split scans
__device__ void StepBookkeeping(const KArgs& a, Step* st) {
  const ChildInfo c = StepChildren(a, st);
  const CurSplit& cs = st->cs;
  const int leaf = cs.leaf, nl = cs.new_leaf;
  const int pb = cs.part_begin, pc = cs.part_count;
  Leaf* P = &a.leaves[leaf];
  Leaf* R = &a.leaves[nl];
  P->begin = pb;
  P->count = c.total_left;
  R->begin = pb + c.total_left;
  R->count = pc - c.total_left;
  P->buf = c.buf;
  R->buf = c.buf;
  if (!a.p.data_parallel) {
    P->global_count = c.left_count;
    R->global_count = c.right_count;
    SplitRecord& rec = a.rec[cs.s];
    rec.left_count = c.left_count;
    rec.right_count = c.right_count;
  }
  const bool swap = !c.skip && c.small_is_left;
  if (swap) {
    // the parent's histogram stays with the larger (right) child
    P->slot = nl;
    R->slot = cs.parent_slot;
    P->frow = cs.new_frow;  // the splittable rows follow (the host swaps its rows too)
    R->frow = cs.parent_frow;
  }
  // smaller / larger child records for the split scans (field-wise: no private copies)
  for (int k = 0; k < 2; ++k) {
    const int lr = (k == 0) == (c.small_is_left != 0) ? 0 : 1;  // k: 0 smaller, 1 larger
    const ChildStats& from = st->lr[lr];
    ChildStats& to = st->child[k];
    to.sum_g = from.sum_g;
    to.sum_h = from.sum_h;
    to.output = from.output;
    to.cmin = from.cmin;
    to.cmax = from.cmax;
    to.depth = from.depth;
    to.leaf = from.leaf;
    to.global_count = a.p.data_parallel ? from.global_count : (lr == 0 ? c.left_count : c.right_count);
    to.slot = swap ? (lr == 0 ? nl : cs.parent_slot) : from.slot;
    to.frow = k == 0 ? cs.new_frow : cs.parent_frow;  // the larger child inherits the parent's row
    to.icmask = from.icmask;
  }
  a.best[leaf].gain = -INFINITY;
  a.best[leaf].feature = -1;
  a.best[leaf].real_feature = -1;
  a.best[nl].gain = -INFINITY;
  a.best[nl].feature = -1;
  a.best[nl].real_feature = -1;
  st->smaller = c.smaller;
  st->larger = c.larger;
  st->skip_find = c.skip;
  if (!c.skip) {  // the host learner samples the smaller, then the larger child
    st->bynode_base = st->bynode_next;
    st->bynode_next += 2;
  }
  st->total_left = c.total_left;
  st->s_begin = c.s_begin;
  st->s_count = c.s_count;
  st->s_buf = c.buf;
  st->fresh = c.skip ? 0 : 2;
  st->nsplit = cs.s + 1;
}

}  // namespace

// per-thread constants of a column tile (one 32-bit word of a row per thread)
struct TileCtx {
  int w0, w1, lo_bin, nbins;
  int tpr, rpp, q, rs;  // threads per row, rows per pass, my word, my row slot
  int goff[4];          // histogram offset of each group of my word (-1: none)
  float sg, sh;         // fixed-point scales
};

template <int MODE>
__device__ __forceinline__ void LoadRowIdx(const int32_t* src, int i, int r1, int rpp, int* r) {
#pragma unroll
  for (int k = 0; k < kRowsInFlight; ++k) {
    const int ii = i + k * rpp;
    r[k] = ii < r1 ? (src ? src[ii] : ii) : -1;
  }
}

// one row block [r0, r1) of one column tile -> its partial histogram `out`.  The index
// loads of each batch are issued one batch ahead (the first ones while the LDS is cleared).
template <int MODE, int GPW>
__device__ __forceinline__ void HistBlock(const KArgs& a, unsigned long long* lds, const int32_t* src, int r0, int r1,
                                          const TileCtx& t, unsigned long long* out, int ts) {
  const bool active = t.rs < t.rpp;
  int i = r0 + t.rs;
  int r[kRowsInFlight];
  if (active) LoadRowIdx<MODE>(src, i, r1, t.rpp, r);
  __syncthreads();  // LDS reuse across row blocks
  for (int j = threadIdx.x; j < t.nbins; j += kHistThreads) lds[j] = 0ull;
  __syncthreads();
  KTrace(a, blockIdx.x == 0 ? ts : -1, kTrHistZeroed);
  if (active) {
    const int w = t.w0 + t.q;
    const uint32_t* bins32 = static_cast<const uint32_t*>(a.bins);
    const float2* gh = reinterpret_cast<const float2*>(a.gh);
    const int64_t wpr = a.words_per_row;
    const bool write_iota = MODE == 0 && src == nullptr && t.q == 0 && blockIdx.y == 0;
    const int stride = kRowsInFlight * t.rpp;
    for (; i < r1; i += stride) {
      if (i == r0 + t.rs) KTrace(a, blockIdx.x == 0 ? ts : -1, kTrHistIdx);
      if (write_iota) {
#pragma unroll
        for (int k = 0; k < kRowsInFlight; ++k) {
          if (r[k] >= 0) a.idx[i + k * t.rpp] = r[k];
        }
      }
      float2 v[kRowsInFlight];
      uint32_t wd[kRowsInFlight];
#pragma unroll
      for (int k = 0; k < kRowsInFlight; ++k) {
        const int rr = r[k] >= 0 ? r[k] : 0;
        v[k] = gh[rr];
        wd[k] = r[k] >= 0 ? bins32[rr * wpr + w] : 0u;  // word 0: every bin skipped
      }
      int rn[kRowsInFlight];
      LoadRowIdx<MODE>(src, i + stride, r1, t.rpp, rn);  // next batch, in flight during the atomics
      if (i == r0 + t.rs) KTrace(a, blockIdx.x == 0 ? ts : -1, kTrHistLoaded);
#pragma unroll
      for (int k = 0; k < kRowsInFlight; ++k) AddRow<GPW>(lds, t.goff, wd[k], PackFixed(v[k], t.sg, t.sh));
#pragma unroll
      for (int k = 0; k < kRowsInFlight; ++k) r[k] = rn[k];
    }
  }
  __syncthreads();
  KTrace(a, blockIdx.x == 0 ? ts : -1, kTrHistAccum);
  for (int j = threadIdx.x; j < t.nbins; j += kHistThreads) out[j] = lds[j];
}

template <int MODE, int GPW>
__global__ __launch_bounds__(kHistThreads) void k_hist(KArgs a) {
  extern __shared__ unsigned long long lds[];
  const long long t_entry = wall_clock64();
  // ---- every load that does not depend on another one first (a single round trip):
  // tile geometry, scales and the Step record (read before it is tested)
  TileCtx t;
  t.w0 = blockIdx.y * a.tile_words;
  t.w1 = min(a.words_per_row, t.w0 + a.tile_words);
  const int g0 = t.w0 * GPW;
  const int g_end = min(a.p.num_groups, t.w1 * GPW);
  t.tpr = t.w1 - t.w0;
  t.rpp = kHistThreads / t.tpr;
  t.q = threadIdx.x % t.tpr;
  t.rs = threadIdx.x / t.tpr;
  const int w = t.w0 + t.q;
  int graw[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int g = w * GPW + j;
    graw[j] = (j < GPW && g < a.p.num_groups) ? a.group_off[g] : -1;
  }
  t.lo_bin = a.group_off[g0];
  const int hi_bin = g_end < a.p.num_groups ? a.group_off[g_end] : a.p.total_bins;
  t.sg = static_cast<float>(a.scales[0]);
  t.sh = static_cast<float>(a.scales[1]);
  int begin = 0, count = 0, ts = -1;
  const int32_t* src = nullptr;
  if (MODE == 0) {
    count = RootRows(a);
    src = a.root_identity ? nullptr : a.idx;
  } else if (MODE == 2) {
    begin = a.range_begin;
    count = a.num_rows;
    src = a.idx;
  } else {
    Step* st = a.st;
    const int done = st->done;
    const ChildInfo c = StepChildren(a, st);
    ts = st->cs.s;
    if (done) return;
    // bookkeeping by the last workgroup: small leaves leave it without row work
    if (blockIdx.x == gridDim.x - 1 && blockIdx.y == 0 && threadIdx.x == 0) StepBookkeeping(a, st);
    if (c.skip) return;
    begin = c.s_begin;
    count = c.s_count;
    src = c.buf ? a.tmp : a.idx;
  }
  if (count <= 0) return;
  if ((threadIdx.x & 63) == 0 && a.ktrace != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && ts >= 0 &&
      ts < a.p.num_leaves) {
    a.ktrace[ts * kTraceSlots + kTrHistWave0 + (threadIdx.x >> 6)] = t_entry;
  }
  t.nbins = hi_bin - t.lo_bin;
#pragma unroll
  for (int j = 0; j < 4; ++j) t.goff[j] = graw[j] >= 0 ? graw[j] - t.lo_bin : -1;
  KTraceAt(a, ts, kTrHistEntry, t_entry);
  KTrace(a, ts, kTrHistRows);
  const int nblk = HistBlocksFor(count, a.hist_max_blocks, a.hist_rows_cap);
  const int chunk = (count + nblk - 1) / nblk;
  // the grid is one workgroup per CU (per tile); row blocks beyond it are strided
  for (int kb = blockIdx.x; kb < nblk; kb += gridDim.x) {
    HistBlock<MODE, GPW>(a, lds, src, begin + kb * chunk, min(begin + count, begin + kb * chunk + chunk), t,
                         a.partials + static_cast<size_t>(kb) * a.p.total_bins + t.lo_bin, ts);
  }
  KTrace(a, ts, kTrHistExit);
}

// partials [block][bin] -> int64 (g, h) pairs of the step's buffer.  Each thread sums up to
// kReduceChunk partials of one bin; with more blocks than that the chunks are combined by
// int64 atomics into the (pre-zeroed) buffer, otherwise the single chunk stores directly.
template <int MODE>
__global__ __launch_bounds__(256) void k_hist_reduce(KArgs a) {
  const long long t_entry = wall_clock64();
  const int ts = MODE == 1 && !a.st->done ? a.st->cs.s : -1;
  KTraceAt(a, ts, kTrRedEntry, t_entry);
  if (MODE == 1 && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    // the partition cursors are final (read by the histogram kernel): reset for the next split
    a.st->cur_left = 0;
    a.st->cur_right = 0;
  }
  int begin, count;
  const int32_t* src;
  if (!HistRows<MODE>(a, true, &begin, &count, &src)) return;
  const int nblk = HistBlocksFor(count, a.hist_max_blocks, a.hist_rows_cap);
  if (MODE == 1 && DirectPartials(a, nblk, a.st->cs.s)) {  // summed by the split scan
    KTrace(a, ts, kTrRedExit);
    return;
  }
  const int k0 = blockIdx.y * kReduceChunk;
  if (k0 >= nblk) return;
  const int bin = blockIdx.x * blockDim.x + threadIdx.x;
  const int nb = a.p.total_bins;
  if (bin >= nb) return;
  const unsigned long long* p = a.partials + static_cast<size_t>(k0) * nb + bin;
  const int kn = min(kReduceChunk, nblk - k0);
  unsigned long long v[kReduceChunk];
#pragma unroll
  for (int k = 0; k < kReduceChunk; ++k) v[k] = k < kn ? p[static_cast<size_t>(k) * nb] : 0ull;
  long long g = 0, h = 0;
#pragma unroll
  for (int k = 0; k < kReduceChunk; ++k) {
    g += static_cast<long long>(v[k]) >> 32;  // h (low half) is non-negative: no borrow
    h += static_cast<long long>(v[k] & 0xffffffffull);
  }
  long long* out = MODE == 1 ? StepScratch(a, a.st->cs.s + 1) : a.scratch;
  if (nblk <= kReduceChunk) {
    out[2 * bin] = g;
    out[2 * bin + 1] = h;
  } else {
    atomicAdd(reinterpret_cast<unsigned long long*>(&out[2 * bin]), static_cast<unsigned long long>(g));
    atomicAdd(reinterpret_cast<unsigned long long*>(&out[2 * bin + 1]), static_cast<unsigned long long>(h));
  }
  KTrace(a, ts, kTrRedExit);
}

template <int MODE>
static void LaunchHistMode(const KArgs& a, int grid_x, hipStream_t s, bool reduce = true) {
  const size_t lds_bytes = sizeof(unsigned long long) * static_cast<size_t>(a.tile_bins);
  dim3 grid(grid_x, a.hist_tiles);
  if (a.bin_bytes == 1) {
    hipLaunchKernelGGL((k_hist<MODE, 4>), grid, dim3(kHistThreads), lds_bytes, s, a);
  } else {
    hipLaunchKernelGGL((k_hist<MODE, 2>), grid, dim3(kHistThreads), lds_bytes, s, a);
  }
  if (!reduce) return;
  dim3 rgrid((a.p.total_bins + 255) / 256, (a.hist_max_blocks + kReduceChunk - 1) / kReduceChunk);
  hipLaunchKernelGGL(k_hist_reduce<MODE>, rgrid, dim3(256), 0, s, a);
}

// the root fills the chip (two workgroups per CU); a step's leaf is usually small, and
// dispatching workgroups that exit at once is not free (~3 us for 512 x 1024 threads)
void HistRoot(const KArgs& a, hipStream_t s) { LaunchHistMode<0>(a, a.hist_max_blocks, s); }
void HistStep(const KArgs& a, hipStream_t s, bool reduce) {
  LaunchHistMode<1>(a, std::min(a.hist_max_blocks, NumCUs()), s, reduce);
}
void HistRange(const KArgs& a, hipStream_t s) { LaunchHistMode<2>(a, a.hist_max_blocks, s); }

}  // namespace dev
}  // namespace lgbm_amd
