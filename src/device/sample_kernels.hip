// Row sampling on the device: bagging (reference src/boosting/gbdt.cpp:162-243,
// BaggingHelper) and GOSS (reference src/boosting/goss.hpp:103-179).
//
// The reference draws from one LCG per 1024-row block (bagging_rands_[row / 1024]), so
// bagging is parallel over blocks and bit-identical to the reference: an in-bag decision
// depends only on its block's generator, and the in-bag rows come out in ascending row
// order whatever the reference's partition of the rows into thread blocks.
//
// GOSS selects, per sampling block, the top_rate largest |g * h| and samples the rest with
// a running probability (rest_need / rest_all) -- a sequential chain inside the block.
// The reference's sampling blocks are its thread blocks (ParallelPartitionRunner:
// min(num_threads, ceil(n / 1024)) blocks of a multiple of 1024 rows); here a sampling
// block is one 1024-row generator block, i.e. the reference run with
// num_threads >= ceil(n / 1024).  One wave per block: a radix select of the top_k-th
// largest weight in LDS, then the chain on lane 0 over the block's LDS-resident weights.
//
// Both write a code per row; a one-workgroup scan of the per-block in-bag counts and a
// compaction kernel then write the in-bag rows (ascending) followed by the out-of-bag
// rows -- the layout of GBDT's bag_data_indices_ -- and the in-bag count, on the device.
#include "device_common.h"

namespace lgbm_amd {
namespace dev {

namespace {

constexpr int kBlockRows = kSampleBlockRows;
constexpr int kGossThreads = 64;  // one wave per GOSS block
constexpr int kScanThreads = 1024;

__device__ __forceinline__ float NextFloat(unsigned* x) {
  *x = 214013u * *x + 2531011u;
  return static_cast<float>(static_cast<int>((*x >> 16) & 0x7FFF)) / 32768.0f;
}

// one thread per generator block: the block's LCG decides its rows in order
__global__ __launch_bounds__(256) void k_bag_codes(SampleArgs s) {
  const int64_t b = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x;
  if (b >= s.num_blocks) return;
  unsigned x = s.rng[b];
  const int64_t r0 = b * kBlockRows;
  const int64_t r1 = min(s.num_data, r0 + kBlockRows);
  int cnt = 0;
  for (int64_t r = r0; r < r1; ++r) {
    double frac = s.fraction;
    if (s.balanced) frac = s.label[r] > 0 ? s.pos_fraction : s.neg_fraction;
    const bool in = static_cast<double>(NextFloat(&x)) < frac;
    s.codes[r] = in ? 1 : 0;
    cnt += in ? 1 : 0;
  }
  s.rng[b] = x;
  s.block_cnt[b] = cnt;
}

// codes: 0 out of bag, 1 large gradient, 2 sampled small gradient (rescaled)
__global__ __launch_bounds__(kGossThreads) void k_goss_codes(SampleArgs s) {
  __shared__ float w[kBlockRows];
  __shared__ uint8_t code[kBlockRows];
  __shared__ int hist[256];
  __shared__ uint32_t s_prefix;
  __shared__ int s_k;
  const int64_t b = blockIdx.x;
  const int64_t r0 = b * kBlockRows;
  const int cnt = static_cast<int>(min(s.num_data - r0, static_cast<int64_t>(kBlockRows)));
  const int lane = threadIdx.x;
  for (int i = lane; i < cnt; i += kGossThreads) {
    float v = 0.0f;
    for (int k = 0; k < s.num_class; ++k) {
      const int64_t idx = static_cast<int64_t>(k) * s.num_data + r0 + i;
      v += fabsf(s.grad[idx] * s.hess[idx]);
    }
    w[i] = v;
  }
  const int top_k = max(1, static_cast<int>(cnt * s.top_rate));
  const int other_k = static_cast<int>(cnt * s.other_rate);
  // radix select (8 bits per pass, MSB first) of the top_k-th largest weight; non-negative
  // floats order like their bit patterns
  if (lane == 0) {
    s_prefix = 0u;
    s_k = top_k;
  }
  __syncthreads();
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    for (int i = lane; i < 256; i += kGossThreads) hist[i] = 0;
    __syncthreads();
    const uint32_t prefix = s_prefix;
    const uint32_t pmask = pass == 0 ? 0u : (0xFFFFFFFFu << (32 - 8 * pass));
    for (int i = lane; i < cnt; i += kGossThreads) {
      const uint32_t u = __float_as_uint(w[i]);
      if ((u & pmask) == prefix) atomicAdd(&hist[(u >> shift) & 0xFFu], 1);
    }
    __syncthreads();
    if (lane == 0) {
      int k = s_k;
      int d = 255;
      for (; d > 0; --d) {
        if (hist[d] >= k) break;
        k -= hist[d];
      }
      s_prefix = prefix | (static_cast<uint32_t>(d) << shift);
      s_k = k;
    }
    __syncthreads();
  }
  const float threshold = __uint_as_float(s_prefix);
  __syncthreads();
  if (lane == 0) {
    // the reference's chain (goss.hpp:124-150), in row order
    const float multiply = static_cast<float>(cnt - top_k) / other_k;
    unsigned x = s.rng[b];
    int left = 0, big = 0;
    for (int i = 0; i < cnt; ++i) {
      if (w[i] >= threshold) {
        code[i] = 1;
        ++left;
        ++big;
      } else {
        const int sampled = left - big;
        const int rest_need = other_k - sampled;
        const int rest_all = (cnt - i) - (top_k - big);
        const double prob = rest_need / static_cast<double>(rest_all);
        if (NextFloat(&x) < prob) {
          code[i] = 2;
          ++left;
        } else {
          code[i] = 0;
        }
      }
    }
    s.rng[b] = x;
    s.block_cnt[b] = left;
    s_prefix = __float_as_uint(multiply);
  }
  __syncthreads();
  const float multiply = __uint_as_float(s_prefix);
  for (int i = lane; i < cnt; i += kGossThreads) {
    const uint8_t c = code[i];
    s.codes[r0 + i] = c;
    if (c == 2) {
      for (int k = 0; k < s.num_class; ++k) {
        const int64_t idx = static_cast<int64_t>(k) * s.num_data + r0 + i;
        s.grad[idx] *= multiply;
        s.hess[idx] *= multiply;
      }
    }
  }
}

// exclusive scan of the per-block in-bag counts (one workgroup, chunks of 1024 blocks);
// the total goes to *bag_count
__global__ __launch_bounds__(kScanThreads) void k_scan_blocks(SampleArgs s) {
  __shared__ int sh[kScanThreads / kWave];
  __shared__ int carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
  for (int64_t base = 0; base < s.num_blocks; base += kScanThreads) {
    const int64_t i = base + threadIdx.x;
    const int v = i < s.num_blocks ? s.block_cnt[i] : 0;
    int incl = v;
    for (int o = 1; o < kWave; o <<= 1) {
      const int t = __shfl_up(incl, o, kWave);
      if (lane >= o) incl += t;
    }
    if (lane == kWave - 1) sh[wv] = incl;
    __syncthreads();
    int woff = 0, total = 0;
    for (int k = 0; k < kScanThreads / kWave; ++k) {
      woff += k < wv ? sh[k] : 0;
      total += sh[k];
    }
    const int c = carry;
    if (i < s.num_blocks) s.block_off[i] = c + woff + incl - v;
    __syncthreads();
    if (threadIdx.x == 0) carry = c + total;
    __syncthreads();
  }
  if (threadIdx.x == 0) *s.bag_count = carry;
}

// the rows of one generator block -> the in-bag list (ascending) and the out-of-bag list
__global__ __launch_bounds__(kBlockRows) void k_bag_compact(SampleArgs s) {
  __shared__ int wsum[kBlockRows / kWave];
  const int64_t b = blockIdx.x;
  const int64_t r = b * kBlockRows + threadIdx.x;
  const bool valid = r < s.num_data;
  const bool in = valid && s.codes[r] != 0;
  const unsigned long long m = __ballot(in);
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
  const int before = __popcll(m & ((1ull << lane) - 1ull));
  if (lane == 0) wsum[wv] = __popcll(m);
  __syncthreads();
  int woff = 0;
  for (int k = 0; k < wv; ++k) woff += wsum[k];
  if (!valid) return;
  const int in_off = s.block_off[b];  // in-bag rows of the earlier blocks
  const int local_in = woff + before;
  if (in) {
    s.bag[in_off + local_in] = static_cast<int32_t>(r);
  } else {
    const int64_t out_before = b * kBlockRows - in_off;  // out-of-bag rows of the earlier blocks
    s.oob[out_before + (threadIdx.x - local_in)] = static_cast<int32_t>(r);
  }
}

}  // namespace

int SampleBlocks(int64_t n) { return static_cast<int>((n + kBlockRows - 1) / kBlockRows); }

void SampleRows(const SampleArgs& s, hipStream_t st) {
  if (s.num_data <= 0) return;
  if (s.goss) {
    hipLaunchKernelGGL(k_goss_codes, dim3(static_cast<unsigned>(s.num_blocks)), dim3(kGossThreads), 0, st, s);
  } else {
    hipLaunchKernelGGL(k_bag_codes, dim3(static_cast<unsigned>((s.num_blocks + 255) / 256)), dim3(256), 0, st, s);
  }
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(kScanThreads), 0, st, s);
  hipLaunchKernelGGL(k_bag_compact, dim3(static_cast<unsigned>(s.num_blocks)), dim3(kBlockRows), 0, st, s);
}

}  // namespace dev
}  // namespace lgbm_amd
