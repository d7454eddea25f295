// Feature binning of dense matrices on the device (reference include/LightGBM/bin.h:132
// BinMapper::ValueToBin, applied per value by Dataset::PushOneRow / FeatureGroup::PushData).
// The bin mappers themselves are found on the host from a row sample (bin.cpp FindBin); this
// maps every value of the matrix to its group bin with them:
//   k_value_to_bin   one thread per (row, slice of groups): for each group, its numerical
//                    features in ascending column order -- the value as double, NaN to the
//                    NaN bin (or 0.0), the binary search over the upper bounds, the most
//                    frequent bin skipped, the group offset added (a later non-default member
//                    of an EFB bundle overwrites an earlier one, as the host's column loop)
// Rows stream through in chunks (one H2D copy of the chunk's values, one D2H copy per group
// column).  Groups with a categorical member stay on the host (category hash map).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "lgbm_amd/dataset.h"
#include "lgbm_amd/device_binning.h"
#include "lgbm_amd/log.h"
#include "lgbm_amd/tuning.h"

namespace lgbm_amd {

namespace {

#define BINCHECK(x)                                                                                   \
  do {                                                                                                \
    hipError_t e_ = (x);                                                                              \
    if (e_ != hipSuccess) Log::Fatal("HIP error %s at %s:%d: %s", #x, __FILE__, __LINE__, hipGetErrorString(e_)); \
  } while (0)

struct BinFeat {
  int col;      // real column in the matrix
  int hi;       // search range [0, hi): num_bin - 1, minus the NaN bin
  int nan_bin;  // NaN -> this bin (missing_type NaN), or -1: NaN -> 0.0
  int mfb;      // most frequent bin (not stored)
  int ub_off;   // upper bounds at ub[ub_off ...]
  uint32_t goff;  // group bin of the feature's bin 1 (its bin_offsets entry)
};

struct BinGroup {
  int fbegin, fend;  // features [fbegin, fend) in ascending column order
  int bytes;         // 1, 2 or 4 per row
  int pad;
  long long out_off;  // byte offset of the group's column in the chunk output
};

constexpr int kBinThreads = 256;
constexpr int kGroupsPerThread = 8;
constexpr int kBinLdsDoubles = 6144;  // 48 KiB of staged upper bounds per workgroup

template <typename T>
__global__ __launch_bounds__(kBinThreads) void k_value_to_bin(const T* x, int rows, long long rs, long long cs,
                                                              const BinGroup* groups, int ngroups,
                                                              const BinFeat* feats, const double* ub,
                                                              uint8_t* out) {
  // the slice's upper bounds staged in LDS when they fit (the binary search is a chain of
  // dependent loads: from L2 it took ~0.85 ms per 2.4M x 28 chunk)
  extern __shared__ double s_ub[];
  const int g0 = blockIdx.y * kGroupsPerThread, g1 = min(ngroups, g0 + kGroupsPerThread);
  const int ub_lo = feats[groups[g0].fbegin].ub_off;
  const int ub_n = g1 > g0 ? feats[groups[g1 - 1].fend - 1].ub_off + feats[groups[g1 - 1].fend - 1].hi + 1 - ub_lo : 0;
  const bool staged = ub_n <= kBinLdsDoubles;
  if (staged) {
    for (int j = threadIdx.x; j < ub_n; j += kBinThreads) s_ub[j] = ub[ub_lo + j];
    __syncthreads();
  }
  const int r = blockIdx.x * kBinThreads + threadIdx.x;
  if (r >= rows) return;
  const T* xr = x + rs * r;
  for (int g = g0; g < g1; ++g) {
    const BinGroup G = groups[g];
    uint32_t v = 0;
    for (int f = G.fbegin; f < G.fend; ++f) {
      const BinFeat F = feats[f];
      double value = static_cast<double>(xr[cs * F.col]);
      int bin;
      if (isnan(value) && F.nan_bin >= 0) {
        bin = F.nan_bin;
      } else {
        if (isnan(value)) value = 0.0;
        const double* u = staged ? s_ub + (F.ub_off - ub_lo) : ub + F.ub_off;
        int lo = 0, hi = F.hi;
        while (lo < hi) {
          const int mid = (lo + hi - 1) / 2;
          if (value <= u[mid]) hi = mid;
          else lo = mid + 1;
        }
        bin = lo;
      }
      if (bin == F.mfb) continue;
      if (F.mfb == 0) bin -= 1;
      v = static_cast<uint32_t>(bin) + F.goff;
    }
    uint8_t* o = out + G.out_off;
    if (G.bytes == 1) o[r] = static_cast<uint8_t>(v);
    else if (G.bytes == 2) reinterpret_cast<uint16_t*>(o)[r] = static_cast<uint16_t>(v);
    else reinterpret_cast<uint32_t*>(o)[r] = v;
  }
}

int BinningDevice(const Config& cfg) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
    (void)hipGetLastError();
    return -1;
  }
  if (cfg.gpu_device_id >= 0) return cfg.gpu_device_id % count;
  if (const char* lr = std::getenv("LOCAL_RANK")) return std::atoi(lr) % count;
  return 0;
}

}  // namespace

bool UseDeviceBinning(const Config& cfg, int64_t nrow, int64_t ncol) {
  const char* e = tuning::Get(tuning::Knob::DeviceBinning);
  if (e != nullptr && e[0] == '0') return false;
  const bool forced = e != nullptr && e[0] == '1';
  if (!forced && (cfg.device_type != "gpu" || nrow * ncol < (int64_t{1} << 22))) return false;
  return BinningDevice(cfg) >= 0;
}

std::vector<char> DeviceBinDenseMatrix(Dataset* ds, const void* data, bool is_f64, int32_t nrow, int32_t ncol,
                                       bool row_major, const Config& cfg) {
  std::vector<char> done_col(std::max(0, ncol), 0);
  const int dev = BinningDevice(cfg);
  if (dev < 0 || nrow <= 0) return done_col;
  // ---- tables: numerical-only groups whose members are all columns of the matrix
  std::vector<BinGroup> groups;
  std::vector<BinFeat> feats;
  std::vector<double> ub;
  std::vector<int> gid;  // dataset group of each device group
  for (int g = 0; g < ds->num_groups(); ++g) {
    const FeatureGroup& fg = ds->group(g);
    std::vector<std::pair<int, int>> members;  // (column, sub-feature)
    bool ok = !fg.sparse;  // (sparse groups: pushed on the host into their stored-row lists)
    for (size_t k = 0; k < fg.inner_features.size(); ++k) {
      const int inner = fg.inner_features[k];
      const int col = ds->RealFeatureIndex(inner);
      const BinMapper* m = ds->FeatureBinMapper(inner);
      if (col >= ncol || m->bin_type() != BinType::Numerical) ok = false;
      members.emplace_back(col, static_cast<int>(k));
    }
    if (!ok || members.empty()) continue;
    std::sort(members.begin(), members.end());
    BinGroup G;
    G.fbegin = static_cast<int>(feats.size());
    for (const auto& cm : members) {
      const int inner = fg.inner_features[cm.second];
      const BinMapper* m = ds->FeatureBinMapper(inner);
      BinFeat F;
      F.col = cm.first;
      const bool nan_miss = m->missing_type() == MissingType::NaN;
      F.hi = m->num_bin() - 1 - (nan_miss ? 1 : 0);
      F.nan_bin = nan_miss ? m->num_bin() - 1 : -1;
      F.mfb = static_cast<int>(m->GetMostFreqBin());
      F.ub_off = static_cast<int>(ub.size());
      F.goff = fg.bin_offsets[cm.second];
      const auto& u = m->upper_bounds();
      ub.insert(ub.end(), u.begin(), u.end());
      feats.push_back(F);
    }
    G.fend = static_cast<int>(feats.size());
    G.bytes = fg.bin_bytes;
    G.pad = 0;
    G.out_off = 0;
    groups.push_back(G);
    gid.push_back(g);
  }
  if (groups.empty()) return done_col;
  const size_t esz = is_f64 ? sizeof(double) : sizeof(float);
  // rows per chunk: at most ~256 MiB of values
  const int64_t chunk = std::max<int64_t>(kBinThreads, std::min<int64_t>(nrow, (int64_t{256} << 20) / (esz * ncol)));
  int64_t out_row_bytes = 0;
  for (auto& G : groups) {
    G.out_off = out_row_bytes * chunk;  // (a column of `chunk` rows per group)
    out_row_bytes += G.bytes;
  }
  int prev = 0;
  BINCHECK(hipGetDevice(&prev));
  BINCHECK(hipSetDevice(dev));
  void* d_x = nullptr;
  uint8_t* d_out = nullptr;
  BinGroup* d_groups = nullptr;
  BinFeat* d_feats = nullptr;
  double* d_ub = nullptr;
  struct Release {  // device buffers and the caller's device, also when a HIP call throws
    void** p[5];
    int dev;
    ~Release() {
      for (void** q : p) {
        if (*q != nullptr) (void)hipFree(*q);
      }
      (void)hipSetDevice(dev);
    }
  } release{{&d_x, reinterpret_cast<void**>(&d_out), reinterpret_cast<void**>(&d_groups),
             reinterpret_cast<void**>(&d_feats), reinterpret_cast<void**>(&d_ub)},
            prev};
  BINCHECK(hipMalloc(&d_x, esz * static_cast<size_t>(chunk) * ncol));
  BINCHECK(hipMalloc(reinterpret_cast<void**>(&d_out), static_cast<size_t>(out_row_bytes * chunk)));
  BINCHECK(hipMalloc(reinterpret_cast<void**>(&d_groups), sizeof(BinGroup) * groups.size()));
  BINCHECK(hipMalloc(reinterpret_cast<void**>(&d_feats), sizeof(BinFeat) * feats.size()));
  BINCHECK(hipMalloc(reinterpret_cast<void**>(&d_ub), sizeof(double) * std::max<size_t>(1, ub.size())));
  BINCHECK(hipMemcpy(d_groups, groups.data(), sizeof(BinGroup) * groups.size(), hipMemcpyHostToDevice));
  BINCHECK(hipMemcpy(d_feats, feats.data(), sizeof(BinFeat) * feats.size(), hipMemcpyHostToDevice));
  if (!ub.empty()) BINCHECK(hipMemcpy(d_ub, ub.data(), sizeof(double) * ub.size(), hipMemcpyHostToDevice));
  const int ngroups = static_cast<int>(groups.size());
  for (int64_t r0 = 0; r0 < nrow; r0 += chunk) {
    const int rows = static_cast<int>(std::min<int64_t>(chunk, nrow - r0));
    const char* src = static_cast<const char*>(data);
    long long rs, cs;
    if (row_major) {
      BINCHECK(hipMemcpy(d_x, src + esz * static_cast<size_t>(r0) * ncol, esz * static_cast<size_t>(rows) * ncol,
                         hipMemcpyHostToDevice));
      rs = ncol;
      cs = 1;
    } else {  // column j of the chunk at d_x + j * rows
      BINCHECK(hipMemcpy2D(d_x, esz * rows, src + esz * r0, esz * static_cast<size_t>(nrow), esz * rows, ncol,
                           hipMemcpyHostToDevice));
      rs = 1;
      cs = rows;
    }
    const dim3 grid((rows + kBinThreads - 1) / kBinThreads, (ngroups + kGroupsPerThread - 1) / kGroupsPerThread);
    if (is_f64) {
      hipLaunchKernelGGL(k_value_to_bin<double>, grid, dim3(kBinThreads), sizeof(double) * kBinLdsDoubles, 0, static_cast<const double*>(d_x), rows,
                         rs, cs, d_groups, ngroups, d_feats, d_ub, d_out);
    } else {
      hipLaunchKernelGGL(k_value_to_bin<float>, grid, dim3(kBinThreads), sizeof(double) * kBinLdsDoubles, 0, static_cast<const float*>(d_x), rows,
                         rs, cs, d_groups, ngroups, d_feats, d_ub, d_out);
    }
    BINCHECK(hipGetLastError());
    for (int k = 0; k < ngroups; ++k) {
      FeatureGroup& fg = ds->mutable_group(gid[k]);
      BINCHECK(hipMemcpy(fg.data.data() + static_cast<size_t>(r0) * fg.bin_bytes, d_out + groups[k].out_off,
                         static_cast<size_t>(rows) * fg.bin_bytes, hipMemcpyDeviceToHost));
    }
  }
  for (const auto& F : feats) done_col[F.col] = 1;
  return done_col;
}

}  // namespace lgbm_amd
