// RCCL (over xGMI) implementation of the device collectives used by the data-parallel
// MI355X learner: the per-split histogram all-reduce and the root statistics.  The
// reference's socket/MPI layer (src/network/linkers_socket.cpp, linkers_mpi.cpp) moves
// host histograms; here histograms never leave HBM.
//
// Bootstrapping: rank 0 obtains an ncclUniqueId (LGBM_AMD_RcclGetUniqueId), the launcher
// (torch.distributed / the Python package, or the host Network layer) broadcasts the
// bytes, and every rank calls LGBM_AMD_RcclInit with its device.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "lgbm_amd/c_api.h"
#include "lgbm_amd/log.h"
#include "lgbm_amd/network.h"

namespace lgbm_amd {

namespace {

#define RCCLCHECK(x)                                                                    \
  do {                                                                                  \
    ncclResult_t r_ = (x);                                                              \
    if (r_ != ncclSuccess) Log::Fatal("RCCL error %s: %s", #x, ncclGetErrorString(r_)); \
  } while (0)

class RcclComm : public DeviceComm {
 public:
  RcclComm(int n, int rank, const ncclUniqueId& id) : rank_(rank), size_(n) {
    RCCLCHECK(ncclCommInitRank(&comm_, n, id, rank));
  }
  ~RcclComm() override {
    if (comm_ != nullptr) ncclCommDestroy(comm_);
  }
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  void AllreduceSumF64(double* buf, size_t count, void* stream) override {
    RCCLCHECK(ncclAllReduce(buf, buf, count, ncclFloat64, ncclSum, comm_, static_cast<hipStream_t>(stream)));
  }
  void AllreduceSumF32(float* buf, size_t count, void* stream) override {
    RCCLCHECK(ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, comm_, static_cast<hipStream_t>(stream)));
  }
  void AllreduceSumI64(long long* buf, size_t count, void* stream) override {
    RCCLCHECK(ncclAllReduce(buf, buf, count, ncclInt64, ncclSum, comm_, static_cast<hipStream_t>(stream)));
  }
  void AllreduceMaxU32(uint32_t* buf, size_t count, void* stream) override {
    RCCLCHECK(ncclAllReduce(buf, buf, count, ncclUint32, ncclMax, comm_, static_cast<hipStream_t>(stream)));
  }
  void Allgather(const void* send, void* recv, size_t bytes_per_rank, void* stream) override {
    RCCLCHECK(ncclAllGather(send, recv, bytes_per_rank, ncclUint8, comm_, static_cast<hipStream_t>(stream)));
  }
  void ReduceScatterSumF64(const double* send, double* recv, size_t recv_count, void* stream) override {
    RCCLCHECK(ncclReduceScatter(send, recv, recv_count, ncclFloat64, ncclSum, comm_, static_cast<hipStream_t>(stream)));
  }
  void ReduceScatterSumI64(const long long* send, long long* recv, size_t recv_count, void* stream) override {
    RCCLCHECK(ncclReduceScatter(send, recv, recv_count, ncclInt64, ncclSum, comm_, static_cast<hipStream_t>(stream)));
  }
  void Broadcast(void* buf, size_t bytes, int root, void* stream) override {
    RCCLCHECK(ncclBroadcast(buf, buf, bytes, ncclUint8, root, comm_, static_cast<hipStream_t>(stream)));
  }
  bool AsyncError(std::string* msg) override {
    ncclResult_t r = ncclSuccess;
    if (comm_ == nullptr || ncclCommGetAsyncError(comm_, &r) != ncclSuccess) return false;
    if (r == ncclSuccess || r == ncclInProgress) return false;
    *msg = ncclGetErrorString(r);
    return true;
  }
  void Abort() override {
    if (comm_ != nullptr) (void)ncclCommAbort(comm_);
    comm_ = nullptr;
  }

 private:
  ncclComm_t comm_ = nullptr;
  int rank_, size_;
};

thread_local std::string g_err;

}  // namespace

}  // namespace lgbm_amd

using namespace lgbm_amd;

extern "C" {

int LGBM_AMD_RcclUniqueIdSize(int* out) {
  *out = static_cast<int>(sizeof(ncclUniqueId));
  return 0;
}

int LGBM_AMD_RcclGetUniqueId(char* out_id) {
  try {
    ncclUniqueId id;
    RCCLCHECK(ncclGetUniqueId(&id));
    std::memcpy(out_id, &id, sizeof(id));
  } catch (std::exception& e) {
    Log::Warning("%s", e.what());
    return -1;
  }
  return 0;
}

int LGBM_AMD_RcclInit(int num_ranks, int rank, int device_id, const char* unique_id) {
  try {
    if (hipSetDevice(device_id) != hipSuccess) Log::Fatal("hipSetDevice(%d) failed", device_id);
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof(id));
    Network::SetDeviceComm(std::make_shared<RcclComm>(num_ranks, rank, id));
  } catch (std::exception& e) {
    Log::Warning("%s", e.what());
    return -1;
  }
  return 0;
}

// every collective of the device comm (RCCL or the in-process one) on small device
// buffers, checked on the host: rank r contributes (r + 1) * i to element i, so sums are
// (n (n + 1) / 2) * i; plus an int64 reduce-scatter and an allgather
int LGBM_AMD_RcclSelfTest(int* out_ok) {
  try {
    DeviceComm* dc = Network::device_comm();
    if (dc == nullptr) Log::Fatal("no device comm (call LGBM_AMD_RcclInit first)");
    const int n = dc->size(), r = dc->rank();
    const size_t cnt = 1000;
    // (a non-blocking stream and stream-ordered copies only: ranks that share the device wait
    // on each other inside the collective kernels, so nothing here may wait for the device)
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) Log::Fatal("hipStreamCreate failed");
    long long* di64;
    double* df64;
    uint32_t* du32;
    if (hipMalloc(&di64, cnt * sizeof(long long)) != hipSuccess || hipMalloc(&df64, cnt * sizeof(double)) != hipSuccess ||
        hipMalloc(&du32, cnt * sizeof(uint32_t)) != hipSuccess) {
      Log::Fatal("hipMalloc failed");
    }
    std::vector<long long> hi(cnt);
    std::vector<double> hf(cnt);
    std::vector<uint32_t> hu(cnt);
    for (size_t i = 0; i < cnt; ++i) {
      hi[i] = static_cast<long long>((r + 1) * i) - 500;
      hf[i] = 0.5 * (r + 1) * i;
      hu[i] = static_cast<uint32_t>(r * 7 + i);
    }
    (void)hipMemcpyAsync(di64, hi.data(), cnt * sizeof(long long), hipMemcpyHostToDevice, s);
    (void)hipMemcpyAsync(df64, hf.data(), cnt * sizeof(double), hipMemcpyHostToDevice, s);
    (void)hipMemcpyAsync(du32, hu.data(), cnt * sizeof(uint32_t), hipMemcpyHostToDevice, s);
    dc->AllreduceSumI64(di64, cnt, s);
    dc->AllreduceSumF64(df64, cnt, s);
    dc->AllreduceMaxU32(du32, cnt, s);
    // reduce-scatter: block r of every rank holds (rank + 1) * (r * 10 + j); rank r receives
    // sum over ranks = tri * (r * 10 + j); allgather of 8-byte records: rank q sends q + 1
    const size_t blk = 10;
    long long *rs_in = nullptr, *rs_out = nullptr, *ag = nullptr;
    if (hipMalloc(&rs_in, blk * n * sizeof(long long)) != hipSuccess || hipMalloc(&rs_out, blk * sizeof(long long)) != hipSuccess ||
        hipMalloc(&ag, n * sizeof(long long)) != hipSuccess) {
      Log::Fatal("hipMalloc failed");
    }
    std::vector<long long> hrs(blk * n), hag(n, 0);
    for (size_t i = 0; i < blk * n; ++i) hrs[i] = static_cast<long long>((r + 1) * i);
    hag[r] = r + 1;
    (void)hipMemcpyAsync(rs_in, hrs.data(), hrs.size() * sizeof(long long), hipMemcpyHostToDevice, s);
    (void)hipMemcpyAsync(ag, hag.data(), hag.size() * sizeof(long long), hipMemcpyHostToDevice, s);
    dc->ReduceScatterSumI64(rs_in, rs_out, blk, s);
    dc->Allgather(ag + r, ag, sizeof(long long), s);
    std::vector<long long> hro(blk);
    (void)hipMemcpyAsync(hro.data(), rs_out, blk * sizeof(long long), hipMemcpyDeviceToHost, s);
    (void)hipMemcpyAsync(hag.data(), ag, n * sizeof(long long), hipMemcpyDeviceToHost, s);
    (void)hipMemcpyAsync(hi.data(), di64, cnt * sizeof(long long), hipMemcpyDeviceToHost, s);
    (void)hipMemcpyAsync(hf.data(), df64, cnt * sizeof(double), hipMemcpyDeviceToHost, s);
    (void)hipMemcpyAsync(hu.data(), du32, cnt * sizeof(uint32_t), hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    // every rank is past its collectives before anyone frees: hipFree waits for the whole
    // device, which would include a faster peer's next collective kernel, spinning until this
    // rank joins it (thread ranks sharing one GPU)
    dc->HostBarrier();
    (void)hipFree(rs_in);
    (void)hipFree(rs_out);
    (void)hipFree(ag);
    const long long tri = static_cast<long long>(n) * (n + 1) / 2;
    bool ok = true;
    for (size_t j = 0; j < blk; ++j) ok = ok && hro[j] == tri * static_cast<long long>(r * blk + j);
    for (int q = 0; q < n; ++q) ok = ok && hag[q] == q + 1;
    for (size_t i = 0; i < cnt; ++i) {
      ok = ok && hi[i] == tri * static_cast<long long>(i) - 500LL * n;
      ok = ok && hf[i] == 0.5 * static_cast<double>(tri) * static_cast<double>(i);
      ok = ok && hu[i] == static_cast<uint32_t>((n - 1) * 7 + i);
    }
    (void)hipFree(di64);
    (void)hipFree(df64);
    (void)hipFree(du32);
    (void)hipStreamDestroy(s);
    *out_ok = ok ? 1 : 0;
  } catch (std::exception& e) {
    Log::Warning("%s", e.what());
    return -1;
  }
  return 0;
}

// the device learner captures its per-split all-reduces into the tree's hipGraph: two
// all-reduces captured from a stream, the graph replayed three times, result checked
// (every rank contributes i to element i, so after 6 all-reduces it holds i * n^6)
int LGBM_AMD_RcclGraphSelfTest(int* out_ok) {
  try {
    DeviceComm* dc = Network::device_comm();
    if (dc == nullptr) Log::Fatal("no device comm (call LGBM_AMD_RcclInit first)");
    const int n = dc->size();
    const size_t cnt = 4096;
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) Log::Fatal("hipStreamCreate failed");
    long long* d = nullptr;
    if (hipMalloc(&d, cnt * sizeof(long long)) != hipSuccess) Log::Fatal("hipMalloc failed");
    std::vector<long long> h(cnt);
    for (size_t i = 0; i < cnt; ++i) h[i] = static_cast<long long>(i);
    (void)hipMemcpyAsync(d, h.data(), cnt * sizeof(long long), hipMemcpyHostToDevice, s);
    (void)hipStreamSynchronize(s);
    dc->HostBarrier();  // (no rank's collectives spin while a peer still allocates)
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) != hipSuccess) Log::Fatal("begin capture failed");
    dc->AllreduceSumI64(d, cnt, s);
    dc->AllreduceSumI64(d, cnt, s);
    if (hipStreamEndCapture(s, &g) != hipSuccess) Log::Fatal("end capture failed");
    if (hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) != hipSuccess) Log::Fatal("graph instantiate failed");
    for (int it = 0; it < 3; ++it) {
      if (hipGraphLaunch(ge, s) != hipSuccess) Log::Fatal("graph launch failed");
    }
    (void)hipMemcpyAsync(h.data(), d, cnt * sizeof(long long), hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    dc->HostBarrier();  // (before the frees below wait for the device)
    long long f = 1;
    for (int k = 0; k < 6; ++k) f *= n;
    bool ok = true;
    for (size_t i = 0; i < cnt; ++i) ok = ok && h[i] == static_cast<long long>(i) * f;
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
    (void)hipFree(d);
    (void)hipStreamDestroy(s);
    *out_ok = ok ? 1 : 0;
  } catch (std::exception& e) {
    Log::Warning("%s", e.what());
    return -1;
  }
  return 0;
}

int LGBM_AMD_RcclFree() {
  Network::SetDeviceComm(nullptr);
  return 0;
}

int LGBM_AMD_DeviceSynchronize() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return 0;
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

int LGBM_AMD_DeviceCount(int* out) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *out = n;
  return 0;
}

}  // extern "C"
