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
  void Broadcast(void* buf, size_t bytes, int root, void* stream) override {
    RCCLCHECK(ncclBroadcast(buf, buf, bytes, ncclUint8, root, comm_, static_cast<hipStream_t>(stream)));
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

int LGBM_AMD_RcclFree() {
  Network::SetDeviceComm(nullptr);
  return 0;
}

int LGBM_AMD_DeviceCount(int* out) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *out = n;
  return 0;
}

}  // extern "C"
