// Host-side collective layer used by distributed training (control plane + CPU
// learners) and the device-collective registry used by the HIP learners.
//
// Reference: include/LightGBM/network.h:89-313 (static Network facade, Allreduce /
// Allgather / ReduceScatter, GlobalSyncUpBy{Min,Max,Sum,Mean}, external functions via
// LGBM_NetworkInitWithFunctions).  Transport here is pluggable:
//   * external functions (C API; the Python package plugs torch.distributed in),
//   * built-in TCP full mesh for `machines=` / `machine_list_filename` configs,
//   * in-process "fake" ranks (threads) for tests.
// Transports with a point-to-point SendRecv (TCP, threads) get Network's own algorithms:
// Bruck / ring allgather, recursive-halving (power-of-two) / ring reduce-scatter, and
// reduce-scatter + allgather all-reduce (src/network/collectives.cpp).
// Device collectives (histogram all-reduce over xGMI) go through `DeviceComm`,
// implemented with RCCL in src/network/rccl_comm.cpp.
#pragma once

#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "lgbm_amd/config.h"
#include "lgbm_amd/meta.h"

namespace lgbm_amd {

// elementwise reducer: dst[i] = reduce(dst[i], src[i]) over `len` bytes of `type_size` items
using ReduceFunction = std::function<void(const char* src, char* dst, int type_size, comm_size_t len)>;

// C-ABI signatures of the reference's external collectives (c_api.h:1266-1288)
typedef void (*ReduceFunctionPtr)(const char* input, char* output, int type_size, comm_size_t array_size);
typedef void (*ReduceScatterFunctionPtr)(char* input, comm_size_t input_size, int type_size,
                                         const comm_size_t* block_start, const comm_size_t* block_len,
                                         int num_block, char* output, comm_size_t output_size,
                                         const ReduceFunctionPtr& reducer);
typedef void (*AllgatherFunctionPtr)(char* input, comm_size_t input_size, const comm_size_t* block_start,
                                     const comm_size_t* block_len, int num_block, char* output,
                                     comm_size_t output_size);

class HostTransport {
 public:
  virtual ~HostTransport() = default;
  virtual int rank() const = 0;
  virtual int num_machines() const = 0;
  // variable-size allgather: every rank contributes block_len[rank] bytes
  virtual void Allgather(const char* input, comm_size_t input_size, const comm_size_t* block_start,
                         const comm_size_t* block_len, char* output, comm_size_t output_size) = 0;
  // optional point-to-point exchange: send `send_len` bytes to rank `to` while receiving
  // `recv_len` bytes from rank `from` (either length may be 0).  When available, Network runs
  // its own collective algorithms over it (src/network/collectives.cpp).
  virtual bool HasPointToPoint() const { return false; }
  virtual void SendRecv(int to, const char* send, comm_size_t send_len, int from, char* recv, comm_size_t recv_len) {
    (void)to; (void)send; (void)send_len; (void)from; (void)recv; (void)recv_len;
  }
  // optional native reduce-scatter; default implemented with Allgather + local reduce
  virtual bool ReduceScatter(char* input, comm_size_t input_size, int type_size, const comm_size_t* block_start,
                             const comm_size_t* block_len, char* output, comm_size_t output_size,
                             const ReduceFunction& reducer) {
    (void)input; (void)input_size; (void)type_size; (void)block_start; (void)block_len; (void)output;
    (void)output_size; (void)reducer;
    return false;
  }
};

// device collectives (all pointers are device pointers, stream-ordered)
class DeviceComm {
 public:
  virtual ~DeviceComm() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  virtual void AllreduceSumF64(double* buf, size_t count, void* stream) = 0;
  virtual void AllreduceSumF32(float* buf, size_t count, void* stream) = 0;
  virtual void AllreduceSumI64(long long* buf, size_t count, void* stream) = 0;
  virtual void AllreduceMaxU32(uint32_t* buf, size_t count, void* stream) = 0;
  virtual void Allgather(const void* send, void* recv, size_t bytes_per_rank, void* stream) = 0;
  virtual void ReduceScatterSumF64(const double* send, double* recv, size_t recv_count, void* stream) = 0;
  // send holds size() blocks of recv_count elements; rank r receives the sum of block r
  virtual void ReduceScatterSumI64(const long long* send, long long* recv, size_t recv_count, void* stream) = 0;
  virtual void Broadcast(void* buf, size_t bytes, int root, void* stream) = 0;
  // the collectives can be captured into a hipGraph (stream-ordered, no host rendezvous)
  virtual bool CaptureSafe() const { return true; }
  // collectives enqueued while a guard is set are skipped when the device flag *d_flag is
  // nonzero at run time (replicated state such as Round::done: every rank skips the same ones);
  // communicators that cannot skip ignore it
  virtual void SetSkipGuard(const int32_t* d_flag) { (void)d_flag; }
  // ranks that share one device (thread ranks) and wait on each other inside kernels must
  // not block in a device-wide synchronisation (hipFree, graph teardown) while a peer's
  // kernel waits for a collective this rank has yet to launch: the learner calls this at the
  // start of each tree and before re-capturing its graphs (the same points on every rank),
  // and such comms rendezvous there.  One GPU per process: nothing to do.
  virtual void HostBarrier() {}
  // bound of every device-side wait of later collectives (communicators without device-side
  // waits ignore it)
  virtual void SetWaitLimit(double seconds) { (void)seconds; }
  // failure detection (watchdog of the device learner): an asynchronous communicator error,
  // and aborting every pending collective so that no rank stays blocked
  virtual bool AsyncError(std::string* msg) {
    (void)msg;
    return false;
  }
  virtual void Abort() {}
};

class Network {
 public:
  // TCP mesh from config (num_machines > 1 with machines / machine_list_filename)
  static void Init(const Config& cfg);
  static void InitWithTransport(std::shared_ptr<HostTransport> t);
  static void InitWithFunctions(int num_machines, int rank, ReduceScatterFunctionPtr rs, AllgatherFunctionPtr ag);
  static void Dispose();
  // called from inside an external collective function that failed: the collective raises
  // on this thread once the function returns
  static void ReportExternalError(const std::string& msg);
  static int rank();
  static int num_machines();
  static bool IsDistributed() { return num_machines() > 1; }

  static void SetDeviceComm(std::shared_ptr<DeviceComm> c);
  static DeviceComm* device_comm();

  static void Allreduce(char* input, comm_size_t input_size, int type_size, char* output,
                        const ReduceFunction& reducer);
  static void Allgather(char* input, comm_size_t send_size, char* output);
  static void Allgather(char* input, const comm_size_t* block_start, const comm_size_t* block_len, char* output,
                        comm_size_t all_size);
  static void ReduceScatter(char* input, comm_size_t input_size, int type_size, const comm_size_t* block_start,
                            const comm_size_t* block_len, char* output, comm_size_t output_size,
                            const ReduceFunction& reducer);

  template <typename T>
  static T GlobalSyncUpByMin(T v) {
    return GlobalReduceScalar<T>(v, [](T a, T b) { return a < b ? a : b; });
  }
  template <typename T>
  static T GlobalSyncUpByMax(T v) {
    return GlobalReduceScalar<T>(v, [](T a, T b) { return a > b ? a : b; });
  }
  template <typename T>
  static T GlobalSyncUpBySum(T v) {
    return GlobalReduceScalar<T>(v, [](T a, T b) { return a + b; });
  }
  template <typename T>
  static T GlobalSyncUpByMean(T v) {
    return static_cast<T>(GlobalSyncUpBySum<double>(static_cast<double>(v)) / num_machines());
  }
  template <typename T>
  static std::vector<T> GlobalSum(const std::vector<T>& v) {
    std::vector<T> out(v.size());
    if (num_machines() <= 1 || v.empty()) return v;
    Allreduce(reinterpret_cast<char*>(const_cast<T*>(v.data())), static_cast<comm_size_t>(sizeof(T) * v.size()),
              sizeof(T), reinterpret_cast<char*>(out.data()), [](const char* src, char* dst, int ts, comm_size_t len) {
                for (comm_size_t i = 0; i < len; i += ts) {
                  T a, b;
                  std::memcpy(&a, src + i, sizeof(T));
                  std::memcpy(&b, dst + i, sizeof(T));
                  b += a;
                  std::memcpy(dst + i, &b, sizeof(T));
                }
              });
    return out;
  }
  // every rank's value, indexed by rank
  template <typename T>
  static std::vector<T> GlobalArray(T v) {
    std::vector<T> out(num_machines());
    if (num_machines() <= 1) {
      out[0] = v;
      return out;
    }
    Allgather(reinterpret_cast<char*>(&v), sizeof(T), reinterpret_cast<char*>(out.data()));
    return out;
  }

 private:
  template <typename T, typename F>
  static T GlobalReduceScalar(T v, F f) {
    if (num_machines() <= 1) return v;
    auto all = GlobalArray<T>(v);
    T r = all[0];
    for (size_t i = 1; i < all.size(); ++i) r = f(r, all[i]);
    return r;
  }
};

// in-process multi-rank transport (ranks are threads sharing a rendezvous object).
// timeout_s > 0: a collective waiting longer raises; fail_rank / fail_at_call inject a fault
// (that rank raises at its fail_at_call-th collective, its peers then raise too)
std::vector<std::shared_ptr<HostTransport>> MakeThreadTransports(int num_ranks, double timeout_s = 0,
                                                                 int fail_rank = -1, int fail_at_call = 0);

// in-process device collectives for ranks that are threads sharing one GPU (tests and
// rehearsal of the distributed device learners without RCCL): each call rendezvouses the
// threads, then device kernels read the peers' buffers directly.  Not graph-capturable.
// fail_rank / fail_at_call inject a fault into that rank's fail_at_call-th device collective
// (it raises before touching any peer buffer; the peers raise at their rendezvous)
std::vector<std::shared_ptr<DeviceComm>> MakeThreadDeviceComms(int num_ranks, double timeout_s = 0, int fail_rank = -1,
                                                               int fail_at_call = 0);

// capture-safe one-shot peer collectives (src/network/peer_comm.cpp): thread ranks sharing
// the current device (timeout_s bounds every device-side wait; fail_rank's collective number
// fail_at_call stops as a dead rank would, its peers time out) ...
std::vector<std::shared_ptr<DeviceComm>> MakePeerThreadComms(int num_ranks, double timeout_s = 0, int fail_rank = -1,
                                                             int fail_at_call = 0);
// ... or one process per GPU: windows exchanged as hipIpc handles over the host Network
std::shared_ptr<DeviceComm> MakePeerIpcComm(int device_id, double timeout_s = 0);

// MPI host transport (src/network/mpi_transport.cpp; reference linkers_mpi.cpp), the MPI library
// opened at run time: Network::Init uses it instead of the TCP mesh when LGBM_AMD_NETWORK=mpi.
// The CLI finalizes MPI at a normal exit (when this process initialised it) and aborts it after
// an error, so that no peer stays blocked in a collective.
bool MpiSelected();
void MpiFinalizeIfStarted();
void MpiAbortIfStarted();

}  // namespace lgbm_amd
