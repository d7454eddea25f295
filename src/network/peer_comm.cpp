// Peer device communicator: capture-safe one-shot collectives over symmetric windows
// (kernels in src/device/peer_kernels.hip).  The reference's distributed learners call
// Network::ReduceScatter / Allreduce once or twice per split over sockets
// (data_parallel_tree_learner.cpp:154-247, voting_parallel_tree_learner.cpp:300-343); the
// MI355X learner batches a whole round of expansions per collective and runs each as a single
// kernel that pulls the peers' inputs over xGMI, inside the round's hipGraph.
//
// Windows: one hipDeviceMallocUncached allocation per rank ([flags][stage]).
//   * thread ranks of one process (tests, rehearsal): every window on the current device,
//     shared as plain pointers (MakePeerThreadComms);
//   * one process per GPU: each rank exports its window with hipIpcGetMemHandle, the handles
//     and device ordinals are all-gathered over the host Network, and every rank maps its
//     peers' windows with hipIpcOpenMemHandle (peer access enabled lazily) -- MakePeerIpcComm.
// Collectives larger than the stage run as consecutive chunks, each its own epoch.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <mutex>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../device/kernels.h"
#include "lgbm_amd/log.h"
#include "lgbm_amd/network.h"
#include "lgbm_amd/tuning.h"

namespace lgbm_amd {

namespace {

#define PCHK(x)                                                                                     \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) Log::Fatal("HIP error %s at %s:%d: %s", #x, __FILE__, __LINE__, hipGetErrorString(e_)); \
  } while (0)

size_t StageBytesFromEnv(size_t dflt) {
  const char* e = tuning::Get(tuning::Knob::PeerStageMb);
  if (e != nullptr && std::atoi(e) > 0) return static_cast<size_t>(std::atoi(e)) << 20;
  return dflt;
}

// one rank's window on the current device
char* AllocWindow(size_t stage_bytes) {
  void* p = nullptr;
  PCHK(hipExtMallocWithFlags(&p, dev::kPeerFlagBytes + stage_bytes, hipDeviceMallocUncached));
  PCHK(hipMemset(p, 0, dev::kPeerFlagBytes));
  return static_cast<char*>(p);
}

// windows shared by the thread ranks of one process (freed with the last comm), and their
// host rendezvous (DeviceComm::HostBarrier)
struct PeerWindows {
  std::vector<char*> win;
  double timeout_s = 60.0;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  long long generation = 0;
  bool failed = false;
  ~PeerWindows() {
    (void)hipDeviceSynchronize();
    for (char* w : win) (void)hipFree(w);
  }
  void Barrier(int rank) {
    std::unique_lock<std::mutex> lk(mu);
    const long long gen = generation;
    if (++arrived == static_cast<int>(win.size())) {
      arrived = 0;
      ++generation;
      cv.notify_all();
    } else if (!cv.wait_for(lk, std::chrono::duration<double>(timeout_s),
                            [&] { return failed || generation != gen; })) {
      failed = true;
      cv.notify_all();
    }
    if (failed) Log::Fatal("peer device comm: rank %d timed out at the host barrier (a peer rank stopped)", rank);
  }
};

class PeerComm : public DeviceComm {
 public:
  PeerComm(int rank, int n, std::vector<char*> wins, size_t stage_bytes, double timeout_s, long long fail_epoch)
      : rank_(rank), n_(n), win_(std::move(wins)), stage_bytes_(stage_bytes), fail_epoch_(fail_epoch) {
    if (n_ > dev::kMaxPeerBufs) Log::Fatal("peer device comm supports at most %d ranks", dev::kMaxPeerBufs);
    timeout_ticks_ = static_cast<long long>(std::max(0.1, timeout_s) * 1e8);
    PCHK(hipMalloc(&ctl_, 4 * sizeof(unsigned long long)));
    PCHK(hipMemset(ctl_, 0, 4 * sizeof(unsigned long long)));
    PCHK(hipHostMalloc(reinterpret_cast<void**>(&status_), 4 * sizeof(unsigned int), hipHostMallocMapped));
    std::memset(status_, 0, 4 * sizeof(unsigned int));
    PCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&status_dev_), status_, 0));
    PCHK(hipDeviceSynchronize());
  }
  ~PeerComm() override {
    (void)hipDeviceSynchronize();
    for (char* p : opened_) (void)hipIpcCloseMemHandle(p);
    if (own_win_ != nullptr) (void)hipFree(own_win_);
    if (ctl_ != nullptr) (void)hipFree(ctl_);
    if (status_ != nullptr) (void)hipHostFree(status_);
  }
  // one process per GPU: ranks skew between trees (evaluation, checkpoints, logging on one
  // rank) while their peers already wait inside the next tree's first collective, so the
  // learner's time_out bounds the waits.  Thread ranks (tests) keep the bound they were made
  // with: their fault-injection tests rely on it.
  void SetWaitLimit(double seconds) override {
    if (seconds > 0 && own_win_ != nullptr) timeout_ticks_ = static_cast<long long>(seconds * 1e8);  // (100 MHz clock)
  }
  // the windows this comm owns / mapped (multi-process)
  void Own(char* own, std::vector<char*> opened) {
    own_win_ = own;
    opened_ = std::move(opened);
  }
  void Share(std::shared_ptr<PeerWindows> w) { shared_ = std::move(w); }

  int rank() const override { return rank_; }
  int size() const override { return n_; }
  bool CaptureSafe() const override { return true; }
  void SetSkipGuard(const int32_t* d_flag) override { guard_ = d_flag; }
  void HostBarrier() override {
    if (shared_ != nullptr) shared_->Barrier(rank_);
  }

  void AllreduceSumF64(double* buf, size_t count, void* stream) override {
    Reduce(dev::kPeerAllreduce, dev::kPeerSumF64, buf, buf, count, 0, sizeof(double), stream);
  }
  void AllreduceSumF32(float* buf, size_t count, void* stream) override {
    Reduce(dev::kPeerAllreduce, dev::kPeerSumF32, buf, buf, count, 0, sizeof(float), stream);
  }
  void AllreduceSumI64(long long* buf, size_t count, void* stream) override {
    Reduce(dev::kPeerAllreduce, dev::kPeerSumI64, buf, buf, count, 0, sizeof(long long), stream);
  }
  void AllreduceMaxU32(uint32_t* buf, size_t count, void* stream) override {
    Reduce(dev::kPeerAllreduce, dev::kPeerMaxU32, buf, buf, count, 0, sizeof(uint32_t), stream);
  }
  void ReduceScatterSumF64(const double* send, double* recv, size_t recv_count, void* stream) override {
    Reduce(dev::kPeerReduceScatter, dev::kPeerSumF64, send, recv, recv_count, recv_count, sizeof(double), stream);
  }
  void ReduceScatterSumI64(const long long* send, long long* recv, size_t recv_count, void* stream) override {
    Reduce(dev::kPeerReduceScatter, dev::kPeerSumI64, send, recv, recv_count, recv_count, sizeof(long long), stream);
  }
  void Allgather(const void* send, void* recv, size_t bytes_per_rank, void* stream) override {
    const int elem = CopyElem(send, recv, bytes_per_rank);
    Copy(dev::kPeerAllgather, send, recv, bytes_per_rank / elem, elem, 0, stream);
  }
  void Broadcast(void* buf, size_t bytes, int root, void* stream) override {
    const int elem = CopyElem(buf, buf, bytes);
    Copy(dev::kPeerBroadcast, buf, buf, bytes / elem, elem, root, stream);
  }
  bool AsyncError(std::string* msg) override {
    const unsigned code = __atomic_load_n(&status_[0], __ATOMIC_ACQUIRE);
    if (code == dev::kPeerOk) return false;
    const unsigned ep = __atomic_load_n(&status_[2], __ATOMIC_ACQUIRE);
    static const char* what[] = {"ok", "timed out waiting for a peer rank", "injected fault", "aborted"};
    *msg = std::string("peer device collective ") + (code < 4 ? what[code] : "failed") + " (rank " +
           std::to_string(rank_) + ", collective " + std::to_string(ep) + ")";
    return true;
  }
  void Abort() override { __atomic_store_n(&status_[1], 1u, __ATOMIC_RELEASE); }

 private:
  static int CopyElem(const void* a, const void* b, size_t bytes) {
    const uintptr_t m = reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) | bytes;
    return (m & 15) == 0 ? 16 : (m & 3) == 0 ? 4 : 1;
  }
  dev::PeerArgs Base(int kind, int op, int elem) const {
    dev::PeerArgs a{};
    for (int p = 0; p < n_; ++p) a.win[p] = win_[p];
    a.n = n_;
    a.rank = rank_;
    a.kind = kind;
    a.op = op;
    a.elem = elem;
    a.fail_epoch = fail_epoch_;
    a.ctl = ctl_;
    a.status = status_dev_;
    a.guard = guard_;
    a.timeout_ticks = timeout_ticks_;
    return a;
  }
  // allreduce (stride unused) / reduce-scatter (send: n blocks of `stride` elements)
  void Reduce(int kind, int op, const void* send, void* recv, size_t count, size_t stride, int elem, void* stream) {
    if (count == 0) return;
    const size_t per_chunk = kind == dev::kPeerReduceScatter ? stage_bytes_ / (static_cast<size_t>(n_) * elem)
                                                             : stage_bytes_ / elem;
    if (per_chunk == 0) Log::Fatal("peer device comm: stage of %zu bytes is too small", stage_bytes_);
    dev::PeerArgs a = Base(kind, op, elem);
    a.send = static_cast<const char*>(send);
    a.recv = static_cast<char*>(recv);
    a.stride = stride;
    for (size_t off = 0; off < count; off += per_chunk) {
      a.off = off;
      a.count = std::min(per_chunk, count - off);
      dev::PeerCollective(a, static_cast<hipStream_t>(stream));
    }
  }
  void Copy(int kind, const void* send, void* recv, size_t count, int elem, int root, void* stream) {
    if (count == 0) return;
    const size_t per_chunk = stage_bytes_ / elem;
    dev::PeerArgs a = Base(kind, 0, elem);
    a.send = static_cast<const char*>(send);
    a.recv = static_cast<char*>(recv);
    a.root = root;
    a.stride = count;  // allgather: elements per rank
    for (size_t off = 0; off < count; off += per_chunk) {
      a.off = off;
      a.count = std::min(per_chunk, count - off);
      dev::PeerCollective(a, static_cast<hipStream_t>(stream));
    }
  }

  int rank_, n_;
  std::vector<char*> win_;
  size_t stage_bytes_;
  long long fail_epoch_;
  long long timeout_ticks_ = 0;
  unsigned long long* ctl_ = nullptr;
  unsigned int* status_ = nullptr;
  unsigned int* status_dev_ = nullptr;
  const int32_t* guard_ = nullptr;
  char* own_win_ = nullptr;
  std::vector<char*> opened_;
  std::shared_ptr<PeerWindows> shared_;
};

// the topology the last MakePeerIpcComm found (LGBM_AMD_DeviceCommTopology): JSON
std::mutex g_topo_mu;
std::string g_topo = "{}";

const char* LinkName(uint32_t t) {
  switch (t) {
    case 4: return "xgmi";  // (HSA_AMD_LINK_INFO_TYPE_XGMI)
    case 2: return "pcie";
    case 3: return "infiniband";
    case 1: return "qpi";
    case 0: return "hypertransport";
    default: return "unknown";
  }
}

}  // namespace

std::vector<std::shared_ptr<DeviceComm>> MakePeerThreadComms(int num_ranks, double timeout_s, int fail_rank,
                                                             int fail_at_call) {
  const size_t stage = StageBytesFromEnv(size_t(tuning::kPeerStageMbThreads) << 20);
  auto wins = std::make_shared<PeerWindows>();
  if (timeout_s > 0) wins->timeout_s = timeout_s;
  for (int r = 0; r < num_ranks; ++r) wins->win.push_back(AllocWindow(stage));
  std::vector<std::shared_ptr<DeviceComm>> out;
  for (int r = 0; r < num_ranks; ++r) {
    auto c = std::make_shared<PeerComm>(r, num_ranks, wins->win, stage, timeout_s > 0 ? timeout_s : 60.0,
                                        r == fail_rank ? fail_at_call : 0);
    c->Share(wins);
    out.push_back(c);
  }
  return out;
}

// one process per GPU: called by every rank (host Network initialised).  Every rank takes part
// in both host exchanges whatever fails locally, so a failure raises on every rank instead of
// leaving the others blocked in the exchange.
std::shared_ptr<DeviceComm> MakePeerIpcComm(int device_id, double timeout_s) {
  const int n = Network::num_machines(), rank = Network::rank();
  if (n > dev::kMaxPeerBufs) Log::Fatal("peer device comm supports at most %d ranks", dev::kMaxPeerBufs);
  const size_t stage = StageBytesFromEnv(size_t(tuning::kPeerStageMbProcesses) << 20);
  // devices are identified by PCI bus id, not by ordinal: under per-process device isolation
  // (HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES) every rank's device is ordinal 0
  struct Entry {
    hipIpcMemHandle_t h;
    int32_t device;
    int32_t ok;
    char bus[32];
  };
  Entry mine{};
  mine.device = device_id;
  char* own = nullptr;
  std::string why;
  try {
    PCHK(hipSetDevice(device_id));
    PCHK(hipDeviceGetPCIBusId(mine.bus, static_cast<int>(sizeof(mine.bus)), device_id));
    own = AllocWindow(stage);
    PCHK(hipDeviceSynchronize());
    PCHK(hipIpcGetMemHandle(&mine.h, own));
    mine.ok = 1;
  } catch (std::exception& e) {
    why = e.what();
  }
  std::vector<Entry> all(n);
  Network::Allgather(reinterpret_cast<char*>(&mine), static_cast<comm_size_t>(sizeof(Entry)),
                     reinterpret_cast<char*>(all.data()));
  std::vector<char*> wins(n, nullptr), opened;
  int32_t ok = 1;
  for (int p = 0; p < n; ++p) ok &= all[p].ok;
  // this rank's view of the topology: per peer, the same device or the link and hops to it
  std::string topo = std::string("{\"rank\": ") + std::to_string(rank) + ", \"world\": " + std::to_string(n) +
                     ", \"device\": " + std::to_string(device_id) + ", \"bus_id\": \"" + mine.bus + "\", \"peers\": [";
  if (ok) {
    try {
      for (int p = 0; p < n; ++p) {
        all[p].bus[sizeof(all[p].bus) - 1] = '\0';
        if (p == rank) {
          wins[p] = own;
          continue;
        }
        std::string rec = std::string("{\"rank\": ") + std::to_string(p) + ", \"bus_id\": \"" + all[p].bus + "\"";
        if (std::strcmp(all[p].bus, mine.bus) == 0) {
          rec += ", \"same_device\": true";  // (ranks sharing one GPU: tests, rehearsals)
        } else {
          int ord = -1;
          if (hipDeviceGetByPCIBusId(&ord, all[p].bus) != hipSuccess) ord = -1;
          (void)hipGetLastError();
          if (ord >= 0 && ord != device_id) {
            int can = 0;
            PCHK(hipDeviceCanAccessPeer(&can, device_id, ord));
            if (!can) Log::Fatal("device %s cannot access device %s", mine.bus, all[p].bus);
            const hipError_t e = hipDeviceEnablePeerAccess(ord, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) PCHK(e);
            (void)hipGetLastError();
            uint32_t lt = 0, hops = 0;
            const bool have = hipExtGetLinkTypeAndHopCount(device_id, ord, &lt, &hops) == hipSuccess;
            (void)hipGetLastError();
            rec += std::string(", \"ordinal\": ") + std::to_string(ord) + ", \"peer_access\": true";
            if (have) rec += std::string(", \"link\": \"") + LinkName(lt) + "\", \"hops\": " + std::to_string(hops);
          } else {
            // not visible to this process (device isolation): the mapping enables access lazily
            rec += ", \"visible\": false";
          }
        }
        rec += "}";
        topo += (topo.back() == '[' ? "" : ", ") + rec;
        void* q = nullptr;
        PCHK(hipIpcOpenMemHandle(&q, all[p].h, hipIpcMemLazyEnablePeerAccess));
        wins[p] = static_cast<char*>(q);
        opened.push_back(wins[p]);
      }
    } catch (std::exception& e) {
      why = e.what();
      ok = 0;
    }
  } else if (why.empty()) {
    why = "a peer rank could not create its window";
  }
  // every window is mapped (and its flags zeroed) before any rank's first collective
  std::vector<int32_t> oks(n);
  Network::Allgather(reinterpret_cast<char*>(&ok), sizeof(int32_t), reinterpret_cast<char*>(oks.data()));
  for (int p = 0; p < n; ++p) ok &= oks[p];
  if (!ok) {
    for (char* q : opened) (void)hipIpcCloseMemHandle(q);
    if (own != nullptr) (void)hipFree(own);
    Log::Fatal("peer device comm setup failed on rank %d: %s", rank,
               why.empty() ? "a peer rank could not map the windows" : why.c_str());
  }
  topo += "]}";
  {
    std::lock_guard<std::mutex> lk(g_topo_mu);
    g_topo = topo;
  }
  Log::Info("peer device comm topology: %s", topo.c_str());
  auto c = std::make_shared<PeerComm>(rank, n, wins, stage, timeout_s > 0 ? timeout_s : 60.0, 0);
  c->Own(own, opened);
  return c;
}

}  // namespace lgbm_amd

using namespace lgbm_amd;

extern "C" {

// one process per GPU: the peer comm over hipIpc-mapped windows (host Network initialised first)
int LGBM_AMD_PeerCommInit(int device_id, double timeout_s) {
  try {
    Network::SetDeviceComm(MakePeerIpcComm(device_id, timeout_s));
  } catch (std::exception& e) {
    Log::Warning("%s", e.what());
    return -1;
  }
  return 0;
}

// the topology this rank's peer comm found (JSON: bus ids, same device or link type and hop
// count per peer); *out_len gets the length, the text is truncated to `len` - 1 bytes
int LGBM_AMD_DeviceCommTopology(char* out, int len, int* out_len) {
  std::lock_guard<std::mutex> lk(g_topo_mu);
  if (out_len != nullptr) *out_len = static_cast<int>(g_topo.size());
  if (out != nullptr && len > 0) {
    const size_t n = std::min(static_cast<size_t>(len - 1), g_topo.size());
    std::memcpy(out, g_topo.data(), n);
    out[n] = '\0';
  }
  return 0;
}

// releases the device comm (peer or RCCL): every rank's kernels are done with every window
// before any window is unmapped or freed
int LGBM_AMD_DeviceCommFree() {
  try {
    if (Network::device_comm() != nullptr) {
      (void)hipDeviceSynchronize();
      if (Network::num_machines() > 1) {
        int dummy = 0;
        std::vector<int> sink(Network::num_machines());
        Network::Allgather(reinterpret_cast<char*>(&dummy), sizeof(int), reinterpret_cast<char*>(sink.data()));
      }
    }
    Network::SetDeviceComm(nullptr);
  } catch (std::exception& e) {
    Log::Warning("%s", e.what());
    Network::SetDeviceComm(nullptr);
    return -1;
  }
  return 0;
}

// microbenchmark of the current device comm (every rank calls it with the same arguments):
// kind 0 int64 reduce-scatter (bytes = the whole send buffer), 1 allgather (bytes per rank),
// 2 int64 all-reduce; `iters` back-to-back collectives, captured in one graph (graph != 0) or
// launched eagerly; *out_us = microseconds per collective
int LGBM_AMD_DeviceCommBench(int kind, int64_t bytes, int iters, int graph, double* out_us) {
  try {
    DeviceComm* dc = Network::device_comm();
    if (dc == nullptr) Log::Fatal("no device comm");
    const int n = dc->size();
    const size_t elems = std::max<size_t>(static_cast<size_t>(n), static_cast<size_t>(bytes) / 8 / n * n);
    void *send = nullptr, *recv = nullptr;
    PCHK(hipMalloc(&send, elems * 8 * (kind == 1 ? n : 1)));
    PCHK(hipMalloc(&recv, elems * 8 * (kind == 1 ? n : 1)));
    PCHK(hipMemset(send, 0, elems * 8 * (kind == 1 ? n : 1)));
    hipStream_t s;
    PCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    auto one = [&]() {
      if (kind == 0) {
        dc->ReduceScatterSumI64(static_cast<long long*>(send), static_cast<long long*>(recv), elems / n, s);
      } else if (kind == 1) {
        dc->Allgather(send, recv, elems * 8, s);
      } else {
        dc->AllreduceSumI64(static_cast<long long*>(send), elems, s);
      }
    };
    for (int i = 0; i < 5; ++i) one();
    PCHK(hipStreamSynchronize(s));
    hipGraphExec_t ge = nullptr;
    if (graph) {
      hipGraph_t g = nullptr;
      PCHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int i = 0; i < iters; ++i) one();
      PCHK(hipStreamEndCapture(s, &g));
      PCHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      (void)hipGraphDestroy(g);
      PCHK(hipGraphLaunch(ge, s));  // (warm: first launch uploads the graph)
      PCHK(hipStreamSynchronize(s));
    }
    hipEvent_t e0, e1;
    PCHK(hipEventCreate(&e0));
    PCHK(hipEventCreate(&e1));
    PCHK(hipEventRecord(e0, s));
    if (graph) {
      PCHK(hipGraphLaunch(ge, s));
    } else {
      for (int i = 0; i < iters; ++i) one();
    }
    PCHK(hipEventRecord(e1, s));
    PCHK(hipEventSynchronize(e1));
    float ms = 0.f;
    PCHK(hipEventElapsedTime(&ms, e0, e1));
    *out_us = 1000.0 * ms / std::max(1, iters);
    std::string err;
    if (dc->AsyncError(&err)) Log::Fatal("%s", err.c_str());
    if (ge != nullptr) (void)hipGraphExecDestroy(ge);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipStreamDestroy(s);
    (void)hipFree(send);
    (void)hipFree(recv);
  } catch (std::exception& e) {
    Log::Warning("%s", e.what());
    return -1;
  }
  return 0;
}

}  // extern "C"
