// In-process device communicator: ranks are threads of one process sharing one GPU, each
// with its own stream.  Every collective is a host rendezvous of the rank threads (their
// streams drained first), then device work on the caller's stream: the reductions run as a
// kernel that reads every rank's input buffer directly (dev::ReducePeers), gathers and
// broadcasts as device-to-device copies.  A second rendezvous keeps the inputs alive until
// every rank has read them.  It lets `pytest -m gpu` run the data- / feature-parallel
// device learners -- their collective sequence, owner-blocked reduce-scatter and gathered
// split records -- on a single MI355X; RCCL (rccl_comm.cpp) is the multi-GPU backend.
// Failure handling follows the host thread hub (network.cpp): a rank that fails or times
// out poisons the hub and its peers raise instead of waiting.
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../device/kernels.h"
#include "lgbm_amd/log.h"
#include "lgbm_amd/network.h"

namespace lgbm_amd {

namespace {

#define HIPCK(x)                                                                                  \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) Log::Fatal("HIP error %s at %s:%d: %s", #x, __FILE__, __LINE__, hipGetErrorString(e_)); \
  } while (0)

struct DeviceHub {
  DeviceHub(int n, double timeout_s) : n(n), timeout_s(timeout_s), ptrs(n, nullptr) {}
  int n;
  double timeout_s;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  long long generation = 0;
  bool failed = false;
  std::string failure;
  std::vector<const void*> ptrs;
};

class ThreadDeviceComm : public DeviceComm {
 public:
  ThreadDeviceComm(std::shared_ptr<DeviceHub> hub, int rank, int fail_at_call)
      : hub_(std::move(hub)), rank_(rank), fail_at_call_(fail_at_call) {}
  ~ThreadDeviceComm() override {
    if (tmp_ != nullptr) (void)hipFree(tmp_);
  }
  int rank() const override { return rank_; }
  int size() const override { return hub_->n; }
  bool CaptureSafe() const override { return false; }

  void AllreduceSumF64(double* buf, size_t count, void* stream) override {
    Reduce(buf, buf, 0, count, sizeof(double), dev::kPeerSumF64, stream);
  }
  void AllreduceSumF32(float* buf, size_t count, void* stream) override {
    Reduce(buf, buf, 0, count, sizeof(float), dev::kPeerSumF32, stream);
  }
  void AllreduceSumI64(long long* buf, size_t count, void* stream) override {
    Reduce(buf, buf, 0, count, sizeof(long long), dev::kPeerSumI64, stream);
  }
  void AllreduceMaxU32(uint32_t* buf, size_t count, void* stream) override {
    Reduce(buf, buf, 0, count, sizeof(uint32_t), dev::kPeerMaxU32, stream);
  }
  void ReduceScatterSumF64(const double* send, double* recv, size_t recv_count, void* stream) override {
    Reduce(send, recv, recv_count * rank_, recv_count, sizeof(double), dev::kPeerSumF64, stream);
  }
  void ReduceScatterSumI64(const long long* send, long long* recv, size_t recv_count, void* stream) override {
    Reduce(send, recv, recv_count * rank_, recv_count, sizeof(long long), dev::kPeerSumI64, stream);
  }
  void Allgather(const void* send, void* recv, size_t bytes_per_rank, void* stream) override {
    Enter();
    hipStream_t s = static_cast<hipStream_t>(stream);
    HIPCK(hipStreamSynchronize(s));
    Rendezvous(send);
    for (int r = 0; r < hub_->n; ++r) {
      char* dst = static_cast<char*>(recv) + bytes_per_rank * r;
      if (dst != hub_->ptrs[r]) HIPCK(hipMemcpyAsync(dst, hub_->ptrs[r], bytes_per_rank, hipMemcpyDeviceToDevice, s));
    }
    HIPCK(hipStreamSynchronize(s));
    Rendezvous(nullptr);  // every rank has copied: the inputs may change again
  }
  void Broadcast(void* buf, size_t bytes, int root, void* stream) override {
    Enter();
    hipStream_t s = static_cast<hipStream_t>(stream);
    HIPCK(hipStreamSynchronize(s));
    Rendezvous(buf);
    if (rank_ != root) HIPCK(hipMemcpyAsync(buf, hub_->ptrs[root], bytes, hipMemcpyDeviceToDevice, s));
    HIPCK(hipStreamSynchronize(s));
    Rendezvous(nullptr);
  }
  bool AsyncError(std::string* msg) override {
    std::lock_guard<std::mutex> lk(hub_->mu);
    if (!hub_->failed) return false;
    *msg = hub_->failure;
    return true;
  }
  void Abort() override {
    std::lock_guard<std::mutex> lk(hub_->mu);
    if (!hub_->failed) {
      hub_->failed = true;
      hub_->failure = "rank " + std::to_string(rank_) + " aborted the device communicator";
    }
    hub_->cv.notify_all();
  }

 private:
  // out = op over the ranks of in[offset, +count): into a private buffer first (in-place
  // all-reduces overwrite inputs the peers still read), then copied out after the second
  // rendezvous
  void Reduce(const void* in, void* out, size_t offset, size_t count, size_t elem, int op, void* stream) {
    Enter();
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (hub_->n > dev::kMaxPeerBufs) Log::Fatal("in-process device comm supports at most %d ranks", dev::kMaxPeerBufs);
    EnsureTmp(count * elem);
    HIPCK(hipStreamSynchronize(s));
    Rendezvous(in);
    dev::PeerBufs pb{};
    for (int r = 0; r < hub_->n; ++r) pb.p[r] = hub_->ptrs[r];
    if (count > 0) dev::ReducePeers(pb, hub_->n, offset, tmp_, count, op, s);
    HIPCK(hipStreamSynchronize(s));
    Rendezvous(nullptr);
    if (count > 0) HIPCK(hipMemcpyAsync(out, tmp_, count * elem, hipMemcpyDeviceToDevice, s));
  }
  // a collective starts: the injected fault fires before any peer buffer is touched
  void Enter() {
    ++calls_;
    if (fail_at_call_ <= 0 || calls_ != fail_at_call_) return;
    std::string why = "injected fault in rank " + std::to_string(rank_) + " at device collective call " +
                      std::to_string(calls_);
    {
      std::lock_guard<std::mutex> lk(hub_->mu);
      if (!hub_->failed) {
        hub_->failed = true;
        hub_->failure = why;
      }
      hub_->cv.notify_all();
    }
    Log::Fatal("device collective failed: %s", why.c_str());
  }
  void EnsureTmp(size_t bytes) {
    if (bytes <= tmp_bytes_) return;
    if (tmp_ != nullptr) HIPCK(hipFree(tmp_));
    HIPCK(hipMalloc(&tmp_, bytes));
    tmp_bytes_ = bytes;
  }
  // publish `p` (if not null) and wait for every rank
  void Rendezvous(const void* p) {
    std::unique_lock<std::mutex> lk(hub_->mu);
    if (p != nullptr) hub_->ptrs[rank_] = p;
    const long long gen = hub_->generation;
    if (++hub_->arrived == hub_->n) {
      hub_->arrived = 0;
      hub_->generation++;
      hub_->cv.notify_all();
    } else {
      auto ready = [&] { return hub_->failed || hub_->generation != gen; };
      if (hub_->timeout_s > 0) {
        if (!hub_->cv.wait_for(lk, std::chrono::duration<double>(hub_->timeout_s), ready)) {
          hub_->failed = true;
          hub_->failure = "device collective timed out after " + std::to_string(hub_->timeout_s) + " s in rank " +
                          std::to_string(rank_) + " (a peer rank did not arrive)";
          hub_->cv.notify_all();
        }
      } else {
        hub_->cv.wait(lk, ready);
      }
    }
    if (hub_->failed) {
      const std::string why = hub_->failure;
      lk.unlock();
      Log::Fatal("device collective failed: %s", why.c_str());
    }
  }

  std::shared_ptr<DeviceHub> hub_;
  int rank_;
  int fail_at_call_;
  long long calls_ = 0;
  void* tmp_ = nullptr;
  size_t tmp_bytes_ = 0;
};

}  // namespace

std::vector<std::shared_ptr<DeviceComm>> MakeThreadDeviceComms(int num_ranks, double timeout_s, int fail_rank,
                                                               int fail_at_call) {
  auto hub = std::make_shared<DeviceHub>(num_ranks, timeout_s);
  std::vector<std::shared_ptr<DeviceComm>> out;
  for (int r = 0; r < num_ranks; ++r) {
    out.push_back(std::make_shared<ThreadDeviceComm>(hub, r, r == fail_rank ? fail_at_call : 0));
  }
  return out;
}

}  // namespace lgbm_amd
