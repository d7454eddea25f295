// Network facade: per-thread state (so tests can run several ranks as threads in one
// process, like the reference's THREAD_LOCAL Network, src/network/network.cpp:17-27),
// collectives built on a pluggable HostTransport.
#include "lgbm_amd/network.h"

#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <stdexcept>
#include <string>

#include "collectives.h"
#include "lgbm_amd/common.h"
#include "lgbm_amd/log.h"

namespace lgbm_amd {

std::shared_ptr<HostTransport> MakeTcpTransport(const Config& cfg);  // tcp_transport.cpp
std::shared_ptr<HostTransport> MakeMpiTransport(const Config& cfg);  // mpi_transport.cpp

namespace {

struct NetState {
  std::shared_ptr<HostTransport> transport;
  std::shared_ptr<DeviceComm> device;
};

NetState& State() {
  static thread_local NetState s;
  return s;
}

// an error the external collective functions reported through
// LGBM_AMD_NetworkReportExternalError while they ran on this thread (their C signature
// returns void, so a failing Python / MPI callback has no other way to stop the caller)
std::string& ReportedError() {
  static thread_local std::string msg;
  return msg;
}

void RaiseReported() {
  if (ReportedError().empty()) return;
  const std::string why = ReportedError();
  ReportedError().clear();
  Log::Fatal("external collective failed: %s", why.c_str());
}

// adapter for the reference's external function pair
class ExternalFnTransport : public HostTransport {
 public:
  ExternalFnTransport(int n, int r, ReduceScatterFunctionPtr rs, AllgatherFunctionPtr ag)
      : n_(n), r_(r), rs_(rs), ag_(ag) {}
  int rank() const override { return r_; }
  int num_machines() const override { return n_; }
  void Allgather(const char* input, comm_size_t input_size, const comm_size_t* block_start,
                 const comm_size_t* block_len, char* output, comm_size_t output_size) override {
    ag_(const_cast<char*>(input), input_size, block_start, block_len, n_, output, output_size);
    RaiseReported();
  }
  bool ReduceScatter(char* input, comm_size_t input_size, int type_size, const comm_size_t* block_start,
                     const comm_size_t* block_len, char* output, comm_size_t output_size,
                     const ReduceFunction& reducer) override {
    if (rs_ == nullptr) return false;
    // the external ABI takes a plain function pointer: route through a thread-local trampoline
    static thread_local const ReduceFunction* active = nullptr;
    active = &reducer;
    ReduceFunctionPtr tramp = [](const char* in, char* out, int ts, comm_size_t len) { (*active)(in, out, ts, len); };
    rs_(input, input_size, type_size, block_start, block_len, n_, output, output_size, tramp);
    active = nullptr;
    RaiseReported();
    return true;
  }

 private:
  int n_, r_;
  ReduceScatterFunctionPtr rs_;
  AllgatherFunctionPtr ag_;
};

// threads-as-ranks rendezvous.  A rank that fails (an exception inside a collective, or
// an injected fault) poisons the hub, so its peers raise instead of waiting forever; a
// rank that never arrives is detected by the per-collective timeout.  This is the
// in-process fake backend of SURVEY.md §5.3 (the reference only has socket timeouts).
struct ThreadHub {
  ThreadHub(int n, double timeout_s) : n(n), timeout_s(timeout_s), bufs(n), lens(n), mail(n * n) {}
  int n;
  double timeout_s;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  int generation = 0;
  int readers_done = 0;
  bool failed = false;
  std::string failure;
  std::vector<const char*> bufs;
  std::vector<comm_size_t> lens;
  // point-to-point mailboxes: mail[src * n + dst] holds the messages src sent to dst, in order
  std::vector<std::deque<std::vector<char>>> mail;
};

class ThreadTransport : public HostTransport {
 public:
  ThreadTransport(std::shared_ptr<ThreadHub> hub, int rank, int fail_at_call)
      : hub_(std::move(hub)), rank_(rank), fail_at_call_(fail_at_call) {}
  int rank() const override { return rank_; }
  int num_machines() const override { return hub_->n; }
  bool HasPointToPoint() const override { return true; }
  // eager buffered send into the (rank, to) mailbox, then wait for the (from, rank) one
  void SendRecv(int to, const char* send, comm_size_t send_len, int from, char* recv,
                comm_size_t recv_len) override {
    std::unique_lock<std::mutex> lk(hub_->mu);
    CountCall(&lk);
    if (send_len > 0) {
      hub_->mail[rank_ * hub_->n + to].emplace_back(send, send + send_len);
      hub_->cv.notify_all();
    }
    if (recv_len > 0) {
      auto& box = hub_->mail[from * hub_->n + rank_];
      Wait(&lk, [&] { return !box.empty(); });
      if (static_cast<comm_size_t>(box.front().size()) != recv_len) {
        Poison(&lk, "message size mismatch from rank " + std::to_string(from) + " to rank " + std::to_string(rank_));
      }
      std::memcpy(recv, box.front().data(), recv_len);
      box.pop_front();
    }
  }
  void Allgather(const char* input, comm_size_t input_size, const comm_size_t* block_start,
                 const comm_size_t* block_len, char* output, comm_size_t output_size) override {
    (void)output_size;
    std::unique_lock<std::mutex> lk(hub_->mu);
    CountCall(&lk);
    // wait until the previous round's readers are done
    Wait(&lk, [&] { return hub_->readers_done == 0 || hub_->readers_done == hub_->n; });
    if (hub_->readers_done == hub_->n) hub_->readers_done = 0;
    const int gen = hub_->generation;
    hub_->bufs[rank_] = input;
    hub_->lens[rank_] = input_size;
    if (++hub_->arrived == hub_->n) {
      hub_->arrived = 0;
      hub_->generation++;
      hub_->cv.notify_all();
    } else {
      Wait(&lk, [&] { return hub_->generation != gen; });
    }
    lk.unlock();
    for (int r = 0; r < hub_->n; ++r) std::memcpy(output + block_start[r], hub_->bufs[r], block_len[r]);
    lk.lock();
    hub_->readers_done++;
    hub_->cv.notify_all();
    // keep inputs alive until everyone has copied
    Wait(&lk, [&] { return hub_->readers_done == hub_->n || hub_->readers_done == 0; });
  }

 private:
  void CountCall(std::unique_lock<std::mutex>* lk) {
    ++calls_;
    if (fail_at_call_ > 0 && calls_ == fail_at_call_) {
      Poison(lk, "injected fault in rank " + std::to_string(rank_) + " at collective call " + std::to_string(calls_));
    }
  }
  [[noreturn]] void Poison(std::unique_lock<std::mutex>* lk, const std::string& why) {
    if (!hub_->failed) {
      hub_->failed = true;
      hub_->failure = why;
    }
    hub_->cv.notify_all();
    lk->unlock();
    Log::Fatal("%s", why.c_str());
    throw std::runtime_error(why);  // not reached
  }
  template <typename Pred>
  void Wait(std::unique_lock<std::mutex>* lk, Pred ready) {
    auto ok = [&] { return hub_->failed || ready(); };
    if (hub_->timeout_s > 0) {
      const auto limit = std::chrono::duration<double>(hub_->timeout_s);
      if (!hub_->cv.wait_for(*lk, limit, ok)) {
        Poison(lk, "collective timed out after " + std::to_string(hub_->timeout_s) + " s in rank " +
                       std::to_string(rank_) + " (a peer rank did not arrive)");
      }
    } else {
      hub_->cv.wait(*lk, ok);
    }
    if (hub_->failed) {
      const std::string why = hub_->failure;
      lk->unlock();
      Log::Fatal("peer rank failed: %s", why.c_str());
    }
  }

  std::shared_ptr<ThreadHub> hub_;
  int rank_;
  int fail_at_call_;
  int calls_ = 0;
};

// collective algorithm choice (bytes)
constexpr comm_size_t kRingAllgatherBytes = 8 << 20;  // Bruck below (log2 n rounds), ring above
constexpr comm_size_t kAllreduceSplitBytes = 4096;    // allgather + local reduce below

bool RankOrdered(int n, const comm_size_t* block_start, const comm_size_t* block_len) {
  for (int i = 1; i < n; ++i) {
    if (block_start[i] != block_start[i - 1] + block_len[i - 1]) return false;
  }
  return true;
}

}  // namespace

std::vector<std::shared_ptr<HostTransport>> MakeThreadTransports(int num_ranks, double timeout_s, int fail_rank,
                                                                 int fail_at_call) {
  auto hub = std::make_shared<ThreadHub>(num_ranks, timeout_s);
  std::vector<std::shared_ptr<HostTransport>> out;
  for (int r = 0; r < num_ranks; ++r) {
    out.push_back(std::make_shared<ThreadTransport>(hub, r, r == fail_rank ? fail_at_call : 0));
  }
  return out;
}

void Network::Init(const Config& cfg) {
  if (cfg.num_machines <= 1) return;
  State().transport = MpiSelected() ? MakeMpiTransport(cfg) : MakeTcpTransport(cfg);
  Log::Info("Local rank: %d, total number of machines: %d", rank(), num_machines());
}

void Network::InitWithTransport(std::shared_ptr<HostTransport> t) { State().transport = std::move(t); }

void Network::InitWithFunctions(int num_machines, int rank, ReduceScatterFunctionPtr rs, AllgatherFunctionPtr ag) {
  if (num_machines <= 1) {
    State().transport.reset();
    return;
  }
  if (ag == nullptr) Log::Fatal("An allgather function is required");
  State().transport = std::make_shared<ExternalFnTransport>(num_machines, rank, rs, ag);
}

void Network::ReportExternalError(const std::string& msg) { ReportedError() = msg.empty() ? "unknown error" : msg; }

void Network::Dispose() {
  State().transport.reset();
  State().device.reset();
}

int Network::rank() { return State().transport ? State().transport->rank() : 0; }
int Network::num_machines() { return State().transport ? State().transport->num_machines() : 1; }

void Network::SetDeviceComm(std::shared_ptr<DeviceComm> c) { State().device = std::move(c); }
DeviceComm* Network::device_comm() { return State().device.get(); }

void Network::Allgather(char* input, comm_size_t send_size, char* output) {
  const int n = num_machines();
  if (n <= 1) {
    std::memcpy(output, input, send_size);
    return;
  }
  std::vector<comm_size_t> start(n), len(n, send_size);
  for (int i = 0; i < n; ++i) start[i] = i * send_size;
  Allgather(input, start.data(), len.data(), output, send_size * n);
}

void Network::Allgather(char* input, const comm_size_t* block_start, const comm_size_t* block_len, char* output,
                        comm_size_t all_size) {
  if (num_machines() <= 1) {
    std::memcpy(output, input, block_len[0]);
    return;
  }
  HostTransport* t = State().transport.get();
  if (!t->HasPointToPoint()) {
    t->Allgather(input, block_len[rank()], block_start, block_len, output, all_size);
  } else if (all_size <= kRingAllgatherBytes) {
    collectives::BruckAllgather(t, input, block_start, block_len, output);
  } else {
    collectives::RingAllgather(t, input, block_start, block_len, output);
  }
}

void Network::ReduceScatter(char* input, comm_size_t input_size, int type_size, const comm_size_t* block_start,
                            const comm_size_t* block_len, char* output, comm_size_t output_size,
                            const ReduceFunction& reducer) {
  const int n = num_machines();
  const int r = rank();
  if (n <= 1) {
    std::memcpy(output, input, input_size);
    return;
  }
  HostTransport* t = State().transport.get();
  if (t->HasPointToPoint() && RankOrdered(n, block_start, block_len)) {
    if ((n & (n - 1)) == 0) {
      collectives::RecursiveHalvingReduceScatter(t, input, input_size, type_size, block_start, block_len, output,
                                                 reducer);
    } else {
      collectives::RingReduceScatter(t, input, input_size, type_size, block_start, block_len, output, reducer);
    }
    return;
  }
  if (t->ReduceScatter(input, input_size, type_size, block_start, block_len, output, output_size, reducer)) {
    return;
  }
  // allgather every rank's full input, reduce own block locally
  std::vector<comm_size_t> st(n), ln(n, input_size);
  for (int i = 0; i < n; ++i) st[i] = i * input_size;
  std::vector<char> all(static_cast<size_t>(input_size) * n);
  State().transport->Allgather(input, input_size, st.data(), ln.data(), all.data(), input_size * n);
  // fixed rank order (0, 1, ..., n-1) so the reduced block is independent of who reduces it
  std::memcpy(output, all.data() + block_start[r], block_len[r]);
  for (int i = 1; i < n; ++i) {
    reducer(all.data() + static_cast<size_t>(i) * input_size + block_start[r], output, type_size, block_len[r]);
  }
}

void Network::Allreduce(char* input, comm_size_t input_size, int type_size, char* output,
                        const ReduceFunction& reducer) {
  const int n = num_machines();
  if (n <= 1) {
    if (output != input) std::memcpy(output, input, input_size);
    return;
  }
  const comm_size_t items = input_size / type_size;
  if (State().transport->HasPointToPoint() && input_size >= kAllreduceSplitBytes && items >= n) {
    // reduce-scatter over n item-aligned blocks, then allgather them: each block is reduced
    // by exactly one rank, so every rank still ends with bitwise identical results
    std::vector<comm_size_t> st(n), ln(n);
    for (int i = 0; i < n; ++i) {
      st[i] = static_cast<comm_size_t>(items * i / n) * type_size;
      ln[i] = static_cast<comm_size_t>(items * (i + 1) / n) * type_size - st[i];
    }
    std::vector<char> mine(static_cast<size_t>(ln[rank()]));
    ReduceScatter(input, input_size, type_size, st.data(), ln.data(), mine.data(), ln[rank()], reducer);
    Allgather(mine.data(), st.data(), ln.data(), output, input_size);
    return;
  }
  // small payloads: allgather + fixed-order local reduce (bitwise identical on every rank)
  std::vector<comm_size_t> st(n), ln(n, input_size);
  for (int i = 0; i < n; ++i) st[i] = i * input_size;
  std::vector<char> all(static_cast<size_t>(input_size) * n);
  State().transport->Allgather(input, input_size, st.data(), ln.data(), all.data(), input_size * n);
  std::memcpy(output, all.data(), input_size);
  for (int i = 1; i < n; ++i) reducer(all.data() + static_cast<size_t>(i) * input_size, output, type_size, input_size);
}

}  // namespace lgbm_amd
