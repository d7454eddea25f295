// Built-in TCP full-mesh transport for `machines=` / `machine_list_filename` configs
// (reference: src/network/linkers_socket.cpp:23-232 -- machine list parsing, rank
// discovery by local address + port, lower rank connects to higher, retries with
// backoff).  Allgather is a direct exchange over the mesh (every rank sends its block
// to every peer); payloads here are control-plane sized (bin mappers, scalars), the
// per-split histogram traffic of GPU learners goes over RCCL instead.
#include <arpa/inet.h>
#include <ifaddrs.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <fstream>
#include <set>
#include <thread>

#include "lgbm_amd/common.h"
#include "lgbm_amd/log.h"
#include "lgbm_amd/network.h"

namespace lgbm_amd {

namespace {

struct Machine {
  std::string ip;
  int port;
};

std::vector<Machine> ParseMachines(const Config& cfg) {
  std::vector<std::string> lines;
  if (!cfg.machines.empty()) {
    lines = common::Split(cfg.machines.c_str(), ',');
  } else if (!cfg.machine_list_filename.empty()) {
    std::ifstream f(cfg.machine_list_filename);
    if (!f) Log::Fatal("Machine list file %s doesn't exist", cfg.machine_list_filename.c_str());
    std::string l;
    while (std::getline(f, l)) {
      l = common::Trim(l);
      if (!l.empty()) lines.push_back(l);
    }
  } else {
    Log::Fatal("Machine list file doesn't exist");
  }
  std::vector<Machine> out;
  for (auto& l : lines) {
    auto t = common::Split(common::Trim(l).c_str(), " :\t");
    if (t.size() < 2) continue;
    out.push_back({t[0], std::stoi(t[1])});
  }
  return out;
}

std::set<std::string> LocalIps() {
  std::set<std::string> ips = {"127.0.0.1", "localhost"};
  ifaddrs* ifa = nullptr;
  if (getifaddrs(&ifa) == 0) {
    for (ifaddrs* p = ifa; p; p = p->ifa_next) {
      if (p->ifa_addr && p->ifa_addr->sa_family == AF_INET) {
        char buf[INET_ADDRSTRLEN];
        inet_ntop(AF_INET, &reinterpret_cast<sockaddr_in*>(p->ifa_addr)->sin_addr, buf, sizeof(buf));
        ips.insert(buf);
      }
    }
    freeifaddrs(ifa);
  }
  return ips;
}

void SendAll(int fd, const char* p, size_t n) {
  while (n > 0) {
    ssize_t k = ::send(fd, p, n, 0);
    if (k <= 0) Log::Fatal("Socket send error");
    p += k;
    n -= static_cast<size_t>(k);
  }
}

void RecvAll(int fd, char* p, size_t n) {
  while (n > 0) {
    ssize_t k = ::recv(fd, p, n, 0);
    if (k <= 0) Log::Fatal("Socket recv error");
    p += k;
    n -= static_cast<size_t>(k);
  }
}

class TcpTransport : public HostTransport {
 public:
  explicit TcpTransport(const Config& cfg) {
    auto ms = ParseMachines(cfg);
    n_ = static_cast<int>(ms.size());
    if (n_ != cfg.num_machines) {
      Log::Warning("num_machines (%d) differs from the machine list (%d); using the list", cfg.num_machines, n_);
    }
    auto ips = LocalIps();
    rank_ = -1;
    for (int i = 0; i < n_; ++i) {
      if (ips.count(ms[i].ip) && ms[i].port == cfg.local_listen_port) { rank_ = i; break; }
    }
    if (rank_ < 0) Log::Fatal("Machine list file doesn't contain the local machine");
    fds_.assign(n_, -1);
    int lfd = ::socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = INADDR_ANY;
    a.sin_port = htons(static_cast<uint16_t>(cfg.local_listen_port));
    if (::bind(lfd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) {
      Log::Fatal("Binding port %d failed", cfg.local_listen_port);
    }
    ::listen(lfd, n_);
    // connect to higher ranks
    std::thread connector([&] {
      for (int p = rank_ + 1; p < n_; ++p) {
        int fd = -1;
        double wait_ms = 200;
        for (int attempt = 0; attempt < 20; ++attempt) {
          fd = ::socket(AF_INET, SOCK_STREAM, 0);
          sockaddr_in pa{};
          pa.sin_family = AF_INET;
          pa.sin_port = htons(static_cast<uint16_t>(ms[p].port));
          hostent* h = gethostbyname(ms[p].ip.c_str());
          if (h) std::memcpy(&pa.sin_addr, h->h_addr, h->h_length);
          if (::connect(fd, reinterpret_cast<sockaddr*>(&pa), sizeof(pa)) == 0) break;
          ::close(fd);
          fd = -1;
          std::this_thread::sleep_for(std::chrono::milliseconds(static_cast<int>(wait_ms)));
          wait_ms *= 1.3;
        }
        if (fd < 0) Log::Fatal("Connecting to rank %d failed", p);
        setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        int32_t me = rank_;
        SendAll(fd, reinterpret_cast<const char*>(&me), 4);
        fds_[p] = fd;
      }
    });
    for (int k = 0; k < rank_; ++k) {
      int fd = ::accept(lfd, nullptr, nullptr);
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      int32_t who = -1;
      RecvAll(fd, reinterpret_cast<char*>(&who), 4);
      if (who < 0 || who >= n_) Log::Fatal("Bad peer rank");
      fds_[who] = fd;
    }
    connector.join();
    ::close(lfd);
  }
  ~TcpTransport() override {
    for (int fd : fds_) {
      if (fd >= 0) ::close(fd);
    }
  }
  int rank() const override { return rank_; }
  int num_machines() const override { return n_; }
  void Allgather(const char* input, comm_size_t input_size, const comm_size_t* block_start,
                 const comm_size_t* block_len, char* output, comm_size_t output_size) override {
    (void)output_size;
    std::memcpy(output + block_start[rank_], input, input_size);
    // pairwise exchange ordered by rank to avoid deadlock: send in a thread, receive here
    std::thread sender([&] {
      for (int p = 0; p < n_; ++p) {
        if (p != rank_) SendAll(fds_[p], input, input_size);
      }
    });
    for (int p = 0; p < n_; ++p) {
      if (p != rank_) RecvAll(fds_[p], output + block_start[p], block_len[p]);
    }
    sender.join();
  }

 private:
  int n_ = 1;
  int rank_ = 0;
  std::vector<int> fds_;
};

}  // namespace

std::shared_ptr<HostTransport> MakeTcpTransport(const Config& cfg) { return std::make_shared<TcpTransport>(cfg); }

}  // namespace lgbm_amd
