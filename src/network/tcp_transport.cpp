// Built-in TCP full-mesh transport for `machines=` / `machine_list_filename` configs
// (reference: src/network/linkers_socket.cpp:23-232 -- machine list parsing, rank
// discovery by local address + port, lower rank connects to higher, retries with
// backoff).
//
// The transport only provides a point-to-point primitive, SendRecv (send to one peer while
// receiving from another, driven by one poll() loop on the calling thread); the collective
// algorithms (Bruck / ring allgather, recursive-halving / ring reduce-scatter) live in
// collectives.cpp.  No helper threads: every socket error, peer hang-up or timeout raises
// on the caller's thread, so a failing peer turns into an error return of the C API on the
// surviving ranks (tests/test_network.py kills a rank mid-training).  Payloads here are
// control-plane sized (bin mappers, split records, CPU-learner histograms); the per-split
// histogram traffic of the GPU learners goes over RCCL.
#include <arpa/inet.h>
#include <fcntl.h>
#include <ifaddrs.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
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

// owned socket descriptors: closed when the transport (or its half-built constructor) goes away
struct Sockets {
  std::vector<int> fds;
  int listen_fd = -1;
  ~Sockets() {
    for (int fd : fds) {
      if (fd >= 0) ::close(fd);
    }
    if (listen_fd >= 0) ::close(listen_fd);
  }
};

void SetNoDelay(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

// blocking exact-size IO used only during the handshake
void WriteExact(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n > 0) {
    const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) Log::Fatal("Socket send error during connection setup (%s)", std::strerror(errno));
    c += k;
    n -= static_cast<size_t>(k);
  }
}

void ReadExact(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n > 0) {
    const ssize_t k = ::recv(fd, c, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) Log::Fatal("Socket recv error during connection setup");
    c += k;
    n -= static_cast<size_t>(k);
  }
}

class TcpTransport : public HostTransport {
 public:
  explicit TcpTransport(const Config& cfg) {
    const auto ms = ParseMachines(cfg);
    n_ = static_cast<int>(ms.size());
    if (n_ != cfg.num_machines) {
      Log::Warning("num_machines (%d) differs from the machine list (%d); using the list", cfg.num_machines, n_);
    }
    const auto ips = LocalIps();
    rank_ = -1;
    for (int i = 0; i < n_; ++i) {
      if (ips.count(ms[i].ip) && ms[i].port == cfg.local_listen_port) {
        rank_ = i;
        break;
      }
    }
    if (rank_ < 0) Log::Fatal("Machine list file doesn't contain the local machine");
    timeout_ms_ = cfg.time_out > 0 ? static_cast<int64_t>(cfg.time_out) * 60 * 1000 : -1;
    sock_.fds.assign(n_, -1);
    Listen(cfg.local_listen_port);
    // connect to every higher rank first: their listen sockets complete the connection from the
    // backlog even before they call accept(), so no rank waits on another's progress
    for (int p = rank_ + 1; p < n_; ++p) {
      const int fd = Connect(ms[p], p);
      const int32_t me = rank_;
      WriteExact(fd, &me, sizeof(me));
      sock_.fds[p] = fd;
    }
    for (int k = 0; k < rank_; ++k) {
      if (!WaitReadable(sock_.listen_fd)) Log::Fatal("Timed out waiting for lower ranks to connect");
      const int fd = ::accept(sock_.listen_fd, nullptr, nullptr);
      if (fd < 0) Log::Fatal("accept() failed (%s)", std::strerror(errno));
      SetNoDelay(fd);
      int32_t who = -1;
      ReadExact(fd, &who, sizeof(who));
      if (who < 0 || who >= rank_ || sock_.fds[who] >= 0) {
        ::close(fd);
        Log::Fatal("Bad peer rank %d in connection handshake", who);
      }
      sock_.fds[who] = fd;
    }
    ::close(sock_.listen_fd);
    sock_.listen_fd = -1;
    for (int p = 0; p < n_; ++p) {
      if (p != rank_) fcntl(sock_.fds[p], F_SETFL, fcntl(sock_.fds[p], F_GETFL) | O_NONBLOCK);
    }
  }

  int rank() const override { return rank_; }
  int num_machines() const override { return n_; }
  bool HasPointToPoint() const override { return true; }

  void SendRecv(int to, const char* send, comm_size_t send_len, int from, char* recv,
                comm_size_t recv_len) override {
    const int sfd = send_len > 0 ? sock_.fds[to] : -1;
    const int rfd = recv_len > 0 ? sock_.fds[from] : -1;
    size_t sent = 0, got = 0;
    const size_t slen = static_cast<size_t>(send_len), rlen = static_cast<size_t>(recv_len);
    while (sent < slen || got < rlen) {
      pollfd pf[2];
      int np = 0, si = -1, ri = -1;
      if (sent < slen && sfd == rfd && got < rlen) {
        pf[np] = {sfd, static_cast<short>(POLLOUT | POLLIN), 0};
        si = ri = np++;
      } else {
        if (sent < slen) {
          pf[np] = {sfd, POLLOUT, 0};
          si = np++;
        }
        if (got < rlen) {
          pf[np] = {rfd, POLLIN, 0};
          ri = np++;
        }
      }
      const int rc = ::poll(pf, np, timeout_ms_ > 0 ? static_cast<int>(std::min<int64_t>(timeout_ms_, 1 << 30)) : -1);
      if (rc < 0 && errno == EINTR) continue;
      if (rc < 0) Log::Fatal("poll() failed in a collective (%s)", std::strerror(errno));
      if (rc == 0) Log::Fatal("Collective timed out after %d minutes waiting for rank %d", static_cast<int>(timeout_ms_ / 60000),
                              got < rlen ? from : to);
      if (si >= 0 && sent < slen && (pf[si].revents & (POLLOUT | POLLERR | POLLHUP))) {
        const ssize_t k = ::send(sfd, send + sent, slen - sent, MSG_NOSIGNAL);
        if (k > 0) {
          sent += static_cast<size_t>(k);
        } else if (k < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) {
          Log::Fatal("Lost connection to rank %d while sending (%s)", to, std::strerror(errno));
        }
      }
      if (ri >= 0 && got < rlen && (pf[ri].revents & (POLLIN | POLLERR | POLLHUP))) {
        const ssize_t k = ::recv(rfd, recv + got, rlen - got, 0);
        if (k > 0) {
          got += static_cast<size_t>(k);
        } else if (k == 0) {
          Log::Fatal("Rank %d closed the connection during a collective", from);
        } else if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) {
          Log::Fatal("Lost connection to rank %d while receiving (%s)", from, std::strerror(errno));
        }
      }
    }
  }

  // direct exchange: every rank sends its block to every peer (used for tiny payloads where
  // one round beats log2(n) rounds); pairs are scheduled as n-1 shifted SendRecv rounds
  void Allgather(const char* input, comm_size_t input_size, const comm_size_t* block_start,
                 const comm_size_t* block_len, char* output, comm_size_t output_size) override {
    (void)output_size;
    std::memcpy(output + block_start[rank_], input, input_size);
    for (int s = 1; s < n_; ++s) {
      const int to = (rank_ + s) % n_, from = (rank_ - s + n_) % n_;
      SendRecv(to, input, input_size, from, output + block_start[from], block_len[from]);
    }
  }

 private:
  void Listen(int port) {
    sock_.listen_fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (sock_.listen_fd < 0) Log::Fatal("socket() failed (%s)", std::strerror(errno));
    int one = 1;
    setsockopt(sock_.listen_fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = INADDR_ANY;
    a.sin_port = htons(static_cast<uint16_t>(port));
    if (::bind(sock_.listen_fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) {
      Log::Fatal("Binding port %d failed (%s)", port, std::strerror(errno));
    }
    if (::listen(sock_.listen_fd, std::max(n_, 8)) != 0) Log::Fatal("listen() failed (%s)", std::strerror(errno));
  }

  // connect with retries (the peer may not be listening yet), backoff x1.3 from 200 ms
  int Connect(const Machine& m, int peer) {
    sockaddr_in pa{};
    pa.sin_family = AF_INET;
    pa.sin_port = htons(static_cast<uint16_t>(m.port));
    addrinfo hints{};
    hints.ai_family = AF_INET;
    addrinfo* res = nullptr;
    if (getaddrinfo(m.ip.c_str(), nullptr, &hints, &res) != 0 || res == nullptr) {
      Log::Fatal("Cannot resolve the address of rank %d (%s)", peer, m.ip.c_str());
    }
    pa.sin_addr = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
    freeaddrinfo(res);
    double wait_ms = 200;
    for (int attempt = 0; attempt < 20; ++attempt) {
      const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
      if (fd < 0) Log::Fatal("socket() failed (%s)", std::strerror(errno));
      if (::connect(fd, reinterpret_cast<sockaddr*>(&pa), sizeof(pa)) == 0) {
        SetNoDelay(fd);
        return fd;
      }
      ::close(fd);
      std::this_thread::sleep_for(std::chrono::milliseconds(static_cast<int>(wait_ms)));
      wait_ms *= 1.3;
    }
    Log::Fatal("Connecting to rank %d (%s:%d) failed", peer, m.ip.c_str(), m.port);
    return -1;  // not reached
  }

  bool WaitReadable(int fd) {
    pollfd pf{fd, POLLIN, 0};
    for (;;) {
      const int rc = ::poll(&pf, 1, timeout_ms_ > 0 ? static_cast<int>(std::min<int64_t>(timeout_ms_, 1 << 30)) : -1);
      if (rc < 0 && errno == EINTR) continue;
      return rc > 0;
    }
  }

  int n_ = 1;
  int rank_ = 0;
  int64_t timeout_ms_ = -1;
  Sockets sock_;
};

}  // namespace

std::shared_ptr<HostTransport> MakeTcpTransport(const Config& cfg) { return std::make_shared<TcpTransport>(cfg); }

}  // namespace lgbm_amd
