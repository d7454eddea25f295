// MPI host transport (reference src/network/linkers_mpi.cpp: MPI_Init_thread(SERIALIZED) when
// MPI is not running yet, rank / size of MPI_COMM_WORLD, a start-up barrier, Finalize at a
// normal exit and Abort after an error).
//
// The reference links MPI at build time (USE_MPI).  Here the library is opened at run time,
// so one build serves MPI and non-MPI launches and no MPI headers are needed to compile:
//   LGBM_AMD_NETWORK=mpi        selects this transport in Network::Init (CLI / LGBM_NetworkInit)
//   LGBM_AMD_MPI_LIB=<path>     the MPI library (default: libmpi.so.40, libmpi.so.12, libmpi.so,
//                               libmpich.so.12 -- whichever dlopen finds first)
// Both ABI families are handled: Open MPI's handles are the addresses of its predefined objects
// (ompi_mpi_comm_world, ompi_mpi_byte); the MPICH ABI (MPICH, Intel MPI, MVAPICH, Cray) uses
// fixed integer handles.  Handles are passed as intptr_t: an int handle travels in the low half
// of the same argument register.
//
// The transport is point-to-point (MPI_Sendrecv), so Network runs its own Bruck / recursive-
// halving / ring algorithms over it exactly as over the TCP mesh; the variable-size allgather
// is MPI_Allgatherv.
#include <dlfcn.h>

#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

#include "lgbm_amd/log.h"
#include "lgbm_amd/network.h"
#include "lgbm_amd/tuning.h"

namespace lgbm_amd {

namespace {

using Handle = intptr_t;
constexpr int kThreadSerialized = 2;  // MPI_THREAD_SERIALIZED in both ABI families
constexpr Handle kMpichCommWorld = 0x44000000;
constexpr Handle kMpichByte = 0x4c00010d;

struct MpiLib {
  void* dl = nullptr;
  Handle comm_world = 0, byte = 0;
  bool started_here = false;  // this process called MPI_Init_thread
  int (*Initialized)(int*) = nullptr;
  int (*Finalized)(int*) = nullptr;
  int (*InitThread)(int*, char***, int, int*) = nullptr;
  int (*CommSize)(Handle, int*) = nullptr;
  int (*CommRank)(Handle, int*) = nullptr;
  int (*Barrier)(Handle) = nullptr;
  int (*Sendrecv)(const void*, int, Handle, int, int, void*, int, Handle, int, int, Handle, void*) = nullptr;
  int (*Allgatherv)(const void*, int, Handle, void*, const int*, const int*, Handle, Handle) = nullptr;
  int (*Finalize)() = nullptr;
  int (*Abort)(Handle, int) = nullptr;
};

std::mutex g_mpi_mu;
MpiLib* g_mpi = nullptr;  // opened once per process, never closed (MPI cannot be re-initialised)

template <typename F>
void Sym(void* dl, const char* name, F* out) {
  void* p = dlsym(dl, name);
  if (p == nullptr) Log::Fatal("MPI library lacks %s", name);
  *out = reinterpret_cast<F>(p);
}

MpiLib* OpenMpi() {
  std::lock_guard<std::mutex> lk(g_mpi_mu);
  if (g_mpi != nullptr) return g_mpi;
  std::vector<std::string> names;
  if (const char* e = tuning::Get(tuning::Knob::MpiLib)) names.push_back(e);
  for (const char* n : {"libmpi.so.40", "libmpi.so.12", "libmpi.so", "libmpich.so.12"}) names.push_back(n);
  void* dl = nullptr;
  std::string tried;
  for (const auto& n : names) {
    dl = dlopen(n.c_str(), RTLD_NOW | RTLD_GLOBAL);
    if (dl != nullptr) break;
    tried += (tried.empty() ? "" : ", ") + n;
  }
  if (dl == nullptr) {
    Log::Fatal("LGBM_AMD_NETWORK=mpi: no MPI library could be opened (tried %s); set LGBM_AMD_MPI_LIB", tried.c_str());
  }
  auto* m = new MpiLib();
  m->dl = dl;
  if (void* cw = dlsym(dl, "ompi_mpi_comm_world")) {  // Open MPI: handles are object addresses
    void* by = dlsym(dl, "ompi_mpi_byte");
    if (by == nullptr) Log::Fatal("Open MPI library without ompi_mpi_byte");
    m->comm_world = reinterpret_cast<Handle>(cw);
    m->byte = reinterpret_cast<Handle>(by);
  } else {
    m->comm_world = kMpichCommWorld;
    m->byte = kMpichByte;
  }
  Sym(dl, "MPI_Initialized", &m->Initialized);
  Sym(dl, "MPI_Finalized", &m->Finalized);
  Sym(dl, "MPI_Init_thread", &m->InitThread);
  Sym(dl, "MPI_Comm_size", &m->CommSize);
  Sym(dl, "MPI_Comm_rank", &m->CommRank);
  Sym(dl, "MPI_Barrier", &m->Barrier);
  Sym(dl, "MPI_Sendrecv", &m->Sendrecv);
  Sym(dl, "MPI_Allgatherv", &m->Allgatherv);
  Sym(dl, "MPI_Finalize", &m->Finalize);
  Sym(dl, "MPI_Abort", &m->Abort);
  g_mpi = m;
  return m;
}

void Check(int rc, const char* what) {
  if (rc != 0) Log::Fatal("MPI error %d in %s", rc, what);
}

class MpiTransport : public HostTransport {
 public:
  explicit MpiTransport(MpiLib* m) : m_(m) {
    int flag = 0;
    Check(m_->Initialized(&flag), "MPI_Initialized");
    if (!flag) {
      int argc = 0, provided = 0;
      char** argv = nullptr;
      Check(m_->InitThread(&argc, &argv, kThreadSerialized, &provided), "MPI_Init_thread");
      m_->started_here = true;
    }
    Check(m_->CommSize(m_->comm_world, &size_), "MPI_Comm_size");
    Check(m_->CommRank(m_->comm_world, &rank_), "MPI_Comm_rank");
    Check(m_->Barrier(m_->comm_world), "MPI_Barrier");  // every rank is up
  }
  int rank() const override { return rank_; }
  int num_machines() const override { return size_; }
  bool HasPointToPoint() const override { return true; }
  void SendRecv(int to, const char* send, comm_size_t send_len, int from, char* recv, comm_size_t recv_len) override {
    // (comm_size_t is 32-bit: every message fits one MPI count)
    alignas(16) char status[64];  // (large enough for either ABI's MPI_Status)
    Check(m_->Sendrecv(send, send_len, m_->byte, to, kTag, recv, recv_len, m_->byte, from, kTag, m_->comm_world, status),
          "MPI_Sendrecv");
  }
  void Allgather(const char* input, comm_size_t input_size, const comm_size_t* block_start,
                 const comm_size_t* block_len, char* output, comm_size_t output_size) override {
    std::vector<int> counts(size_), displs(size_);
    for (int r = 0; r < size_; ++r) {
      counts[r] = block_len[r];
      displs[r] = block_start[r];
    }
    (void)output_size;
    Check(m_->Allgatherv(input, input_size, m_->byte, output, counts.data(), displs.data(), m_->byte, m_->comm_world),
          "MPI_Allgatherv");
  }

 private:
  static constexpr int kTag = 0x4c47;
  MpiLib* m_;
  int rank_ = 0, size_ = 1;
};

}  // namespace

std::shared_ptr<HostTransport> MakeMpiTransport(const Config& cfg) {
  auto t = std::make_shared<MpiTransport>(OpenMpi());
  if (cfg.num_machines > 1 && cfg.num_machines != t->num_machines()) {
    Log::Warning("num_machines=%d but MPI_COMM_WORLD has %d ranks; using %d", cfg.num_machines, t->num_machines(),
                 t->num_machines());
  }
  return t;
}

bool MpiSelected() {
  const char* e = tuning::Get(tuning::Knob::Network);
  return e != nullptr && std::string(e) == "mpi";
}

void MpiFinalizeIfStarted() {
  std::lock_guard<std::mutex> lk(g_mpi_mu);
  if (g_mpi == nullptr || !g_mpi->started_here) return;
  int fin = 0;
  g_mpi->Finalized(&fin);
  if (!fin) {
    Log::Debug("Finalizing MPI session.");
    g_mpi->Finalize();
  }
}

void MpiAbortIfStarted() {
  std::lock_guard<std::mutex> lk(g_mpi_mu);
  if (g_mpi == nullptr) return;
  int init = 0, fin = 0;
  g_mpi->Initialized(&init);
  g_mpi->Finalized(&fin);
  if (init && !fin) {
    fprintf(stderr, "Aborting MPI communication.\n");
    g_mpi->Abort(g_mpi->comm_world, -1);
  }
}

}  // namespace lgbm_amd
