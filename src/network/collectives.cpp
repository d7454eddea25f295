// Host collective algorithms over HostTransport::SendRecv (see collectives.h).
#include <cstring>
#include "collectives.h"

#include <algorithm>
#include <vector>

namespace lgbm_amd {
namespace collectives {

void BruckAllgather(HostTransport* t, const char* input, const comm_size_t* block_start,
                    const comm_size_t* block_len, char* output) {
  const int n = t->num_machines(), r = t->rank();
  // work holds the blocks of ranks r, r+1, ... (mod n) back to back
  std::vector<comm_size_t> rot_off(n + 1, 0);
  for (int i = 0; i < n; ++i) rot_off[i + 1] = rot_off[i] + block_len[(r + i) % n];
  std::vector<char> work(static_cast<size_t>(rot_off[n]));
  std::memcpy(work.data(), input, block_len[r]);
  int have = 1;
  for (int d = 1; d < n; d <<= 1) {
    const int m = std::min(d, n - have);
    const int to = (r - d + n) % n, from = (r + d) % n;
    // my first m blocks go to rank r-d, whose blocks d..d+m-1 they are; rank r+d's first m
    // blocks are my blocks have..have+m-1 (have == d)
    const comm_size_t send_len = rot_off[m];
    comm_size_t recv_len = 0;
    for (int i = 0; i < m; ++i) recv_len += block_len[(from + i) % n];
    t->SendRecv(to, work.data(), send_len, from, work.data() + rot_off[have], recv_len);
    have += m;
  }
  for (int i = 0; i < n; ++i) {
    const int owner = (r + i) % n;
    std::memcpy(output + block_start[owner], work.data() + rot_off[i], block_len[owner]);
  }
}

void RingAllgather(HostTransport* t, const char* input, const comm_size_t* block_start,
                   const comm_size_t* block_len, char* output) {
  const int n = t->num_machines(), r = t->rank();
  std::memcpy(output + block_start[r], input, block_len[r]);
  const int next = (r + 1) % n, prev = (r - 1 + n) % n;
  for (int k = 0; k < n - 1; ++k) {
    const int sb = (r - k + n) % n, rb = (r - k - 1 + n) % n;
    t->SendRecv(next, output + block_start[sb], block_len[sb], prev, output + block_start[rb], block_len[rb]);
  }
}

void RecursiveHalvingReduceScatter(HostTransport* t, const char* input, comm_size_t input_size, int type_size,
                                   const comm_size_t* block_start, const comm_size_t* block_len, char* output,
                                   const ReduceFunction& reducer) {
  const int n = t->num_machines(), r = t->rank();
  std::vector<char> work(input, input + input_size);
  std::vector<char> incoming;
  auto span = [&](int lo, int hi) { return block_start[hi - 1] + block_len[hi - 1] - block_start[lo]; };
  int lo = 0, hi = n;
  for (int d = n / 2; d >= 1; d /= 2) {
    const int partner = r ^ d;
    const int mid = lo + (hi - lo) / 2;
    const bool lower = (r & d) == 0;
    const int keep_lo = lower ? lo : mid, keep_hi = lower ? mid : hi;
    const int give_lo = lower ? mid : lo, give_hi = lower ? hi : mid;
    const comm_size_t keep_len = span(keep_lo, keep_hi);
    incoming.resize(static_cast<size_t>(keep_len));
    t->SendRecv(partner, work.data() + block_start[give_lo], span(give_lo, give_hi), partner, incoming.data(),
                keep_len);
    reducer(incoming.data(), work.data() + block_start[keep_lo], type_size, keep_len);
    lo = keep_lo;
    hi = keep_hi;
  }
  std::memcpy(output, work.data() + block_start[r], block_len[r]);
}

void RingReduceScatter(HostTransport* t, const char* input, comm_size_t input_size, int type_size,
                       const comm_size_t* block_start, const comm_size_t* block_len, char* output,
                       const ReduceFunction& reducer) {
  const int n = t->num_machines(), r = t->rank();
  std::vector<char> work(input, input + input_size);
  comm_size_t max_len = 0;
  for (int i = 0; i < n; ++i) max_len = std::max(max_len, block_len[i]);
  std::vector<char> incoming(static_cast<size_t>(max_len));
  const int next = (r + 1) % n, prev = (r - 1 + n) % n;
  // round k: pass on block r-k-1 (k+1 contributions so far), receive block r-k-2 from the
  // previous rank and add the local contribution; after n-1 rounds block r is complete
  for (int k = 0; k < n - 1; ++k) {
    const int sb = (r - k - 1 + 2 * n) % n, rb = (r - k - 2 + 2 * n) % n;
    t->SendRecv(next, work.data() + block_start[sb], block_len[sb], prev, incoming.data(), block_len[rb]);
    reducer(incoming.data(), work.data() + block_start[rb], type_size, block_len[rb]);
  }
  std::memcpy(output, work.data() + block_start[r], block_len[r]);
}

}  // namespace collectives
}  // namespace lgbm_amd
