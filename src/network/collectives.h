// Host collective algorithms over a point-to-point transport (HostTransport::SendRecv).
// Reference: src/network/network.cpp:68-318 (Bruck / recursive-doubling allgather,
// recursive-halving reduce-scatter over the socket linkers).  Blocks are laid out in rank
// order: block_start[i] is rank i's offset, the blocks are contiguous and ascending.
#pragma once

#include "lgbm_amd/network.h"

namespace lgbm_amd {
namespace collectives {

// ceil(log2 n) rounds; round k exchanges min(2^k, n - 2^k) blocks with ranks r -/+ 2^k
void BruckAllgather(HostTransport* t, const char* input, const comm_size_t* block_start,
                    const comm_size_t* block_len, char* output);
// n-1 rounds of one block each, to rank r+1 / from rank r-1 (writes straight into output)
void RingAllgather(HostTransport* t, const char* input, const comm_size_t* block_start,
                   const comm_size_t* block_len, char* output);
// n a power of two: log2 n rounds, each halving the block range a rank is responsible for
void RecursiveHalvingReduceScatter(HostTransport* t, const char* input, comm_size_t input_size, int type_size,
                                   const comm_size_t* block_start, const comm_size_t* block_len, char* output,
                                   const ReduceFunction& reducer);
// any n: n-1 rounds around the ring, each adding the local contribution to one block
void RingReduceScatter(HostTransport* t, const char* input, comm_size_t input_size, int type_size,
                       const comm_size_t* block_start, const comm_size_t* block_len, char* output,
                       const ReduceFunction& reducer);

}  // namespace collectives
}  // namespace lgbm_amd
