// exchange.hpp -- the collectives of the slice-sharded prepass,
// built on the one primitive the caller supplies (alvrl_exchange::allgather:
// fixed-size bytes per rank, rank order).  Host code only; the caller's
// communicator moves the bytes (RCCL through torch.distributed over xGMI, MPI,
// or gloo in the CPU tests).
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/alvrl_host.h"

namespace alvrl {
namespace host {

struct CommError : std::runtime_error {
    int code;
    CommError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// counts[r] = bytes rank r contributes.
std::vector<uint64_t> allgather_counts(const alvrl_exchange& ex, uint32_t world, uint64_t bytes);
// Variable-size all-gather: ranks' data concatenated in rank order.
std::vector<uint8_t> allgatherv(const alvrl_exchange& ex, uint32_t world, const void* send, uint64_t bytes,
                                std::vector<uint64_t>* counts);
// Element-wise OR over ranks, in place.
void or_reduce(const alvrl_exchange& ex, uint32_t world, uint8_t* buf, uint64_t n);

// Per-slice cluster lists over all slices (vrlClusterInfo's m_selectedVrls /
// m_clusterWeight, vrlIntegrator.cpp:17-115) after every rank refined its own.
struct SliceClusters {
    std::vector<int> refined;         // per slice; 0 for slices no rank reported
    std::vector<uint32_t> off, reps;  // CSR, nslices + 1 offsets
    std::vector<float> w;
};
SliceClusters merge_clusters(const alvrl_exchange& ex, uint32_t world, uint32_t nslices, uint32_t n_local,
                             const uint32_t* local_slice, const int* local_refined, const uint32_t* local_off,
                             const uint32_t* local_reps, const float* local_w);

}  // namespace host
}  // namespace alvrl
