// kmp_multi.hpp — the multi-GPU split behind the C ABI (kmp_ctx_create_multi).
//
// Two flows over the same ranks (each its own device, stream, workspace and copy of the packed
// batch); rank g always ends with the canonical edges of rows [start[g], start[g+1])
// (kmp_row_split), and the gather to device 0 in rank order is the canonical list:
//   k-mer split (default): rank g expands its share of the k-mers (kmp_dev_split_expand), one
//     all-to-all routes the pair keys to their row owners, each rank reduces its rows
//     (kmp_dev_split_edges);
//   row split (batches whose frequent k-mers spill, and the bounded-memory passes): rank g
//     groups every k-mer and expands only its rows (kmp_dev_pairs_rows); no exchange.
// The collectives go through a Transport, so the same flows run over RCCL between GPUs
// (library-owned communicators, ncclCommInitAll in-process) and over device copies between
// virtual ranks that share one GPU (tests; RCCL admits one rank per device).
#pragma once

#include <hip/hip_runtime.h>

#include <array>
#include <memory>
#include <string>
#include <vector>

namespace kmp {

using EdgeArrays = std::array<uint32_t*, 3>;  // p, q, w

struct Transport {
    virtual ~Transport() = default;
    virtual const char* name() const = 0;
    // dst[a][off[g] .. off[g] + counts[g]) <- src[g][a][0 .. counts[g]) for every rank g, a < 3;
    // dst lives on rank 0's device; enqueued on the ranks' streams, complete on return.
    // Returns KMP_OK, KMP_ERCCL or KMP_EDEVICE; *err describes a failure.
    virtual int gather(const std::vector<EdgeArrays>& src, const EdgeArrays& dst, const std::vector<uint64_t>& counts,
                       const std::vector<hipStream_t>& streams, std::string* err) = 0;
    // the k-mer split's exchange: recv[d] + g * bytes <- send[g] + d * bytes for every pair of
    // ranks (g, d), ordered after the work already on the ranks' streams, complete on return
    virtual int alltoall(const std::vector<const char*>& send, const std::vector<char*>& recv, uint64_t bytes,
                         const std::vector<hipStream_t>& streams, std::string* err) = 0;
};

// device-to-device copies (hipMemcpyPeerAsync): any set of devices, repeated ones included
std::unique_ptr<Transport> make_copy_transport(const std::vector<int>& devices);
// RCCL over the given (distinct) devices, communicators created in-process with
// ncclCommInitAll; librccl is loaded at run time.  nullptr (and *err) if RCCL is unavailable.
std::unique_ptr<Transport> make_rccl_transport(const std::vector<int>& devices, std::string* err);

}  // namespace kmp
