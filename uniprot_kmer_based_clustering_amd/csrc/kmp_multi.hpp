// kmp_multi.hpp — the multi-GPU split behind the C ABI (kmp_ctx_create_multi).
//
// The pair space is split by rows: rank g expands the pairs (p, q), p < q, whose smaller protein
// lies in rows [start[g], start[g+1]) (kmp_row_split), with kmp_dev_pairs_rows on its own device
// and its own copy of the packed batch.  Ranks never exchange keys; the only collective is the
// gather of every rank's edges to device 0 in rank order, which is already the canonical list.
// The gather goes through a Transport, so the same flow runs over RCCL between GPUs
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
};

// device-to-device copies (hipMemcpyPeerAsync): any set of devices, repeated ones included
std::unique_ptr<Transport> make_copy_transport(const std::vector<int>& devices);
// RCCL over the given (distinct) devices, communicators created in-process with
// ncclCommInitAll; librccl is loaded at run time.  nullptr (and *err) if RCCL is unavailable.
std::unique_ptr<Transport> make_rccl_transport(const std::vector<int>& devices, std::string* err);

}  // namespace kmp
