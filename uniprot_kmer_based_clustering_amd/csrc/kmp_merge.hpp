// kmp_merge.hpp — device union of per-k canonical edge lists (kmp_merge.hip; config 5).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "kmerpair.h"

namespace kmp {

struct MergeIn {  // nk device lists; list j = entries [off[j], off[j+1]) of the concatenation
    uint32_t nk;
    const uint32_t* p[KMP_MULTI_K_MAX];
    const uint32_t* q[KMP_MULTI_K_MAX];
    const uint32_t* w[KMP_MULTI_K_MAX];
    const uint32_t* s[KMP_MULTI_K_MAX];  // per-edge integer scores (nullptr: none)
    uint64_t off[KMP_MULTI_K_MAX + 1];
};

struct MergeOut {  // device arrays of cap entries
    uint32_t *p, *q, *w;
    uint32_t* s;                   // nullptr: no scores
    uint32_t* wk[KMP_MULTI_K_MAX];  // w_j of every merged edge
    uint64_t cap;
    uint32_t min_shared;            // a pair is kept when some w_j >= min_shared (the lists hold every w_j >= 1)
};

uint64_t merge_scratch_bytes(uint64_t total);
// union of the lists in canonical order (the pairs some w_j reaches out.min_shared with); *n_out = merged edges (KMP_EOVERFLOW if > out.cap);
// host-synchronous
int merge_edges_device(const MergeIn& in, const MergeOut& out, void* scratch, uint64_t scratch_bytes,
                       uint64_t* n_out, hipStream_t st);

}  // namespace kmp
