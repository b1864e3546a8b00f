// kmp_stream.hpp — device summary of a streamed edge chunk (kmp_stream.hip; kmp_pairs_stream).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "kmerpair.h"

namespace kmp {

struct DigestIn {  // one chunk of canonical edges on the device
    const uint32_t *p, *q, *w;
    const uint32_t* s;   // integer score per edge (nullptr: s = w)
    const uint32_t* w0;  // multi-k: w of the first k (nullptr: w0 = w)
    uint64_t n;
    uint32_t n_prot, row_lo, row_hi;
    const uint16_t* cls;  // class per protein (Σ w of class-differing pairs; nullptr: none)
    uint32_t align_threshold;
};

struct DigestAcc {  // device accumulators (zeroed by the caller), summed over the chunks
    unsigned long long seg_edges[KMP_DIGEST_SEGMENTS];
    unsigned long long seg_digest[KMP_DIGEST_SEGMENTS];
    unsigned long long tot[4];  // Σ w, Σ score, w > align_threshold, Σ w of class-differing pairs
    unsigned int bad;           // a chunk out of (p, q) order, or an edge outside its rows / the batch
};

hipError_t edge_digest_enqueue(const DigestIn& in, DigestAcc* acc, hipStream_t st);

}  // namespace kmp
