// kmp_edges.hpp — the library-owned edge list behind the opaque kmp_edges handle (kmp_api.cpp,
// kmp_output.cpp).
#pragma once
#include <cstdint>
#include <vector>

struct kmp_edges {
    std::vector<uint32_t> p, q, w;  // canonical (p, q) order, p < q
    std::vector<float> score;
    // shared k-mer lists (kmp_edges_kmers): edge i owns kmers[kofs[i] .. kofs[i+1])
    int kspace = -1;                // -1 none, KMP_KMERS_CODES, KMP_KMERS_IDS
    std::vector<uint64_t> kofs;
    std::vector<uint32_t> kmers;
    std::vector<uint64_t> ref_key;  // IDS only: index in the reference's final edge order
    // kmp_pairs_multi_k: the k of each merged list and the per-k weights (k-major: wk[j*count + i])
    std::vector<int> ks;
    std::vector<uint32_t> wk;
};
