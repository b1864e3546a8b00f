// kmp_mphf.hpp — device minimal perfect hashing (kmp_mphf.hip) for the host API (kmp_api.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "kmerpair.h"

namespace kmp {

// MPHF of n distinct device keys (gamma >= 1)
int mphf_build_device(const uint32_t* d_keys, uint64_t n, double gamma, hipStream_t st, kmp_mphf** out);
// ids (uint64, ~0 for keys outside the set that miss every level) of n device keys
int mphf_lookup_device(const kmp_mphf* m, const uint32_t* d_keys, uint64_t n, uint64_t* d_ids, hipStream_t st);

// The repeat k-mers of main.rs:127-149 and their MPHF (:140): from the distinct codes and their df
// (one run per k-mer), keep df >= 2, hash them, and scatter code_by_id / df_by_id (R entries,
// device buffers the caller frees with hipFree).  df_by_id is five_mer_hash_freq (main.rs:187-193).
int repeat_mphf_build(const uint32_t* d_uniq, const uint32_t* d_counts, uint64_t runs, double gamma, hipStream_t st,
                      kmp_mphf** mphf, uint32_t** d_code_by_id, uint32_t** d_df_by_id, uint64_t* repeat);

// hash_five_mers of every protein (remove_unique_five_mers + modify_hash_five_mer,
// protein.rs:151-174): the repeat-MPHF ids of each protein's windows at k, first-occurrence order,
// duplicates dropped.  *d_ids (hipFree) holds h_ids_off[n] ids; protein p owns
// [h_ids_off[p], h_ids_off[p + 1]).  Membership is checked against code_by_id.
int hash_kmers_device(const kmp_mphf* m, const uint8_t* d_res, const uint64_t* d_off, const uint64_t* h_off,
                      uint32_t n, int k, const uint32_t* d_code_by_id, uint64_t repeat, hipStream_t st,
                      uint32_t** d_ids, std::vector<uint64_t>& h_ids_off);

// shared k-mers of each edge (p[i], q[i]) (kmp_edgekmers.hip): w[i] = kofs[i+1] - kofs[i]
// ascending codes at out[kofs[i] ..), from the repeat-filtered sets.  KMP_EINVAL when an edge's
// intersection is not w long (edges of another kmp_build_sets).
int edge_blosum_device(const uint32_t* d_rep, const uint32_t* d_rep_len, const uint64_t* d_off, const uint32_t* d_p,
                       const uint32_t* d_q, const uint32_t* d_w, uint64_t count, int k, float* d_score,
                       hipStream_t st);
int edge_kmers_device(const uint32_t* d_rep, const uint32_t* d_rep_len, const uint64_t* d_off, const uint32_t* d_p,
                      const uint32_t* d_q, const uint64_t* d_kofs, uint64_t count, uint32_t* d_out, hipStream_t st);
// codes -> repeat-MPHF ids in place, ascending within each edge; with d_ref_key, each edge's
// index in the reference's final order (ascending (min shared id, p, q)).
int edge_kmers_to_ids(const kmp_mphf* m, const uint64_t* d_kofs, uint64_t count, uint64_t total, uint32_t* d_inout,
                      uint64_t* d_ref_key, hipStream_t st);

}  // namespace kmp
