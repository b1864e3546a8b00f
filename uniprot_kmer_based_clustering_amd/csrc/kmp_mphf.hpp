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

}  // namespace kmp
