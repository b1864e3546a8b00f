// kmp_df.hpp — device document-frequency pass (main.rs:77-149): distinct k-mers, repeat
// (df >= 2) k-mers, Σ C(df,2) and max df over all per-protein sets.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace kmp {

struct DfCounters {
    uint64_t distinct, repeat, sum_cdf2, max_df;
};

// d_set: per-protein sorted distinct codes in set_base slots; h_set_len/h_off: host copies
// of the set lengths and residue offsets; d_res_off: device residue offsets.  With keep_uniq /
// keep_counts the distinct codes (ascending) and their df (out->distinct entries each) are handed
// to the caller (hipFree); they stay null when there are no set entries.
int device_df_counters(const uint32_t* d_set, const uint32_t* h_set_len, const uint64_t* h_off,
                       const uint64_t* d_res_off, uint32_t n, int k, hipStream_t stream, DfCounters* out,
                       std::string& err, uint32_t** keep_uniq = nullptr, uint32_t** keep_counts = nullptr);

}  // namespace kmp
