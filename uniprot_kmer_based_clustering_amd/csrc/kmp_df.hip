// kmp_df.hip — device df counters: gather every K(p) into one dense array, radix-sort it,
// run-length encode (one run per distinct k-mer, run length = df), reduce the runs.
// Replaces the global Vec<(kmer, df)> of src/main.rs:77-122 (binary insertion under one
// mutex) and the unique/repeat split of :127-149.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_run_length_encode.hpp>
#include <vector>

#include "kmerpair.h"
#include "kmp_df.hpp"
#include "kmp_internal.hpp"

namespace kmp {
namespace {

__global__ void gather_sets_kernel(const uint32_t* __restrict__ set, const uint64_t* __restrict__ res_off,
                                   const uint64_t* __restrict__ dofs, uint32_t* __restrict__ dense) {
    const uint32_t p = blockIdx.x;
    const uint64_t b = dofs[p], len = dofs[p + 1] - b;
    const uint32_t* s = set + set_base(res_off[p], p);
    for (uint64_t e = threadIdx.x; e < len; e += blockDim.x) dense[b + e] = s[e];
}

__global__ void reduce_runs_kernel(const uint32_t* __restrict__ counts, const uint32_t* __restrict__ runs,
                                   unsigned long long* __restrict__ acc) {
    const uint32_t nr = *runs;
    unsigned long long rep = 0, cdf2 = 0, mx = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nr; i += gridDim.x * blockDim.x) {
        const unsigned long long c = counts[i];
        rep += c >= 2;
        cdf2 += c * (c - 1) / 2;
        mx = c > mx ? c : mx;
    }
    for (int o = 32; o > 0; o >>= 1) {
        rep += __shfl_down(rep, o);
        cdf2 += __shfl_down(cdf2, o);
        const unsigned long long m2 = __shfl_down(mx, o);
        mx = m2 > mx ? m2 : mx;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&acc[0], rep);
        atomicAdd(&acc[1], cdf2);
        atomicMax(&acc[2], mx);
    }
}

unsigned bits_for(uint64_t v) {
    unsigned b = 0;
    while (b < 64 && (v - 1) >> b) ++b;
    return b ? b : 1;
}

struct Scratch {
    std::vector<void*> ptrs;
    ~Scratch() {
        for (void* p : ptrs)
            if (p) (void)hipFree(p);
    }
    template <class T>
    T* release(T* p) {  // hand one buffer to the caller
        for (auto& q : ptrs)
            if (q == p) q = nullptr;
        return p;
    }
    template <class T>
    hipError_t alloc(T** p, size_t bytes) {
        void* v = nullptr;
        hipError_t e = hipMalloc(&v, bytes ? bytes : 16);
        if (e == hipSuccess) ptrs.push_back(v);
        *p = static_cast<T*>(v);
        return e;
    }
};

}  // namespace

int device_df_counters(const uint32_t* d_set, const uint32_t* h_set_len, const uint64_t* h_off,
                       const uint64_t* d_res_off, uint32_t n, int k, hipStream_t st, DfCounters* out,
                       std::string& err, uint32_t** keep_uniq, uint32_t** keep_counts) {
    (void)h_off;
    *out = DfCounters{};
    if (keep_uniq) *keep_uniq = nullptr;
    if (keep_counts) *keep_counts = nullptr;
    if (n == 0) return KMP_OK;
    std::vector<uint64_t> dofs(n + 1, 0);
    for (uint32_t p = 0; p < n; ++p) dofs[p + 1] = dofs[p] + h_set_len[p];
    const uint64_t S = dofs[n];
    if (S == 0) return KMP_OK;
    if (S > 0xFFFFFFFFull) {
        err = "df pass: more than 2^32 set entries";
        return KMP_EINVAL;
    }
    Scratch sc;
    uint64_t* d_dofs;
    uint32_t *dense, *sorted, *uniq, *counts, *runs;
    unsigned long long* acc;
#define DF_HIP(x)                                              \
    do {                                                       \
        hipError_t e_ = (x);                                   \
        if (e_ != hipSuccess) {                                \
            err = std::string(#x) + ": " + hipGetErrorString(e_); \
            return e_ == hipErrorOutOfMemory ? KMP_ENOMEM : KMP_EDEVICE; \
        }                                                      \
    } while (0)
    DF_HIP(sc.alloc(&d_dofs, (n + 1) * sizeof(uint64_t)));
    DF_HIP(sc.alloc(&dense, S * 4));
    DF_HIP(sc.alloc(&sorted, S * 4));
    DF_HIP(sc.alloc(&uniq, S * 4));
    DF_HIP(sc.alloc(&counts, S * 4));
    DF_HIP(sc.alloc(&runs, 16));
    DF_HIP(sc.alloc(&acc, 3 * sizeof(unsigned long long)));
    DF_HIP(hipMemcpyAsync(d_dofs, dofs.data(), (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    DF_HIP(hipMemsetAsync(acc, 0, 3 * sizeof(unsigned long long), st));
    gather_sets_kernel<<<n, 256, 0, st>>>(d_set, d_res_off, d_dofs, dense);
    DF_HIP(hipGetLastError());
    const unsigned end_bit = bits_for(pow21(k));
    size_t b1 = 0, b2 = 0;
    DF_HIP(rocprim::radix_sort_keys(nullptr, b1, dense, sorted, (size_t)S, 0u, end_bit, st));
    DF_HIP(rocprim::run_length_encode(nullptr, b2, sorted, (unsigned int)S, uniq, counts, runs, st));
    void* tmp;
    DF_HIP(sc.alloc(&tmp, b1 > b2 ? b1 : b2));
    DF_HIP(rocprim::radix_sort_keys(tmp, b1, dense, sorted, (size_t)S, 0u, end_bit, st));
    DF_HIP(rocprim::run_length_encode(tmp, b2, sorted, (unsigned int)S, uniq, counts, runs, st));
    reduce_runs_kernel<<<1024, 256, 0, st>>>(counts, runs, acc);
    DF_HIP(hipGetLastError());
    uint32_t h_runs = 0;
    unsigned long long h_acc[3];
    DF_HIP(hipMemcpyAsync(&h_runs, runs, 4, hipMemcpyDeviceToHost, st));
    DF_HIP(hipMemcpyAsync(h_acc, acc, sizeof h_acc, hipMemcpyDeviceToHost, st));
    DF_HIP(hipStreamSynchronize(st));
#undef DF_HIP
    out->distinct = h_runs;
    out->repeat = h_acc[0];
    out->sum_cdf2 = h_acc[1];
    out->max_df = h_acc[2];
    if (keep_uniq) *keep_uniq = sc.release(uniq);
    if (keep_counts) *keep_counts = sc.release(counts);
    return KMP_OK;
}

}  // namespace kmp
