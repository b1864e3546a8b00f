// kmp_merge.hip — the config-5 combination of per-k edge lists on the device (SURVEY.md §8d:
// "w5, w7 computed independently per pair; an edge is emitted if w5 >= 1 or w7 >= 1").
// nk canonical lists (each (p, q)-sorted, unique pairs) -> their union in canonical order with
// w = Σ_j w_j, score = Σ_j score_j and every w_j kept (0 where list j lacks the pair).
//   keys (p << 32 | q) of all lists, values = position in the concatenation -> one radix sort of
//   pairs; a run of equal keys is one pair (at most nk entries, one per list); its head sums the
//   run and writes the merged edge at its rank among the heads (an exclusive scan).
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cstdint>

#include "kmerpair.h"
#include "kmp_merge.hpp"

namespace {

using SortCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                           rocprim::default_config, 0>;  // see kmp_postings.hip

__global__ void merge_keys_kernel(kmp::MergeIn in, uint64_t total, unsigned long long* __restrict__ key,
                                  uint32_t* __restrict__ val) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t j = 0;
        while (j + 1 < in.nk && i >= in.off[j + 1]) ++j;
        const uint64_t t = i - in.off[j];
        key[i] = (unsigned long long)in.p[j][t] << 32 | in.q[j][t];
        val[i] = (uint32_t)i;
    }
}

// a head (first entry of a run = one pair) that some w_j reaches min_shared with
__global__ void merge_heads_kernel(kmp::MergeIn in, const unsigned long long* __restrict__ key,
                                   const uint32_t* __restrict__ val, uint64_t total, uint32_t min_shared,
                                   uint32_t* __restrict__ head) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i <= total; i += (uint64_t)gridDim.x * blockDim.x) {
        bool h = i < total && (i == 0 || key[i] != key[i - 1]);
        if (h && min_shared > 1) {
            bool keep = false;
            for (uint64_t t = i; t < total && key[t] == key[i]; ++t) {
                const uint64_t g = val[t];
                uint32_t j = 0;
                while (j + 1 < in.nk && g >= in.off[j + 1]) ++j;
                keep |= in.w[j][g - in.off[j]] >= min_shared;
            }
            h = keep;
        }
        head[i] = h;
    }
}

__global__ void merge_write_kernel(kmp::MergeIn in, const unsigned long long* __restrict__ key,
                                   const uint32_t* __restrict__ val, const uint32_t* __restrict__ pos, uint64_t total,
                                   kmp::MergeOut out) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        if (i && key[i] == key[i - 1]) continue;  // not a head
        if (pos[i + 1] == pos[i]) continue;      // a pair no w_j reaches min_shared with
        const uint64_t o = pos[i];
        if (o >= out.cap) continue;
        uint32_t wsum = 0;
        uint32_t ssum = 0;
        uint32_t wk[KMP_MULTI_K_MAX] = {0, 0, 0, 0};
        for (uint64_t t = i; t < total && key[t] == key[i]; ++t) {
            const uint64_t g = val[t];
            uint32_t j = 0;
            while (j + 1 < in.nk && g >= in.off[j + 1]) ++j;
            const uint64_t s = g - in.off[j];
            wk[j] = in.w[j][s];
            wsum += wk[j];
            if (in.s[j]) ssum += in.s[j][s];
        }
        out.p[o] = (uint32_t)(key[i] >> 32);
        out.q[o] = (uint32_t)key[i];
        out.w[o] = wsum;
        if (out.s) out.s[o] = ssum;
        for (uint32_t j = 0; j < in.nk; ++j) out.wk[j][o] = wk[j];
    }
}

}  // namespace

namespace kmp {

uint64_t merge_scratch_bytes(uint64_t total) {
    size_t t1 = 0, t2 = 0;
    (void)rocprim::radix_sort_pairs<SortCfg>(nullptr, t1, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                             (uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)total, 0u, 64u);
    (void)rocprim::exclusive_scan(nullptr, t2, (uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)total + 1,
                                  rocprim::plus<uint32_t>());
    // keys x2 (u64), values x2, heads, positions (u32), each region 256-byte aligned, + rocprim's
    return 24 * total + 8 * (total + 1) + 7 * 256 + std::max(t1, t2) + 256;
}

int merge_edges_device(const MergeIn& in, const MergeOut& out, void* scratch, uint64_t scratch_bytes,
                       uint64_t* n_out, hipStream_t st) {
    uint64_t total = in.off[in.nk];
    *n_out = 0;
    if (total == 0) return KMP_OK;
    if (total >= 0xFFFFFFFFull || scratch_bytes < merge_scratch_bytes(total)) return KMP_EINVAL;
    char* b = static_cast<char*>(scratch);
    auto take = [&](uint64_t bytes) {
        char* r = b;
        b += (bytes + 255) & ~255ull;
        return r;
    };
    auto* k0 = reinterpret_cast<unsigned long long*>(take(8 * total));
    auto* k1 = reinterpret_cast<unsigned long long*>(take(8 * total));
    auto* v0 = reinterpret_cast<uint32_t*>(take(4 * total));
    auto* v1 = reinterpret_cast<uint32_t*>(take(4 * total));
    auto* head = reinterpret_cast<uint32_t*>(take(4 * (total + 1)));
    auto* pos = reinterpret_cast<uint32_t*>(take(4 * (total + 1)));
    void* tmp = b;
    size_t tb = scratch_bytes - (uint64_t)(b - static_cast<char*>(scratch));
    const uint32_t grid = (uint32_t)std::min<uint64_t>((total + 255) / 256, 8192);
    merge_keys_kernel<<<grid, 256, 0, st>>>(in, total, k0, v0);
    if (rocprim::radix_sort_pairs<SortCfg>(tmp, tb, k0, k1, v0, v1, (size_t)total, 0u, 64u, st) != hipSuccess)
        return KMP_EDEVICE;
    merge_heads_kernel<<<grid, 256, 0, st>>>(in, k1, v1, total, out.min_shared, head);
    tb = scratch_bytes - (uint64_t)(static_cast<char*>(tmp) - static_cast<char*>(scratch));
    if (rocprim::exclusive_scan(tmp, tb, head, pos, 0u, (size_t)total + 1, rocprim::plus<uint32_t>(), st) != hipSuccess)
        return KMP_EDEVICE;
    merge_write_kernel<<<grid, 256, 0, st>>>(in, k1, v1, pos, total, out);
    uint32_t m = 0;
    if (hipMemcpyAsync(&m, pos + total, 4, hipMemcpyDeviceToHost, st) != hipSuccess) return KMP_EDEVICE;
    if (hipStreamSynchronize(st) != hipSuccess) return KMP_EDEVICE;
    *n_out = m;
    return m > out.cap ? KMP_EOVERFLOW : KMP_OK;
}

}  // namespace kmp
