// kmp_postings.hip — the postings engine: the reference's own pair algorithm restated for the
// GPU as sort / expand / reduce.
//
//   reference (file:line)                                  here
//   global df: sorted Vec<(kmer, df)> (main.rs:77-122)     radix sort of (code << pbits | p) keys;
//                                                          one run per distinct k-mer, run length = df
//   repeat split df >= 2 (main.rs:127-149)                 runs of length >= 2
//   Graph::new: C(df,2) KmerEdge::Single per k-mer         expand_kernel: every (k-mer, p, q) incidence
//     (graph/mod.rs:39-193, vertex.rs:59-140)                of a run, one thread per run element
//   remove_uninteresting_edges (mod.rs:549-697)            class test fused into the expansion
//   combine_edges: Group per pair, len = w (mod.rs:322-546) radix sort of pair keys p*N+q, run-length
//                                                          encode: run length = w; the runs come out in
//                                                          canonical (p, q) order
// Work is O(Σ C(df,2)) like the reference (no N² scan); k-mers whose df exceeds heavy_df are
// skipped here and counted by the tiled kernel over the proteins' heavy k-mers (kmp_api.cpp).
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_run_length_encode.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include <algorithm>
#include <cstdint>
#include <vector>

#include "kmerpair.h"
#include "kmp_internal.hpp"

using namespace kmp;

namespace {

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

unsigned bits_for(uint64_t v) {  // bits needed for values < v
    unsigned b = 0;
    while (b < 64 && (v - 1) >> b) ++b;
    return b ? b : 1;
}

__device__ __forceinline__ uint32_t mask_rank(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

constexpr unsigned long long kNoKey = ~0ull;

// every slot of protein p's region: its k-mer key, or kNoKey past |K(p)|
__global__ __launch_bounds__(256) void kmer_keys_kernel(const uint32_t* __restrict__ set,
                                                        const uint32_t* __restrict__ set_len,
                                                        const uint64_t* __restrict__ res_off, unsigned pbits,
                                                        unsigned long long* __restrict__ keys) {
    const uint32_t p = blockIdx.x;
    const uint64_t b = set_base(res_off[p], p), e = set_base(res_off[p + 1], p + 1);
    const uint32_t len = set_len[p];
    for (uint64_t i = b + threadIdx.x; i < e; i += 256) {
        const uint64_t o = i - b;
        keys[i] = o < len ? ((unsigned long long)set[i] << pbits) | p : kNoKey;
    }
}

// run heads of the sorted keys (a run = one distinct k-mer); invalid keys are never heads
__global__ void heads_kernel(const unsigned long long* __restrict__ k, uint64_t n, unsigned pbits,
                             uint32_t* __restrict__ head) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long x = k[i];
        head[i] = x != kNoKey && (i == 0 || (k[i - 1] >> pbits) != (x >> pbits));
    }
}

// per-run statistics: distinct / repeat / Σ C(df,2) (light runs) / max df / heavy elements
__global__ void run_stats_kernel(const uint32_t* __restrict__ starts, const uint32_t* __restrict__ nruns,
                                 uint32_t heavy_df, unsigned long long* __restrict__ acc) {
    const uint32_t R = *nruns;
    unsigned long long rep = 0, cdf2 = 0, mx = 0, heavy = 0;
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < R; r += gridDim.x * blockDim.x) {
        const unsigned long long f = starts[r + 1] - starts[r];
        rep += f >= 2;
        if (f <= heavy_df) cdf2 += f * (f - 1) / 2;
        else heavy += f;
        mx = f > mx ? f : mx;
    }
    for (int o = 32; o > 0; o >>= 1) {
        rep += __shfl_down(rep, o);
        cdf2 += __shfl_down(cdf2, o);
        heavy += __shfl_down(heavy, o);
        const unsigned long long m2 = __shfl_down(mx, o);
        mx = m2 > mx ? m2 : mx;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&acc[0], rep);
        atomicAdd(&acc[1], cdf2);
        atomicMax(&acc[2], mx);
        atomicAdd(&acc[3], heavy);
    }
}

// Σ C(df,2) incidence expansion (vertex.rs:103-137) with the AMR test of mod.rs:580-587:
// element i of a light run [s, e) pairs with every later element of the run.  Two passes, no
// atomics: kWrite = false counts each element's kept partners, an exclusive scan turns the
// counts into output offsets, kWrite = true writes the pair keys p*N+q (p < q) there.
template <bool kWrite>
__global__ __launch_bounds__(256) void expand_kernel(const unsigned long long* __restrict__ k,
                                                     const uint32_t* __restrict__ rid,
                                                     const uint32_t* __restrict__ starts, uint64_t n_valid,
                                                     unsigned pbits, const uint16_t* __restrict__ cls,
                                                     uint32_t n_prot, int require_diff, uint32_t heavy_df,
                                                     uint32_t* __restrict__ counts,
                                                     const unsigned long long* __restrict__ offs,
                                                     unsigned long long* __restrict__ out) {
    const unsigned long long pmask = (1ull << pbits) - 1;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n_valid;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t r = rid[i] - 1;  // inclusive head count -> run index
        const uint32_t s = starts[r], e = starts[r + 1];
        const uint32_t f = e - s;
        uint32_t c = 0;
        if (f >= 2 && f <= heavy_df) {
            const uint32_t p = (uint32_t)(k[i] & pmask);
            const uint16_t cp = cls[p];
            unsigned long long o = kWrite ? offs[i] : 0ull;
            for (uint64_t j = i + 1; j < e; ++j) {
                const uint32_t q = (uint32_t)(k[j] & pmask);
                if (require_diff && cls[q] == cp) continue;
                if (kWrite) {
                    const uint32_t a = min(p, q), b = max(p, q);
                    out[o++] = (unsigned long long)a * n_prot + b;
                } else {
                    ++c;
                }
            }
        }
        if (!kWrite) counts[i] = c;
    }
}

// (pair key, w) runs -> edges with w >= min_shared, canonical order kept
__global__ void emit_edges_kernel(const unsigned long long* __restrict__ uniq, const uint32_t* __restrict__ w,
                                  const uint32_t* __restrict__ nuniq, uint32_t n_prot, uint32_t min_shared,
                                  const uint32_t* __restrict__ pos, uint32_t* __restrict__ out_p,
                                  uint32_t* __restrict__ out_q, uint32_t* __restrict__ out_w, uint64_t cap) {
    const uint32_t U = *nuniq;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < U; i += gridDim.x * blockDim.x) {
        if (w[i] < min_shared) continue;
        const uint32_t o = pos[i];
        if (o >= cap) continue;
        out_p[o] = (uint32_t)(uniq[i] / n_prot);
        out_q[o] = (uint32_t)(uniq[i] % n_prot);
        out_w[o] = w[i];
    }
}

__global__ void keep_flags_kernel(const uint32_t* __restrict__ w, const uint32_t* __restrict__ nuniq,
                                  uint32_t min_shared, uint32_t* __restrict__ keep, uint64_t n) {
    const uint32_t U = *nuniq;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        keep[i] = i < U && w[i] >= min_shared;
}

template <class T>
struct Grow {
    T* p = nullptr;
    size_t n = 0;
    hipError_t reserve(size_t m) {
        if (m <= n && p) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipMalloc(&p, std::max<size_t>(1, m) * sizeof(T));
        if (e == hipSuccess) n = std::max<size_t>(1, m);
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

}  // namespace

struct kmp_postings {
    Grow<unsigned long long> keys, sorted, inc, inc_sorted, uniq;
    Grow<uint32_t> head, rid, starts, w, keep, pos, small, cnt;
    Grow<unsigned long long> acc, offs;
    Grow<char> tmp;
    ~kmp_postings() {
        keys.release(); sorted.release(); inc.release(); inc_sorted.release(); uniq.release();
        head.release(); rid.release(); starts.release(); w.release(); keep.release(); pos.release();
        small.release(); acc.release(); tmp.release(); cnt.release(); offs.release();
    }
};

extern "C" {

int kmp_postings_create(kmp_postings** ws) {
    if (!ws) return KMP_EINVAL;
    *ws = new (std::nothrow) kmp_postings;
    return *ws ? KMP_OK : KMP_ENOMEM;
}

void kmp_postings_destroy(kmp_postings* ws) { delete ws; }

#define PG(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) return e_ == hipErrorOutOfMemory ? KMP_ENOMEM : KMP_EDEVICE; \
    } while (0)

int kmp_dev_pairs_postings(kmp_postings* ws, const uint32_t* d_set, const uint32_t* d_set_len,
                           const uint64_t* d_res_off, const uint16_t* d_class, uint32_t n, int k, uint64_t slots,
                           uint32_t heavy_df, uint32_t min_shared, int require_class_diff, uint32_t* d_p,
                           uint32_t* d_q, uint32_t* d_w, uint64_t cap, uint64_t* n_edges,
                           kmp_postings_stats* stats, void* stream) {
    if (!ws || !n_edges || k < 1 || k > kMaxK) return KMP_EINVAL;
    *n_edges = 0;
    if (stats) *stats = kmp_postings_stats{};
    if (n < 2) return KMP_OK;
    if (!d_set || !d_set_len || !d_res_off || !d_class || (cap && (!d_p || !d_q || !d_w))) return KMP_EINVAL;
    if (min_shared < 1) min_shared = 1;
    if (heavy_df < 2) heavy_df = 2;
    hipStream_t st = as_stream(stream);
    const unsigned pbits = bits_for(n);
    const unsigned end_bit = bits_for(pow21(k)) + pbits;
    if (end_bit > 64) return KMP_EINVAL;
    if (slots > 0xFFFFFFFFull) return KMP_EINVAL;  // run ids are u32

    // 1. keys of every slot, sorted; invalid slots (kNoKey) sort last
    PG(ws->keys.reserve(slots));
    PG(ws->sorted.reserve(slots));
    PG(hipMemsetAsync(ws->keys.p, 0xFF, slots * sizeof(unsigned long long), st));
    kmer_keys_kernel<<<n, 256, 0, st>>>(d_set, d_set_len, d_res_off, pbits, ws->keys.p);
    size_t t_sort = 0, t_scan = 0, t_sel = 0;
    PG(rocprim::radix_sort_keys(nullptr, t_sort, ws->keys.p, ws->sorted.p, (size_t)slots, 0u, 64u, st));
    PG(rocprim::inclusive_scan(nullptr, t_scan, ws->head.p, ws->rid.p, (size_t)slots, rocprim::plus<uint32_t>(), st));
    PG(rocprim::select(nullptr, t_sel, rocprim::counting_iterator<uint32_t>(0), ws->head.p, ws->starts.p,
                       ws->small.p, (size_t)slots, st));
    PG(ws->tmp.reserve(std::max({t_sort, t_scan, t_sel})));
    PG(rocprim::radix_sort_keys(ws->tmp.p, t_sort, ws->keys.p, ws->sorted.p, (size_t)slots, 0u, end_bit, st));
    // valid keys = Σ |K(p)| (everything before the first kNoKey); counted from the heads pass below

    // 2. run heads -> run index per element (inclusive scan) and run starts (select)
    PG(ws->head.reserve(slots));
    PG(ws->rid.reserve(slots));
    PG(ws->starts.reserve(slots + 1));
    PG(ws->small.reserve(16));
    PG(ws->acc.reserve(8));
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((slots + 255) / 256, 8192);
    heads_kernel<<<blocks, 256, 0, st>>>(ws->sorted.p, slots, pbits, ws->head.p);
    PG(rocprim::inclusive_scan(ws->tmp.p, t_scan, ws->head.p, ws->rid.p, (size_t)slots, rocprim::plus<uint32_t>(), st));
    PG(rocprim::select(ws->tmp.p, t_sel, rocprim::counting_iterator<uint32_t>(0), ws->head.p, ws->starts.p,
                       ws->small.p, (size_t)slots, st));
    // number of valid keys: position of the first kNoKey = Σ set_len (host knows it cheaply? no:
    // read the run count and use the total from the set lengths)
    uint32_t h_runs = 0;
    unsigned long long h_total = 0;
    {
        // Σ |K(p)| via a tiny reduction on the set lengths
        size_t t_red = 0;
        PG(rocprim::inclusive_scan(nullptr, t_red, d_set_len, ws->pos.p, (size_t)n, rocprim::plus<uint32_t>(), st));
        PG(ws->pos.reserve(n));
        if (t_red > ws->tmp.n) PG(ws->tmp.reserve(t_red));
        PG(rocprim::inclusive_scan(ws->tmp.p, t_red, d_set_len, ws->pos.p, (size_t)n, rocprim::plus<uint32_t>(), st));
        uint32_t tot32 = 0;
        PG(hipMemcpyAsync(&tot32, ws->pos.p + (n - 1), 4, hipMemcpyDeviceToHost, st));
        PG(hipMemcpyAsync(&h_runs, ws->small.p, 4, hipMemcpyDeviceToHost, st));
        PG(hipStreamSynchronize(st));
        h_total = tot32;
    }
    // starts[R] = number of valid keys (end of the last run)
    {
        const uint32_t tot = (uint32_t)h_total;
        PG(hipMemcpyAsync(ws->starts.p + h_runs, &tot, 4, hipMemcpyHostToDevice, st));
    }
    PG(hipMemsetAsync(ws->acc.p, 0, 8 * sizeof(unsigned long long), st));
    if (h_runs) run_stats_kernel<<<1024, 256, 0, st>>>(ws->starts.p, ws->small.p, heavy_df, ws->acc.p);
    unsigned long long acc[4] = {0, 0, 0, 0};
    PG(hipMemcpyAsync(acc, ws->acc.p, sizeof acc, hipMemcpyDeviceToHost, st));
    PG(hipStreamSynchronize(st));
    if (stats) {
        stats->sum_S = h_total;
        stats->distinct = h_runs;
        stats->repeat = acc[0];
        stats->sum_cdf2_light = acc[1];
        stats->max_df = acc[2];
        stats->heavy_entries = acc[3];
    }

    // 3. expansion of the light runs (class filter fused): count, scan, write
    unsigned long long n_inc = 0;
    if (h_total) {
        PG(ws->cnt.reserve(h_total));
        PG(ws->offs.reserve(h_total));
        const uint32_t eb = (uint32_t)std::min<uint64_t>((h_total + 255) / 256, 16384);
        expand_kernel<false><<<eb, 256, 0, st>>>(ws->sorted.p, ws->rid.p, ws->starts.p, h_total, pbits, d_class,
                                                 n, require_class_diff, heavy_df, ws->cnt.p, nullptr, nullptr);
        size_t t5 = 0;
        PG(rocprim::exclusive_scan(nullptr, t5, ws->cnt.p, ws->offs.p, 0ull, (size_t)h_total,
                                   rocprim::plus<unsigned long long>(), st));
        if (t5 > ws->tmp.n) PG(ws->tmp.reserve(t5));
        PG(rocprim::exclusive_scan(ws->tmp.p, t5, ws->cnt.p, ws->offs.p, 0ull, (size_t)h_total,
                                   rocprim::plus<unsigned long long>(), st));
        unsigned long long last_off = 0;
        uint32_t last_cnt = 0;
        PG(hipMemcpyAsync(&last_off, ws->offs.p + (h_total - 1), 8, hipMemcpyDeviceToHost, st));
        PG(hipMemcpyAsync(&last_cnt, ws->cnt.p + (h_total - 1), 4, hipMemcpyDeviceToHost, st));
        PG(hipStreamSynchronize(st));
        n_inc = last_off + last_cnt;
        if (n_inc) {
            PG(ws->inc.reserve(n_inc));
            PG(ws->inc_sorted.reserve(n_inc));
            expand_kernel<true><<<eb, 256, 0, st>>>(ws->sorted.p, ws->rid.p, ws->starts.p, h_total, pbits, d_class,
                                                    n, require_class_diff, heavy_df, nullptr, ws->offs.p, ws->inc.p);
        }
    }
    if (stats) stats->incidences = n_inc;
    if (n_inc == 0) return KMP_OK;

    // 4. sort pair keys, run-length encode -> (pair, w) in canonical order
    const unsigned pair_bits = bits_for((uint64_t)n * n);
    PG(ws->uniq.reserve(n_inc));
    PG(ws->w.reserve(n_inc));
    PG(ws->keep.reserve(n_inc));
    PG(ws->pos.reserve(std::max<uint64_t>(n, n_inc)));
    size_t t2 = 0, t3 = 0, t4 = 0;
    PG(rocprim::radix_sort_keys(nullptr, t2, ws->inc.p, ws->inc_sorted.p, (size_t)n_inc, 0u, pair_bits, st));
    PG(rocprim::run_length_encode(nullptr, t3, ws->inc_sorted.p, (unsigned int)n_inc, ws->uniq.p, ws->w.p,
                                  ws->small.p + 1, st));
    PG(rocprim::exclusive_scan(nullptr, t4, ws->keep.p, ws->pos.p, 0u, (size_t)n_inc, rocprim::plus<uint32_t>(), st));
    PG(ws->tmp.reserve(std::max({t2, t3, t4, ws->tmp.n})));
    PG(rocprim::radix_sort_keys(ws->tmp.p, t2, ws->inc.p, ws->inc_sorted.p, (size_t)n_inc, 0u, pair_bits, st));
    PG(rocprim::run_length_encode(ws->tmp.p, t3, ws->inc_sorted.p, (unsigned int)n_inc, ws->uniq.p, ws->w.p,
                                  ws->small.p + 1, st));
    // 5. keep w >= min_shared (order preserved) and unpack
    const uint32_t kb = (uint32_t)std::min<uint64_t>((n_inc + 255) / 256, 8192);
    keep_flags_kernel<<<kb, 256, 0, st>>>(ws->w.p, ws->small.p + 1, min_shared, ws->keep.p, n_inc);
    PG(rocprim::exclusive_scan(ws->tmp.p, t4, ws->keep.p, ws->pos.p, 0u, (size_t)n_inc, rocprim::plus<uint32_t>(), st));
    uint32_t h_uniq = 0, last_pos = 0, last_keep = 0;
    PG(hipMemcpyAsync(&h_uniq, ws->small.p + 1, 4, hipMemcpyDeviceToHost, st));
    PG(hipMemcpyAsync(&last_pos, ws->pos.p + (n_inc - 1), 4, hipMemcpyDeviceToHost, st));
    PG(hipMemcpyAsync(&last_keep, ws->keep.p + (n_inc - 1), 4, hipMemcpyDeviceToHost, st));
    PG(hipStreamSynchronize(st));
    const uint64_t ne = (uint64_t)last_pos + last_keep;
    if (stats) stats->pairs = h_uniq;
    *n_edges = ne;
    if (ne > cap) return KMP_EOVERFLOW;
    emit_edges_kernel<<<kb, 256, 0, st>>>(ws->uniq.p, ws->w.p, ws->small.p + 1, n, min_shared, ws->pos.p, d_p, d_q,
                                          d_w, cap);
    PG(hipGetLastError());
    return KMP_OK;
}

#undef PG

}  // extern "C"
