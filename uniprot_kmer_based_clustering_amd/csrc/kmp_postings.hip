// kmp_postings.hip — the postings engine: the reference's own pair algorithm restated for the
// GPU as sort / expand / reduce.
//
//   reference (file:line)                                  here
//   Protein::new windows + codes (protein.rs:82-94)        residue_keys_kernel: one key per window
//   per-protein sort + dedup (main.rs:280-282)             duplicates of (k-mer, p) end up adjacent
//                                                          after the stable code sort; skipped there
//   global df: sorted Vec<(kmer, df)> (main.rs:77-122)     radix sort of the keys on the code bits;
//                                                          one run per distinct k-mer, df = distinct
//                                                          proteins in the run
//   repeat split df >= 2 (main.rs:127-149)                 runs with df >= 2
//   Graph::new: C(df,2) KmerEdge::Single per k-mer         expand_kernel: every (k-mer, p, q) incidence
//     (graph/mod.rs:39-193, vertex.rs:59-140)                of a run, one thread per run element
//   remove_uninteresting_edges (mod.rs:549-697)            class test fused into the expansion
//   combine_edges: Group per pair, len = w (mod.rs:322-546) radix sort of pair keys p*N+q, run-length
//                                                          encode: run length = w; the runs come out in
//                                                          canonical (p, q) order
// Work is O(Σ C(df,2)) like the reference (no N² scan).
//
// Key layout (u64): [ code | class (16 bits, when it fits) | p (pbits) ].  Only the code bits are
// sorted; the sort is stable and keys are laid out in protein order, so every run lists its
// proteins ascending.  Carrying the class in the key keeps the expansion free of random loads.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_run_length_encode.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cstdint>
#include <vector>

#include "kmerpair.h"
#include "kmp_internal.hpp"

using namespace kmp;

namespace {

__constant__ CodeLut c_lut = make_lut();

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

unsigned bits_for(uint64_t v) {  // bits needed for values < v
    unsigned b = 0;
    while (b < 64 && (v - 1) >> b) ++b;
    return b ? b : 1;
}

constexpr unsigned long long kNoKey = ~0ull;
constexpr unsigned kClsBits = 16;

struct Layout {
    unsigned pbits;   // protein index bits
    unsigned shift;   // code starts here: pbits (+ kClsBits when the class is in the key)
    unsigned end_bit; // shift + code bits
    bool cls_in_key;
};

Layout make_layout(uint32_t n, int k) {
    Layout l;
    l.pbits = bits_for(n);
    const unsigned cbits = bits_for(pow21(k));
    l.cls_in_key = l.pbits + kClsBits + cbits <= 64;
    l.shift = l.pbits + (l.cls_in_key ? kClsBits : 0);
    l.end_bit = l.shift + cbits;
    return l;
}

__device__ __forceinline__ unsigned long long make_key(uint32_t code, uint16_t c, uint32_t p, unsigned pbits,
                                                       unsigned shift, bool cls_in_key) {
    unsigned long long x = ((unsigned long long)code << shift) | p;
    if (cls_in_key) x |= (unsigned long long)c << pbits;
    return x;
}

// keys of the unfiltered K(p) slots: K(p)[t] for t < |K(p)|, kNoKey for the rest of the region;
// block n fills the tail of the buffer past the last region (no memset needed)
__global__ __launch_bounds__(256) void set_keys_kernel(const uint32_t* __restrict__ set,
                                                       const uint32_t* __restrict__ set_len,
                                                       const uint64_t* __restrict__ res_off,
                                                       const uint16_t* __restrict__ cls, uint32_t n, uint64_t slots,
                                                       Layout lay, unsigned long long* __restrict__ keys) {
    const uint32_t p = blockIdx.x;
    if (p == n) {
        for (uint64_t i = set_base(res_off[n], n) + threadIdx.x; i < slots; i += 256) keys[i] = kNoKey;
        return;
    }
    const uint64_t b = set_base(res_off[p], p), e = set_base(res_off[p + 1], p + 1);
    const uint32_t len = set_len[p];
    const uint16_t c = cls[p];
    for (uint64_t i = b + threadIdx.x; i < e; i += 256) {
        const uint64_t o = i - b;
        keys[i] = o < len ? make_key(set[i], c, p, lay.pbits, lay.shift, lay.cls_in_key) : kNoKey;
    }
}

// one key per window straight from the residues (Protein::new, protein.rs:82-94: window j of
// protein p is residues [j, j+k), radix-21, first residue most significant); same slot layout
constexpr int kResThreads = 256;
__global__ __launch_bounds__(kResThreads) void residue_keys_kernel(const uint8_t* __restrict__ res,
                                                                   const uint64_t* __restrict__ res_off,
                                                                   const uint16_t* __restrict__ cls, uint32_t n,
                                                                   int k, uint64_t slots, Layout lay,
                                                                   unsigned long long* __restrict__ keys) {
    const uint32_t p = blockIdx.x;
    if (p == n) {
        for (uint64_t i = set_base(res_off[n], n) + threadIdx.x; i < slots; i += kResThreads) keys[i] = kNoKey;
        return;
    }
    const uint64_t off = res_off[p], L = res_off[p + 1] - off;
    const uint64_t nw = L >= (uint64_t)k ? L - k + 1 : 0;
    const uint64_t b = set_base(off, p), e = set_base(res_off[p + 1], p + 1);
    const uint16_t c = cls[p];
    for (uint64_t i = b + threadIdx.x; i < e; i += kResThreads) {
        const uint64_t j = i - b;
        unsigned long long x = kNoKey;
        if (j < nw) {
            uint32_t v = 0;
            for (int t = 0; t < k; ++t) v = v * kRadix + c_lut.v[res[off + j + t]];
            x = make_key(v, c, p, lay.pbits, lay.shift, lay.cls_in_key);
        }
        keys[i] = x;
    }
}

enum : int { kStSumS, kStDistinct, kStRepeat, kStCdf2, kStMaxDf, kStHeavy, kStInc, kStN };

constexpr int kExpThreads = 256;
constexpr int kExpRounds = 8;
constexpr uint64_t kExpChunk = (uint64_t)kExpThreads * kExpRounds;  // keys per workgroup

__device__ __forceinline__ unsigned long long stat_op(int t, unsigned long long a, unsigned long long b) {
    return t == kStMaxDf ? (a > b ? a : b) : a + b;
}

// exclusive scan of one value per thread over the workgroup; returns (prefix, total)
__device__ __forceinline__ void block_scan(uint32_t v, uint32_t& excl, uint32_t& total, uint32_t* wave_tot) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) wave_tot[w] = x;
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kExpThreads / 64; ++i) {
        const uint32_t t = wave_tot[i];
        before += i < w ? t : 0;
        tot += t;
    }
    __syncthreads();
    excl = before + x - v;
    total = tot;
}

// Σ C(df,2) incidence expansion (vertex.rs:103-137) with the AMR test of mod.rs:580-587.
// Element i (a key of protein p) is the smaller protein of every pair it forms with a later,
// non-duplicate element j of its run: pair key p * N + q.  The run's extent is found by scanning
// forward while the code matches.  Workgroup b owns keys [b*kExpChunk, (b+1)*kExpChunk).
//   kWrite = false: per-key kept-partner counts, the workgroup total and, at run heads, the df
//                   statistics (per-workgroup partials, no atomics);
//   kWrite = true:  workgroup offset (scan of the totals) + in-workgroup scan of the counts,
//                   then the pair keys are written there.
template <bool kWrite, bool kClsKey>
__global__ __launch_bounds__(kExpThreads) void expand_kernel(const unsigned long long* __restrict__ k, uint64_t slots,
                                                             Layout lay, const uint16_t* __restrict__ cls,
                                                             uint32_t n_prot, int require_diff, uint32_t heavy_df,
                                                             uint32_t* __restrict__ counts,
                                                             unsigned long long* __restrict__ block_stats,
                                                             unsigned long long* __restrict__ block_tot,
                                                             const unsigned long long* __restrict__ block_off,
                                                             unsigned long long* __restrict__ out) {
    __shared__ uint32_t wave_tot[kExpThreads / 64];
    const unsigned long long pmask = (1ull << lay.pbits) - 1;
    const unsigned shift = lay.shift;
    const bool bounded = heavy_df != 0xFFFFFFFFu;
    const uint64_t base = blockIdx.x * kExpChunk;
    unsigned long long st[kStN] = {0, 0, 0, 0, 0, 0, 0};
    unsigned long long o = kWrite ? block_off[blockIdx.x] : 0ull;
    for (int r = 0; r < kExpRounds; ++r) {
        const uint64_t i = base + (uint64_t)r * kExpThreads + threadIdx.x;
        const unsigned long long x = i < slots ? k[i] : kNoKey;
        const unsigned long long prev = (i > 0 && i < slots) ? k[i - 1] : kNoKey;
        // kNoKey sorts last, so a valid key's predecessor is valid or absent (i == 0)
        const bool live = x != kNoKey && x != prev;  // not padding, not a duplicate window of p
        const unsigned long long code = x >> shift;
        const bool head = live && (i == 0 || (prev >> shift) != code);
        uint32_t c = 0;
        if (kWrite) {
            uint32_t excl, total;
            const uint32_t mine = i < slots ? counts[i] : 0u;
            block_scan(mine, excl, total, wave_tot);
            if (mine) {
                unsigned long long pos = o + excl;
                const uint32_t p = (uint32_t)(x & pmask);
                const uint32_t cp = kClsKey ? (uint32_t)((x >> lay.pbits) & 0xFFFFu) : cls[p];
                const unsigned long long row = (unsigned long long)p * n_prot;
                unsigned long long last = x;
                for (uint64_t j = i + 1; j < slots; ++j) {
                    const unsigned long long y = k[j];
                    if ((y >> shift) != code) break;
                    if (y == last) continue;
                    last = y;
                    const uint32_t q = (uint32_t)(y & pmask);
                    const uint32_t cq = kClsKey ? (uint32_t)((y >> lay.pbits) & 0xFFFFu) : cls[q];
                    if (require_diff && cq == cp) continue;
                    out[pos++] = row + q;
                }
            }
            o += total;
            continue;
        }
        if (live) {
            uint64_t f = 1;  // df of the run (exact at heads; exact everywhere when bounded)
            if (bounded && !head) {
                unsigned long long last = x;
                for (uint64_t s = i; s > 0; --s) {
                    const unsigned long long y = k[s - 1];
                    if ((y >> shift) != code) break;
                    if (y != last) ++f;
                    last = y;
                }
            }
            const uint32_t p = (uint32_t)(x & pmask);
            const uint32_t cp = kClsKey ? (uint32_t)((x >> lay.pbits) & 0xFFFFu) : cls[p];
            unsigned long long last = x;
            uint64_t after = 0;
            for (uint64_t j = i + 1; j < slots; ++j) {
                const unsigned long long y = k[j];
                if ((y >> shift) != code) break;
                if (y == last) continue;
                last = y;
                ++after;
                const uint32_t q = (uint32_t)(y & pmask);
                const uint32_t cq = kClsKey ? (uint32_t)((y >> lay.pbits) & 0xFFFFu) : cls[q];
                c += !require_diff || cq != cp;
            }
            f += after;
            if (f > heavy_df) c = 0;
            st[kStSumS] += 1;
            if (head) {
                st[kStDistinct] += 1;
                st[kStRepeat] += f >= 2;
                if (f <= heavy_df) st[kStCdf2] += f * (f - 1) / 2;
                else st[kStHeavy] += f;
                st[kStMaxDf] = f > st[kStMaxDf] ? f : st[kStMaxDf];
            }
        }
        if (i < slots) counts[i] = c;
        st[kStInc] += c;
    }
    if (kWrite) return;
    __shared__ unsigned long long red[kExpThreads / 64][kStN];
#pragma unroll
    for (int t = 0; t < kStN; ++t) {
        unsigned long long v = st[t];
        for (int s = 32; s > 0; s >>= 1) v = stat_op(t, v, __shfl_down(v, s));
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][t] = v;
    }
    __syncthreads();
    if (threadIdx.x < kStN) {
        const int t = threadIdx.x;
        unsigned long long v = red[0][t];
        for (int w = 1; w < kExpThreads / 64; ++w) v = stat_op(t, v, red[w][t]);
        block_stats[(uint64_t)blockIdx.x * kStN + t] = v;
        if (t == kStInc) block_tot[blockIdx.x] = v;
    }
}

// reduction of the per-workgroup statistics: one workgroup
__global__ __launch_bounds__(1024) void reduce_stats_kernel(const unsigned long long* __restrict__ bs, uint32_t nb,
                                                            unsigned long long* __restrict__ acc) {
    __shared__ unsigned long long red[16][kStN];
    unsigned long long v[kStN] = {0, 0, 0, 0, 0, 0, 0};
    for (uint32_t b = threadIdx.x; b < nb; b += 1024)
#pragma unroll
        for (int t = 0; t < kStN; ++t) v[t] = stat_op(t, v[t], bs[(uint64_t)b * kStN + t]);
#pragma unroll
    for (int t = 0; t < kStN; ++t) {
        for (int s = 32; s > 0; s >>= 1) v[t] = stat_op(t, v[t], __shfl_down(v[t], s));
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][t] = v[t];
    }
    __syncthreads();
    if (threadIdx.x < kStN) {
        const int t = threadIdx.x;
        unsigned long long x = red[0][t];
        for (int w = 1; w < 16; ++w) x = stat_op(t, x, red[w][t]);
        acc[t] = x;
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
        const uint32_t o = pos ? pos[i] : i;
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
    Grow<unsigned long long> keys, sorted, inc, inc_sorted, uniq, bstats, btot, boff;
    Grow<uint32_t> w, keep, pos, small, cnt;
    Grow<char> tmp;
    bool timing = false;
    hipEvent_t ev[KMP_POSTINGS_STAGES + 1] = {};
    ~kmp_postings() {
        keys.release(); sorted.release(); inc.release(); inc_sorted.release(); uniq.release();
        bstats.release(); btot.release(); boff.release();
        w.release(); keep.release(); pos.release(); small.release(); cnt.release(); tmp.release();
        for (auto& e : ev)
            if (e) (void)hipEventDestroy(e);
    }
    void mark(int stage, hipStream_t st) {
        if (timing) (void)hipEventRecord(ev[stage], st);
    }
};

#define PG(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) return e_ == hipErrorOutOfMemory ? KMP_ENOMEM : KMP_EDEVICE; \
    } while (0)

namespace {

// Everything after the keys are in ws->keys: stable code sort, count/scan/write, pair sort,
// run-length encode, min_shared filter, unpack.  Stage marks: 1 keys done, 2 code sort,
// 3 count + offsets, 4 write, 5 pair sort, 6 run-length encode + emit.
int postings_core(kmp_postings* ws, uint64_t slots, const Layout& lay, const uint16_t* d_class, uint32_t n,
                  uint32_t heavy_df, uint32_t min_shared, int require_class_diff, uint32_t* d_p, uint32_t* d_q,
                  uint32_t* d_w, uint64_t cap, uint64_t* n_edges, kmp_postings_stats* stats, hipStream_t st) {
    // 1. stable sort on the code bits: runs = distinct k-mers, proteins ascending inside a run
    size_t t_sort = 0;
    PG(rocprim::radix_sort_keys(nullptr, t_sort, ws->keys.p, ws->sorted.p, (size_t)slots, lay.shift, lay.end_bit,
                                st));
    PG(ws->tmp.reserve(std::max(t_sort, ws->tmp.n)));
    PG(rocprim::radix_sort_keys(ws->tmp.p, t_sort, ws->keys.p, ws->sorted.p, (size_t)slots, lay.shift, lay.end_bit,
                                st));
    ws->mark(2, st);

    // 2. count pass (+ df statistics), workgroup offsets
    const uint64_t nb64 = (slots + kExpChunk - 1) / kExpChunk;
    if (nb64 > 0x7FFFFFFFull) return KMP_EINVAL;
    const uint32_t nb = (uint32_t)nb64;
    PG(ws->cnt.reserve(slots));
    PG(ws->bstats.reserve((uint64_t)nb * kStN + kStN));
    PG(ws->btot.reserve(nb));
    PG(ws->boff.reserve(nb));
    unsigned long long* acc_d = ws->bstats.p + (uint64_t)nb * kStN;
    if (lay.cls_in_key)
        expand_kernel<false, true><<<nb, kExpThreads, 0, st>>>(ws->sorted.p, slots, lay, d_class, n, require_class_diff,
                                                               heavy_df, ws->cnt.p, ws->bstats.p, ws->btot.p, nullptr,
                                                               nullptr);
    else
        expand_kernel<false, false><<<nb, kExpThreads, 0, st>>>(ws->sorted.p, slots, lay, d_class, n,
                                                                require_class_diff, heavy_df, ws->cnt.p, ws->bstats.p,
                                                                ws->btot.p, nullptr, nullptr);
    reduce_stats_kernel<<<1, 1024, 0, st>>>(ws->bstats.p, nb, acc_d);
    size_t t_scan = 0;
    PG(rocprim::exclusive_scan(nullptr, t_scan, ws->btot.p, ws->boff.p, 0ull, (size_t)nb,
                               rocprim::plus<unsigned long long>(), st));
    PG(ws->tmp.reserve(std::max(t_scan, ws->tmp.n)));
    PG(rocprim::exclusive_scan(ws->tmp.p, t_scan, ws->btot.p, ws->boff.p, 0ull, (size_t)nb,
                               rocprim::plus<unsigned long long>(), st));
    ws->mark(3, st);
    unsigned long long acc[kStN];
    PG(hipMemcpyAsync(acc, acc_d, sizeof acc, hipMemcpyDeviceToHost, st));
    PG(hipStreamSynchronize(st));
    const unsigned long long n_inc = acc[kStInc];
    if (stats) {
        stats->sum_S = acc[kStSumS];
        stats->distinct = acc[kStDistinct];
        stats->repeat = acc[kStRepeat];
        stats->sum_cdf2_light = acc[kStCdf2];
        stats->max_df = acc[kStMaxDf];
        stats->heavy_entries = acc[kStHeavy];
        stats->incidences = n_inc;
    }
    if (n_inc == 0) {
        for (int s = 4; s <= KMP_POSTINGS_STAGES; ++s) ws->mark(s, st);
        return KMP_OK;
    }
    if (n_inc > 0xFFFFFFFFull) return KMP_ENOMEM;  // run-length counts are u32

    // 3. write pass
    PG(ws->inc.reserve(n_inc));
    PG(ws->inc_sorted.reserve(n_inc));
    if (lay.cls_in_key)
        expand_kernel<true, true><<<nb, kExpThreads, 0, st>>>(ws->sorted.p, slots, lay, d_class, n, require_class_diff,
                                                              heavy_df, ws->cnt.p, nullptr, nullptr, ws->boff.p,
                                                              ws->inc.p);
    else
        expand_kernel<true, false><<<nb, kExpThreads, 0, st>>>(ws->sorted.p, slots, lay, d_class, n,
                                                               require_class_diff, heavy_df, ws->cnt.p, nullptr,
                                                               nullptr, ws->boff.p, ws->inc.p);
    ws->mark(4, st);

    // 4. sort pair keys p*N+q, run-length encode -> (pair, w) in canonical order
    const unsigned pair_bits = bits_for((uint64_t)n * n);
    PG(ws->uniq.reserve(n_inc));
    PG(ws->w.reserve(n_inc));
    PG(ws->small.reserve(16));
    const bool filter_w = min_shared > 1;
    if (filter_w) {
        PG(ws->keep.reserve(n_inc));
        PG(ws->pos.reserve(n_inc));
    }
    size_t t2 = 0, t3 = 0, t4 = 0;
    PG(rocprim::radix_sort_keys(nullptr, t2, ws->inc.p, ws->inc_sorted.p, (size_t)n_inc, 0u, pair_bits, st));
    PG(rocprim::run_length_encode(nullptr, t3, ws->inc_sorted.p, (unsigned int)n_inc, ws->uniq.p, ws->w.p,
                                  ws->small.p + 1, st));
    if (filter_w)
        PG(rocprim::exclusive_scan(nullptr, t4, ws->keep.p, ws->pos.p, 0u, (size_t)n_inc, rocprim::plus<uint32_t>(),
                                   st));
    PG(ws->tmp.reserve(std::max({t2, t3, t4, ws->tmp.n})));
    PG(rocprim::radix_sort_keys(ws->tmp.p, t2, ws->inc.p, ws->inc_sorted.p, (size_t)n_inc, 0u, pair_bits, st));
    ws->mark(5, st);
    PG(rocprim::run_length_encode(ws->tmp.p, t3, ws->inc_sorted.p, (unsigned int)n_inc, ws->uniq.p, ws->w.p,
                                  ws->small.p + 1, st));
    // 5. keep w >= min_shared (order preserved) and unpack
    const uint32_t kb = (uint32_t)std::min<uint64_t>((n_inc + 255) / 256, 8192);
    uint32_t h_uniq = 0, last_pos = 0, last_keep = 0;
    if (filter_w) {
        keep_flags_kernel<<<kb, 256, 0, st>>>(ws->w.p, ws->small.p + 1, min_shared, ws->keep.p, n_inc);
        PG(rocprim::exclusive_scan(ws->tmp.p, t4, ws->keep.p, ws->pos.p, 0u, (size_t)n_inc,
                                   rocprim::plus<uint32_t>(), st));
        PG(hipMemcpyAsync(&last_pos, ws->pos.p + (n_inc - 1), 4, hipMemcpyDeviceToHost, st));
        PG(hipMemcpyAsync(&last_keep, ws->keep.p + (n_inc - 1), 4, hipMemcpyDeviceToHost, st));
    }
    PG(hipMemcpyAsync(&h_uniq, ws->small.p + 1, 4, hipMemcpyDeviceToHost, st));
    PG(hipStreamSynchronize(st));
    const uint64_t ne = filter_w ? (uint64_t)last_pos + last_keep : h_uniq;
    if (stats) stats->pairs = h_uniq;
    *n_edges = ne;
    if (ne > cap) return KMP_EOVERFLOW;
    emit_edges_kernel<<<kb, 256, 0, st>>>(ws->uniq.p, ws->w.p, ws->small.p + 1, n, min_shared,
                                          filter_w ? ws->pos.p : nullptr, d_p, d_q, d_w, cap);
    ws->mark(6, st);
    PG(hipGetLastError());
    return KMP_OK;
}

void finish_timing(kmp_postings* ws, kmp_postings_stats* stats, hipStream_t st) {
    if (!ws->timing || !stats) return;
    (void)hipStreamSynchronize(st);
    for (int s = 0; s < KMP_POSTINGS_STAGES; ++s) {
        float ms = 0.f;
        stats->stage_ms[s] = hipEventElapsedTime(&ms, ws->ev[s], ws->ev[s + 1]) == hipSuccess ? ms : -1.f;
    }
}

int postings_args(kmp_postings* ws, int k, uint64_t* n_edges, kmp_postings_stats* stats, uint32_t* d_p,
                  uint32_t* d_q, uint32_t* d_w, uint64_t cap) {
    if (!ws || !n_edges || k < 1 || k > kMaxK) return KMP_EINVAL;
    *n_edges = 0;
    if (stats) *stats = kmp_postings_stats{};
    if (cap && (!d_p || !d_q || !d_w)) return KMP_EINVAL;
    return KMP_OK;
}

}  // namespace

extern "C" {

int kmp_postings_create(kmp_postings** ws) {
    if (!ws) return KMP_EINVAL;
    *ws = new (std::nothrow) kmp_postings;
    return *ws ? KMP_OK : KMP_ENOMEM;
}

void kmp_postings_destroy(kmp_postings* ws) { delete ws; }

int kmp_postings_set_timing(kmp_postings* ws, int enable) {
    if (!ws) return KMP_EINVAL;
    if (enable && !ws->ev[0])
        for (auto& e : ws->ev) PG(hipEventCreate(&e));
    ws->timing = enable != 0;
    return KMP_OK;
}

int kmp_dev_pairs_postings(kmp_postings* ws, const uint32_t* d_set, const uint32_t* d_set_len,
                           const uint64_t* d_res_off, const uint16_t* d_class, uint32_t n, int k, uint64_t slots,
                           uint32_t heavy_df, uint32_t min_shared, int require_class_diff, uint32_t* d_p,
                           uint32_t* d_q, uint32_t* d_w, uint64_t cap, uint64_t* n_edges,
                           kmp_postings_stats* stats, void* stream) {
    int rc = postings_args(ws, k, n_edges, stats, d_p, d_q, d_w, cap);
    if (rc != KMP_OK || n < 2) return rc;
    if (!d_set || !d_set_len || !d_res_off || !d_class) return KMP_EINVAL;
    const Layout lay = make_layout(n, k);
    if (lay.end_bit > 64) return KMP_EINVAL;
    hipStream_t st = as_stream(stream);
    PG(ws->keys.reserve(slots));
    PG(ws->sorted.reserve(slots));
    ws->mark(0, st);
    set_keys_kernel<<<n + 1, 256, 0, st>>>(d_set, d_set_len, d_res_off, d_class, n, slots, lay, ws->keys.p);
    ws->mark(1, st);
    rc = postings_core(ws, slots, lay, d_class, n, heavy_df < 2 ? 2 : heavy_df, min_shared < 1 ? 1 : min_shared,
                       require_class_diff, d_p, d_q, d_w, cap, n_edges, stats, st);
    if (rc == KMP_OK) finish_timing(ws, stats, st);
    return rc;
}

int kmp_dev_pairs_residues(kmp_postings* ws, const uint8_t* d_res, const uint64_t* d_res_off,
                           const uint16_t* d_class, uint32_t n, int k, uint64_t slots, uint32_t heavy_df,
                           uint32_t min_shared, int require_class_diff, uint32_t* d_p, uint32_t* d_q, uint32_t* d_w,
                           uint64_t cap, uint64_t* n_edges, kmp_postings_stats* stats, void* stream) {
    int rc = postings_args(ws, k, n_edges, stats, d_p, d_q, d_w, cap);
    if (rc != KMP_OK || n < 2) return rc;
    if (!d_res || !d_res_off || !d_class) return KMP_EINVAL;
    const Layout lay = make_layout(n, k);
    if (lay.end_bit > 64) return KMP_EINVAL;
    hipStream_t st = as_stream(stream);
    PG(ws->keys.reserve(slots));
    PG(ws->sorted.reserve(slots));
    ws->mark(0, st);
    residue_keys_kernel<<<n + 1, kResThreads, 0, st>>>(d_res, d_res_off, d_class, n, k, slots, lay, ws->keys.p);
    ws->mark(1, st);
    rc = postings_core(ws, slots, lay, d_class, n, heavy_df < 2 ? 2 : heavy_df, min_shared < 1 ? 1 : min_shared,
                       require_class_diff, d_p, d_q, d_w, cap, n_edges, stats, st);
    if (rc == KMP_OK) finish_timing(ws, stats, st);
    return rc;
}

}  // extern "C"

#undef PG
