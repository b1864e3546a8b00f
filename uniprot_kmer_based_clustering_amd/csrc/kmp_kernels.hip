// kmp_kernels.hip — gfx950 (CDNA4) kernels of the k-mer pair path and their C-ABI
// device-stage entry points (include/kmerpair.h, "device stages").
//
// Path (reference file:line it replaces):
//   build_sets_kernel   Protein::new windows + radix-21 codes (src/protein.rs:29-37,107-132)
//                       fused with the per-protein sort+dedup of src/main.rs:99-101,187-189
//   mark/compact        remove_unique_five_mers (src/protein.rs:151-162) with the df>=2 test
//                       of src/main.rs:127-149 as two bitmaps over the 21^k code space
//   pair_kernel         Graph::new + remove_uninteresting_edges + combine_edges
//                       (src/graph/mod.rs:39-193, :549-697, :322-546): w(p,q) = |K(p) ∩ K(q)|
//                       for every p < q of a row tile × column range, class filter, emit
//   sort edges          the reference's single-thread (p, q) edge order (vertex.rs:100)
//
// Wave = 64 lanes everywhere; ballots are 64-bit.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cstdlib>
#include <vector>

#include "kmerpair.h"
#include "kmp_internal.hpp"

using namespace kmp;

namespace {

__constant__ CodeLut c_lut = make_lut();

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// number of set bits of m strictly below this lane
__device__ __forceinline__ uint32_t mask_rank(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint32_t next_pow2(uint32_t n) {
    return n <= 1 ? 1u : 1u << (32 - __clz(n - 1));
}

// Block-wide ordered compaction step: every thread offers (keep, value) for position
// `slot` of the block's 256-element chunk; kept values land at out[carry + rank] in input
// order.  Returns the number kept by the whole chunk.  Uses wave ballots + 4 LDS words.
template <int kThreads>
__device__ __forceinline__ uint32_t block_compact(bool keep, uint32_t value, uint32_t* out, uint32_t carry,
                                                  uint32_t* wave_tot) {
    constexpr int kWaves = kThreads / 64;
    const uint64_t m = __ballot(keep);
    const uint32_t w = threadIdx.x >> 6;
    if (lane_id() == 0) wave_tot[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int i = 0; i < kWaves; ++i) {
        const uint32_t t = wave_tot[i];
        before += (i < (int)w) ? t : 0u;
        total += t;
    }
    if (keep) out[carry + before + mask_rank(m)] = value;
    __syncthreads();  // wave_tot reused by the next chunk
    return total;
}

// Ascending bitonic sort of s[0, n) in LDS with the "flip" first stage, so every comparator
// is ascending and positions >= n behave as +inf without being stored (no padding writes).
template <int kThreads>
__device__ void bitonic_sort_lds(uint32_t* s, uint32_t n) {
    if (n <= 1) return;
    const uint32_t n2 = next_pow2(n);
    const uint32_t pairs = n2 >> 1;
    for (uint32_t m = 2; m <= n2; m <<= 1) {
        const uint32_t half = m >> 1;
        const uint32_t hl = __builtin_ctz(half);
        for (uint32_t t = threadIdx.x; t < pairs; t += kThreads) {
            const uint32_t blk = t >> hl, o = t & (half - 1);
            const uint32_t i = blk * m + o, l = blk * m + m - 1 - o;
            if (l < n) {
                const uint32_t a = s[i], b = s[l];
                if (a > b) { s[i] = b; s[l] = a; }
            }
        }
        __syncthreads();
        for (uint32_t j = half >> 1; j > 0; j >>= 1) {
            const uint32_t jl = __builtin_ctz(j);
            for (uint32_t t = threadIdx.x; t < pairs; t += kThreads) {
                const uint32_t i = ((t >> jl) << (jl + 1)) + (t & (j - 1)), l = i + j;
                if (l < n) {
                    const uint32_t a = s[i], b = s[l];
                    if (a > b) { s[i] = b; s[l] = a; }
                }
            }
            __syncthreads();
        }
    }
}

// The same network over global memory, one workgroup per protein (long proteins only).
template <int kThreads>
__device__ void bitonic_sort_global(uint32_t* s, uint32_t n) {
    if (n <= 1) return;
    const uint32_t n2 = next_pow2(n);
    const uint32_t pairs = n2 >> 1;
    for (uint32_t m = 2; m <= n2; m <<= 1) {
        const uint32_t half = m >> 1;
        for (uint32_t j = half; j > 0; j >>= 1) {
            for (uint32_t t = threadIdx.x; t < pairs; t += kThreads) {
                uint32_t i, l;
                if (j == half) {
                    const uint32_t blk = t / half, o = t % half;
                    i = blk * m + o;
                    l = blk * m + m - 1 - o;
                } else {
                    i = (t / j) * 2 * j + (t % j);
                    l = i + j;
                }
                if (l < n) {
                    const uint32_t a = s[i], b = s[l];
                    if (a > b) { s[i] = b; s[l] = a; }
                }
            }
            __threadfence_block();
            __syncthreads();
        }
    }
}

// ------------------------------------------------------------------------------------
// Protein::new windows (protein.rs:107-132): every window's code, position order.
constexpr int kExtractThreads = 256;
__global__ __launch_bounds__(kExtractThreads) void extract_kernel(const uint8_t* __restrict__ res,
                                                                  const uint64_t* __restrict__ res_off,
                                                                  int k, uint32_t* __restrict__ codes) {
    const uint32_t p = blockIdx.x;
    const uint64_t off = res_off[p];
    const uint64_t L = res_off[p + 1] - off;
    const uint64_t nw = L >= (uint64_t)k ? L - k + 1 : 0;
    const uint64_t base = set_base(off, p);
    for (uint64_t j = threadIdx.x; j < nw; j += kExtractThreads) {
        uint32_t v = 0;
        for (int i = 0; i < k; ++i) v = v * kRadix + c_lut.v[res[off + j + i]];
        codes[base + j] = v;
    }
}

// Fused windows + per-protein sort + dedup (K(p)), one workgroup per protein, in LDS.
constexpr int kSetThreads = 256;
__global__ __launch_bounds__(kSetThreads) void build_sets_kernel(const uint8_t* __restrict__ res,
                                                                 const uint64_t* __restrict__ res_off,
                                                                 int k, uint32_t* __restrict__ set,
                                                                 uint32_t* __restrict__ set_len) {
    __shared__ uint32_t s[KMP_LDS_SORT_MAX];
    __shared__ uint8_t rc[KMP_LDS_SORT_MAX + kMaxK];
    __shared__ uint8_t lut[256];
    __shared__ uint32_t wave_tot[kSetThreads / 64];
    const uint32_t p = blockIdx.x;
    const uint64_t off = res_off[p];
    const uint64_t L = res_off[p + 1] - off;
    const uint64_t nw64 = L >= (uint64_t)k ? L - k + 1 : 0;
    if (nw64 > KMP_LDS_SORT_MAX) return;  // block-uniform: long proteins take the global path
    const uint32_t nw = (uint32_t)nw64;
    const uint32_t t = threadIdx.x;
    lut[t] = c_lut.v[t];
    __syncthreads();
    const uint32_t Lr = nw ? nw + k - 1 : 0;  // residues that belong to some window
    for (uint32_t i = t; i < Lr; i += kSetThreads) rc[i] = lut[res[off + i]];
    __syncthreads();
    for (uint32_t j = t; j < nw; j += kSetThreads) {
        uint32_t v = 0;
        for (int i = 0; i < k; ++i) v = v * kRadix + rc[j + i];
        s[j] = v;
    }
    __syncthreads();
    bitonic_sort_lds<kSetThreads>(s, nw);
    uint32_t* out = set + set_base(off, p);
    uint32_t carry = 0;
    for (uint32_t c = 0; c < nw; c += kSetThreads) {
        const uint32_t i = c + t;
        const bool keep = i < nw && (i == 0 || s[i] != s[i - 1]);
        carry += block_compact<kSetThreads>(keep, keep ? s[i] : 0u, out, carry, wave_tot);
    }
    if (t == 0) set_len[p] = carry;
}

constexpr int kLongThreads = 1024;
__global__ __launch_bounds__(kLongThreads) void build_sets_long_kernel(const uint8_t* __restrict__ res,
                                                                       const uint64_t* __restrict__ res_off,
                                                                       int k, uint32_t* __restrict__ set,
                                                                       uint32_t* __restrict__ set_len,
                                                                       uint32_t* __restrict__ scratch) {
    __shared__ uint32_t wave_tot[kLongThreads / 64];
    const uint32_t p = blockIdx.x;
    const uint64_t off = res_off[p];
    const uint64_t L = res_off[p + 1] - off;
    const uint64_t nw64 = L >= (uint64_t)k ? L - k + 1 : 0;
    if (nw64 <= KMP_LDS_SORT_MAX) return;
    const uint32_t nw = (uint32_t)nw64;
    const uint64_t base = set_base(off, p);
    uint32_t* s = scratch + base;
    for (uint32_t j = threadIdx.x; j < nw; j += kLongThreads) {
        uint32_t v = 0;
        for (int i = 0; i < k; ++i) v = v * kRadix + c_lut.v[res[off + j + i]];
        s[j] = v;
    }
    __threadfence_block();
    __syncthreads();
    bitonic_sort_global<kLongThreads>(s, nw);
    uint32_t carry = 0;
    for (uint32_t c = 0; c < nw; c += kLongThreads) {
        const uint32_t i = c + threadIdx.x;
        const bool keep = i < nw && (i == 0 || s[i] != s[i - 1]);
        carry += block_compact<kLongThreads>(keep, keep ? s[i] : 0u, set + base, carry, wave_tot);
    }
    if (threadIdx.x == 0) set_len[p] = carry;
}

// ------------------------------------------------------------------------------------
// remove_unique_five_mers (protein.rs:151-162).  Pass 1 marks every (protein, distinct
// k-mer) occurrence in bits1; a second occurrence (bit already set) marks bits2 (df >= 2).
constexpr int kFilterThreads = 256;
__global__ __launch_bounds__(kFilterThreads) void mark_kernel(const uint32_t* __restrict__ set,
                                                              const uint32_t* __restrict__ set_len,
                                                              const uint64_t* __restrict__ res_off,
                                                              uint32_t* __restrict__ bits1,
                                                              uint32_t* __restrict__ bits2) {
    const uint32_t p = blockIdx.x;
    const uint32_t len = set_len[p];
    const uint32_t* s = set + set_base(res_off[p], p);
    // plain loads first: a k-mer already marked twice needs nothing, one already seen by another
    // protein (a set holds each k-mer once) only the second mark — at k = 5 nearly every k-mer of a
    // large batch, so the atomics (two per entry, on a 512 KB bitmap) mostly become cached loads.
    // A stale 0 falls through to the atomics: the bits only ever gain ones.
    for (uint32_t e = threadIdx.x; e < len; e += kFilterThreads) {
        const uint32_t x = s[e];
        const uint32_t bit = 1u << (x & 31u);
        if (bits2[x >> 5] & bit) continue;
        if ((bits1[x >> 5] & bit) || (atomicOr(&bits1[x >> 5], bit) & bit))
            atomicOr(&bits2[x >> 5], bit);
    }
}

__global__ __launch_bounds__(kFilterThreads) void compact_repeats_kernel(
    const uint32_t* __restrict__ set, const uint32_t* __restrict__ set_len,
    const uint64_t* __restrict__ res_off, const uint32_t* __restrict__ bits2, uint32_t* __restrict__ rep,
    uint32_t* __restrict__ rep_len) {
    __shared__ uint32_t wave_tot[kFilterThreads / 64];
    const uint32_t p = blockIdx.x;
    const uint32_t len = set_len[p];
    const uint64_t base = set_base(res_off[p], p);
    uint32_t carry = 0;
    for (uint32_t c = 0; c < len; c += kFilterThreads) {
        const uint32_t e = c + threadIdx.x;
        uint32_t x = 0;
        bool keep = false;
        if (e < len) {
            x = set[base + e];
            keep = (bits2[x >> 5] >> (x & 31u)) & 1u;
        }
        carry += block_compact<kFilterThreads>(keep, x, rep + base, carry, wave_tot);
    }
    if (threadIdx.x == 0) rep_len[p] = carry;
}

// ------------------------------------------------------------------------------------
// Dense CSR of the repeat-filtered sets (column stream of the pair kernel).
__global__ __launch_bounds__(256) void pack_dense_kernel(const uint32_t* __restrict__ rep,
                                                         const uint64_t* __restrict__ res_off,
                                                         const uint64_t* __restrict__ dense_off,
                                                         uint32_t* __restrict__ dense) {
    const uint32_t p = blockIdx.x;
    const uint64_t d = dense_off[p], len = dense_off[p + 1] - d;
    const uint32_t* s = rep + set_base(res_off[p], p);
    for (uint64_t e = threadIdx.x; e < len; e += 256) dense[d + e] = s[e];
}

// ------------------------------------------------------------------------------------
// Pair kernel.  One workgroup (16 waves) per work item = one row tile × one column chunk.
// LDS holds the row tile as
//   * a blocked Bloom filter: 4,096 64-bit blocks, 4 bits per key inside the block picked
//     by the key's top 12 hash bits (≈0.4 % false positives at a full tile; no false
//     negatives) — the only LDS access of ~all column k-mers (one ds_read_b64);
//   * an exact multiset table: the tile's k-mers counting-sorted by the same 12-bit block
//     (keys u32 + owning row u8, bucket b = [F[b], F[b+1])), read only by lanes that pass
//     the filter;
//   * per-wave hit counters.
// Each wave owns the item's columns q ≡ wave (mod 16) and streams them from HBM/L2 straight
// into registers in batches (see "Batched column stream" above).  A confirmed hit on row r bumps the wave's
// counter for r (rows with p = row_beg + r < q only: upper triangle); after the column the
// touched rows are emitted as (p, q, w) when w >= min_shared and the AMR classes differ
// (mod.rs:580-587), one global atomic per wave (ballot + mbcnt).
static_assert(kBuckets == 4 * kPairThreads, "bucket scan assumes 4 buckets per thread");
static_assert(kTileCap <= 65536, "tile positions fit the exact table");
constexpr uint32_t kEdgeBuf = 64;  // per-wave edge buffer (one global atomic per flush)
constexpr uint32_t kDefer = 48;    // per-wave list of long columns

__device__ __forceinline__ uint64_t bloom_bits(uint32_t x) {
    const uint32_t g = x * kHashMul2;
    return (1ull << (g & 63u)) | (1ull << ((g >> 6) & 63u)) | (1ull << ((g >> 12) & 63u)) |
           (1ull << ((g >> 18) & 63u));
}
__device__ __forceinline__ uint32_t bloom_block(uint32_t x) { return (x * kHashMul) >> (32 - kBloomLog2); }

// exclusive scan of one value per thread over the 1024-thread block
__device__ __forceinline__ uint32_t block_scan_1024(uint32_t v, uint32_t* wave_tot) {
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) wave_tot[w] = x;
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t i = 0; i < w; ++i) before += wave_tot[i];
    return before + x - v;
}

// Batched column stream.  A wave owns the item's columns q = qw + 16*t.  Their meta (dense
// range, class) is fetched 2*B columns at a time (lane j = column t0 + j); their k-mers in
// batches of B columns (C k-mers per lane per column), ping-pong: batch i is probed from
// registers while batch i+1's loads are in flight.  Every load of the pipelined loop is
// issued unconditionally (clamped, in-bounds addresses) so the number of younger loads at
// each use is the same on every path and the compiler's vmcnt waits stay partial; columns
// longer than 64*C k-mers are deferred to after the loop.
struct Meta {
    uint64_t beg, end;  // lane j < 2B: dense range of column t0 + j
    uint32_t cls;       // lane j < 2B: its class
};

__device__ __forceinline__ void meta_load(Meta& m, const uint64_t* __restrict__ dense_off,
                                          const uint16_t* __restrict__ cls, uint32_t qw, uint32_t t0,
                                          uint32_t ncol, uint32_t lane) {
    const uint32_t t = t0 + lane;
    const uint32_t q = qw + kPairWaves * min(t, ncol - 1);  // ncol >= 1 here: always in bounds
    const uint64_t b = dense_off[q], e = dense_off[q + 1];
    const uint32_t c = cls[q];
    const bool v = t < ncol;
    m.beg = v ? b : 0ull;
    m.end = v ? e : 0ull;
    m.cls = v ? c : 0u;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t l) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

template <uint32_t B, uint32_t C>
struct BatchX {
    uint32_t x[B][C];
};

// unconditionally issue the loads of batch columns j0 .. j0+B-1 of meta m
template <uint32_t B, uint32_t C>
__device__ __forceinline__ void batch_issue(BatchX<B, C>& b, const uint32_t* __restrict__ dense, const Meta& m,
                                            uint32_t j0, uint32_t lane) {
#pragma unroll
    for (uint32_t j = 0; j < B; ++j) {
        const uint64_t s = readlane64(m.beg, j0 + j);
        const uint32_t len = (uint32_t)(readlane64(m.end, j0 + j) - s);
#pragma unroll
        for (uint32_t i = 0; i < C; ++i) {
            const uint32_t e = lane + 64 * i;
            b.x[j][i] = dense[e < len ? s + e : 0ull];  // lanes past len read element 0 (ignored)
        }
    }
}

template <uint32_t C, uint32_t B>
__global__ __launch_bounds__(kPairThreads) void pair_kernel(
    const uint32_t* __restrict__ dense, const uint64_t* __restrict__ dense_off, const uint16_t* __restrict__ cls,
    const kmp_work_item* __restrict__ items, uint32_t min_shared, int require_diff, uint32_t* __restrict__ out_p,
    uint32_t* __restrict__ out_q, uint32_t* __restrict__ out_w, uint64_t cap, unsigned long long* __restrict__ count) {
    __shared__ uint64_t bloom[kBloomBlocks];
    __shared__ uint16_t F[kBuckets + 2];          // bucket starts (u16: the tile has <= 16384 keys)
    __shared__ uint32_t keys[kTileCap];
    __shared__ uint8_t rows[kTileCap];
    __shared__ uint32_t scratch[kPairWaves * kRowsMax + 16];  // build: u32 bucket counts; probe: hit counters
    __shared__ uint64_t tmask[kPairWaves][kRowsMax / 64];     // rows touched by the wave's current column
    __shared__ uint32_t ebuf[kPairWaves][3][kEdgeBuf];        // per-wave edge buffer (p, q, w)
    __shared__ uint16_t row_cls[kRowsMax];
    __shared__ uint32_t row_start[kRowsMax + 1];
    __shared__ uint32_t wave_tot[kPairWaves];
    __shared__ uint32_t defer[kPairWaves][kDefer];            // long columns, probed after the loop
    static_assert(kPairWaves * kRowsMax + 16 >= kBuckets + 2, "bucket counts fit the counter scratch");

    const kmp_work_item it = items[blockIdx.x];
    const uint32_t r0 = it.row_beg, nrows = it.row_end - it.row_beg;
    if (nrows == 0) return;  // padding item
    const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const uint32_t qfirst = max(it.col_beg, r0 + 1);

    // column stream: meta of pairs 0 and 1 and batch 0's k-mers are in flight during the build
    const uint32_t qw = qfirst + wave;
    const uint32_t ncol = qw < it.col_end ? (it.col_end - qw + kPairWaves - 1) / kPairWaves : 0u;
    Meta mcur, mnext;
    BatchX<B, C> xa, xb;
    if (ncol > 0) {
        meta_load(mcur, dense_off, cls, qw, 0, ncol, lane);
        meta_load(mnext, dense_off, cls, qw, 2 * B, ncol, lane);
        batch_issue(xa, dense, mcur, 0, lane);
    }

    uint32_t* Fc = scratch;  // u32 bucket counts during the build
    for (uint32_t i = tid; i < kBloomBlocks; i += kPairThreads) bloom[i] = 0;
    for (uint32_t i = tid; i < kBuckets + 2; i += kPairThreads) Fc[i] = 0;
    if (tid < kPairWaves * (kRowsMax / 64)) (&tmask[0][0])[tid] = 0;
    const uint64_t d0 = dense_off[r0];
    for (uint32_t r = tid; r <= nrows; r += kPairThreads) row_start[r] = (uint32_t)(dense_off[r0 + r] - d0);
    for (uint32_t r = tid; r < nrows; r += kPairThreads) row_cls[r] = cls[r0 + r];
    __syncthreads();
    const uint32_t ntile = row_start[nrows];

    // row tile -> Bloom blocks + bucket counts (pass 1), bucket scan, scatter (pass 2)
    for (uint32_t e = tid; e < ntile; e += kPairThreads) {
        const uint32_t x = dense[d0 + e];
        const uint32_t b = bloom_block(x);
        atomicOr(&bloom[b], bloom_bits(x));
        atomicAdd(&Fc[b + 2], 1u);
    }
    __syncthreads();
    {
        const uint32_t c0 = Fc[4 * tid + 2], c1 = Fc[4 * tid + 3], c2 = Fc[4 * tid + 4], c3 = Fc[4 * tid + 5];
        const uint32_t ex = block_scan_1024(c0 + c1 + c2 + c3, wave_tot);
        __syncthreads();
        Fc[4 * tid + 1] = ex;  // Fc[b+1] = start of bucket b (Fc[0] = 0)
        Fc[4 * tid + 2] = ex + c0;
        Fc[4 * tid + 3] = ex + c0 + c1;
        Fc[4 * tid + 4] = ex + c0 + c1 + c2;
    }
    __syncthreads();
    for (uint32_t r = wave; r < nrows; r += kPairWaves) {
        const uint32_t rb = row_start[r], re = row_start[r + 1];
        for (uint32_t e = rb + lane; e < re; e += 64) {
            const uint32_t x = dense[d0 + e];
            const uint32_t pos = atomicAdd(&Fc[bloom_block(x) + 1], 1u);
            keys[pos] = x;
            rows[pos] = (uint8_t)r;
        }
    }
    __syncthreads();  // Fc[b] .. Fc[b+1] = bucket b
    for (uint32_t i = tid; i < kBuckets + 1; i += kPairThreads) F[i] = (uint16_t)Fc[i];
    __syncthreads();
    for (uint32_t i = tid; i < kPairWaves * kRowsMax; i += kPairThreads) scratch[i] = 0;  // hit counters
    __syncthreads();
    uint32_t* cnt = scratch + wave * kRowsMax;
    uint64_t* tm = tmask[wave];
    uint32_t nbuf = 0;  // wave-uniform fill of the wave's edge buffer

    // flush the wave's edge buffer to HBM: one global atomic per kEdgeBuf edges
    auto flush = [&]() {
        if (nbuf == 0) return;
        unsigned long long first = 0;
        if (lane == 0) first = atomicAdd(count, (unsigned long long)nbuf);
        first = __shfl(first, 0);
        for (uint32_t e = lane; e < nbuf; e += 64) {
            const unsigned long long pos = first + e;
            if (pos < cap) {
                out_p[pos] = ebuf[wave][0][e];
                out_q[pos] = ebuf[wave][1][e];
                out_w[pos] = ebuf[wave][2][e];
            }
        }
        nbuf = 0;
    };

    // probe 64*C k-mers x[] of column q (lanes/registers past len are ignored)
    auto probe = [&](uint32_t q, uint32_t len, uint32_t base, const uint32_t (&x)[C], bool& hit_any) {
        const uint32_t lim = min(q - r0, nrows);  // rows with p < q
        uint64_t word[C], want[C];
        uint32_t blk[C];
#pragma unroll
        for (uint32_t i = 0; i < C; ++i) {
            blk[i] = bloom_block(x[i]);
            want[i] = bloom_bits(x[i]);
            word[i] = bloom[blk[i]];
        }
        bool any = false;
        bool pass[C];
#pragma unroll
        for (uint32_t i = 0; i < C; ++i) {
            pass[i] = base + lane + 64 * i < len && (word[i] & want[i]) == want[i];
            any |= pass[i];
        }
        if (__ballot(any) == 0) return;
#pragma unroll
        for (uint32_t i = 0; i < C; ++i) {
            if (!pass[i]) continue;
            const uint32_t be = F[blk[i] + 1];
            for (uint32_t s0 = F[blk[i]]; s0 < be; s0 += 4) {
                uint32_t kk[4];
#pragma unroll
                for (uint32_t u = 0; u < 4; ++u) kk[u] = s0 + u < be ? keys[s0 + u] : ~x[i];
#pragma unroll
                for (uint32_t u = 0; u < 4; ++u) {
                    if (kk[u] != x[i]) continue;
                    const uint32_t r = rows[s0 + u];
                    if (r < lim) {
                        atomicAdd(&cnt[r], 1u);  // no return: nothing waits
                        atomicOr(&tm[r >> 6], 1ull << (r & 63u));
                        hit_any = true;
                    }
                }
            }
        }
    };

    // emit the rows touched by column q (class cq) into the wave's edge buffer
    auto epilogue = [&](uint32_t q, uint32_t cq, bool hit_any) {
        if (__ballot(hit_any) != 0) {
#pragma unroll
            for (uint32_t i = 0; i < kRowsMax / 64; ++i) {
                const uint64_t m = tm[i];  // same word for every lane
                if (m == 0) continue;
                const uint32_t r = 64 * i + lane;
                bool ok = false;
                uint32_t wv = 0;
                if ((m >> lane) & 1ull) {
                    wv = cnt[r];
                    cnt[r] = 0;
                    ok = wv >= min_shared && (!require_diff || row_cls[r] != cq);
                }
                const uint64_t okm = __ballot(ok);
                const uint32_t nok = (uint32_t)__popcll(okm);
                if (nok == 0) continue;
                if (nbuf + nok > kEdgeBuf) flush();
                if (ok) {
                    const uint32_t slot = nbuf + mask_rank(okm);
                    ebuf[wave][0][slot] = r0 + r;
                    ebuf[wave][1][slot] = q;
                    ebuf[wave][2][slot] = wv;
                }
                nbuf += nok;
            }
            if (lane < kRowsMax / 64) tm[lane] = 0;
        }
    };

    // a column held entirely in registers (len <= 64*C): no global load
    auto column_short = [&](uint32_t q, uint32_t len, uint32_t cq, const uint32_t (&x)[C]) {
        bool hit_any = false;
        probe(q, len, 0, x, hit_any);
        epilogue(q, cq, hit_any);
    };
    // any column, loaded here (used after the batches only)
    auto column_long = [&](uint32_t q) {
        const uint64_t s = dense_off[q];
        const uint32_t len = (uint32_t)(dense_off[q + 1] - s);
        bool hit_any = false;
        for (uint32_t base = 0; base < len; base += 64 * C) {
            uint32_t x[C];
#pragma unroll
            for (uint32_t i = 0; i < C; ++i) {
                const uint32_t e = base + lane + 64 * i;
                x[i] = e < len ? dense[s + e] : 0u;
            }
            probe(q, len, base, x, hit_any);
        }
        epilogue(q, cls[q], hit_any);
    };

    // pair iterations: issue B -> probe A -> issue next A -> probe B -> rotate meta
    uint32_t ndefer = 0;  // columns longer than the register window (probed after the loop)
    auto probe_batch = [&](const BatchX<B, C>& cur, uint32_t t0, uint32_t j0) {
#pragma unroll
        for (uint32_t j = 0; j < B; ++j) {
            const uint32_t t = t0 + j;
            if (t >= ncol) break;
            const uint64_t s = readlane64(mcur.beg, j0 + j);
            const uint32_t len = (uint32_t)(readlane64(mcur.end, j0 + j) - s);
            if (len == 0) continue;
            const uint32_t q = qw + kPairWaves * t;
            if (len > 64 * C) {
                if (ndefer < kDefer && lane == 0) defer[wave][ndefer] = q;
                ++ndefer;
                continue;
            }
            column_short(q, len, __builtin_amdgcn_readlane(mcur.cls, j0 + j), cur.x[j]);
        }
    };
    for (uint32_t t0 = 0; t0 < ncol; t0 += 2 * B) {
        batch_issue(xb, dense, mcur, B, lane);        // batch t0+B
        probe_batch(xa, t0, 0);                       // batch t0
        batch_issue(xa, dense, mnext, 0, lane);       // batch t0+2B
        probe_batch(xb, t0 + B, B);                   // batch t0+B
        mcur = mnext;
        meta_load(mnext, dense_off, cls, qw, t0 + 4 * B, ncol, lane);
    }
    // deferred long columns (their k-mers are loaded here, in order)
    for (uint32_t d = 0; d < min(ndefer, kDefer); ++d) column_long(defer[wave][d]);
    if (ndefer > kDefer) {
        // list overflowed: walk the wave's columns again and probe every long one beyond it
        uint32_t seen = 0;
        for (uint32_t t = 0; t < ncol; ++t) {
            const uint32_t q = qw + kPairWaves * t;
            const uint32_t len = (uint32_t)(dense_off[q + 1] - dense_off[q]);
            if (len > 64 * C && seen++ >= kDefer) column_long(q);
        }
    }
    flush();
}

// ------------------------------------------------------------------------------------
// Long proteins: a repeat-filtered set longer than the tile capacity never enters a row tile
// or a column stream (its planned length is 0).  Its pairs are counted here instead: one
// workgroup per (long protein p, chunk of column proteins), one wave per column q at a time;
// each lane binary-searches q's k-mers in K(p) (sorted, L2-resident) and the wave reduces the
// hits.  Pairs of two long proteins are counted once, from the smaller index.
constexpr uint32_t kLongPairThreads = 256;
constexpr uint32_t kLongCols = 2048;  // column proteins per workgroup

__global__ __launch_bounds__(kLongPairThreads) void pair_long_kernel(
    const uint32_t* __restrict__ rep, const uint32_t* __restrict__ rep_len, const uint64_t* __restrict__ res_off,
    const uint16_t* __restrict__ cls, const uint32_t* __restrict__ long_ids, uint32_t tile_cap, uint32_t n,
    uint32_t min_shared, int require_diff, uint32_t* __restrict__ out_p, uint32_t* __restrict__ out_q,
    uint32_t* __restrict__ out_w, uint64_t cap, unsigned long long* __restrict__ count) {
    const uint32_t p = long_ids[blockIdx.y];
    const uint32_t lp = rep_len[p];
    const uint32_t* A = rep + set_base(res_off[p], p);
    const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
    const uint32_t q0 = blockIdx.x * kLongCols, q1 = min(n, q0 + kLongCols);
    const uint16_t cp = cls[p];
    for (uint32_t q = q0 + wave; q < q1; q += kLongPairThreads / 64) {
        const uint32_t lq = rep_len[q];
        if (q == p || lq == 0 || (lq > tile_cap && q < p)) continue;
        const uint32_t* B = rep + set_base(res_off[q], q);
        uint32_t hits = 0;
        for (uint32_t e = lane; e < lq; e += 64) {
            const uint32_t x = B[e];
            uint32_t lo = 0, hi = lp;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (A[mid] < x) lo = mid + 1; else hi = mid;
            }
            hits += (lo < lp && A[lo] == x);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) hits += __shfl_xor(hits, o);
        const bool ok = hits >= min_shared && (!require_diff || cls[q] != cp);
        if (ok && lane == 0) {
            const unsigned long long pos = atomicAdd(count, 1ull);
            if (pos < cap) {
                out_p[pos] = min(p, q);
                out_q[pos] = max(p, q);
                out_w[pos] = hits;
            }
        }
    }
}

// ------------------------------------------------------------------------------------
__global__ void pack_edges_kernel(const uint32_t* __restrict__ p, const uint32_t* __restrict__ q, uint64_t n,
                                  uint64_t np, unsigned long long* __restrict__ key) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        key[i] = (unsigned long long)p[i] * np + q[i];
}
__global__ void unpack_edges_kernel(const unsigned long long* __restrict__ key, uint64_t n, uint64_t np,
                                    uint32_t* __restrict__ p, uint32_t* __restrict__ q) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        p[i] = (uint32_t)(key[i] / np);
        q[i] = (uint32_t)(key[i] % np);
    }
}

int hip_status(hipError_t e) { return e == hipSuccess ? KMP_OK : KMP_EDEVICE; }

unsigned bits_for(uint64_t v) {  // bits needed to represent values < v
    unsigned b = 0;
    while (b < 64 && (v - 1) >> b) ++b;
    return b ? b : 1;
}

inline uint64_t align_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

struct SortLayout {
    uint64_t keys_in, keys_out, vals_out, prim, prim_bytes, total;
};

SortLayout sort_layout(uint64_t n, uint32_t np) {
    SortLayout l{};
    size_t prim = 0;
    const unsigned end_bit = bits_for((uint64_t)np * np);
    (void)rocprim::radix_sort_pairs(nullptr, prim, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                    (uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)n, 0u, end_bit);
    l.keys_in = 0;
    l.keys_out = align_up(l.keys_in + 8 * n, 256);
    l.vals_out = align_up(l.keys_out + 8 * n, 256);
    l.prim = align_up(l.vals_out + 4 * n, 256);
    l.prim_bytes = prim;
    l.total = l.prim + prim + 256;
    return l;
}

}  // namespace

// ====================================================================================
extern "C" {

uint64_t kmp_set_capacity(uint32_t n, uint64_t total_residues) { return total_residues + 4ull * n + 8ull; }
uint64_t kmp_set_base(uint64_t res_off, uint32_t p) { return set_base(res_off, p); }

int kmp_dev_extract(const uint8_t* d_res, const uint64_t* d_res_off, uint32_t n, int k, uint32_t* d_codes,
                    void* stream) {
    if (k < 1 || k > kMaxK || (n && (!d_res_off || !d_codes))) return KMP_EINVAL;
    if (n == 0) return KMP_OK;
    extract_kernel<<<n, kExtractThreads, 0, as_stream(stream)>>>(d_res, d_res_off, k, d_codes);
    return hip_status(hipGetLastError());
}

int kmp_dev_build_sets(const uint8_t* d_res, const uint64_t* d_res_off, uint32_t n, int k, uint32_t max_len,
                       uint32_t* d_set, uint32_t* d_set_len, uint32_t* d_scratch, void* stream) {
    if (k < 1 || k > kMaxK || (n && (!d_res_off || !d_set || !d_set_len))) return KMP_EINVAL;
    if (n == 0) return KMP_OK;
    hipStream_t st = as_stream(stream);
    build_sets_kernel<<<n, kSetThreads, 0, st>>>(d_res, d_res_off, k, d_set, d_set_len);
    const bool maybe_long = max_len == 0 || n_windows(max_len, k) > KMP_LDS_SORT_MAX;
    if (maybe_long) {
        if (!d_scratch) return KMP_EINVAL;
        build_sets_long_kernel<<<n, kLongThreads, 0, st>>>(d_res, d_res_off, k, d_set, d_set_len, d_scratch);
    }
    return hip_status(hipGetLastError());
}

uint64_t kmp_dev_repeat_bitmap_words(int k) {
    if (k < 1 || k > kMaxK) return 0;
    return (pow21(k) + 31) / 32;
}

int kmp_dev_filter_repeats(const uint32_t* d_set, const uint32_t* d_set_len, const uint64_t* d_res_off,
                           uint32_t n, int k, uint32_t* d_bits, uint32_t* d_rep, uint32_t* d_rep_len,
                           void* stream) {
    if (k < 1 || k > kMaxK || (n && (!d_set || !d_set_len || !d_res_off || !d_bits || !d_rep || !d_rep_len)))
        return KMP_EINVAL;
    if (n == 0) return KMP_OK;
    hipStream_t st = as_stream(stream);
    const uint64_t words = kmp_dev_repeat_bitmap_words(k);
    hipError_t e = hipMemsetAsync(d_bits, 0, 2 * words * sizeof(uint32_t), st);
    if (e != hipSuccess) return KMP_EDEVICE;
    mark_kernel<<<n, kFilterThreads, 0, st>>>(d_set, d_set_len, d_res_off, d_bits, d_bits + words);
    compact_repeats_kernel<<<n, kFilterThreads, 0, st>>>(d_set, d_set_len, d_res_off, d_bits + words, d_rep,
                                                         d_rep_len);
    return hip_status(hipGetLastError());
}

void kmp_pair_geometry_get(kmp_pair_geometry* g) {
    if (!g) return;
    g->tile_slots = kTileSlots;
    g->tile_cap = kTileCap;
    g->rows_max = kRowsMax;
    g->threads = kPairThreads;
}

int kmp_plan_pairs(const uint32_t* set_len, uint32_t n, uint64_t chunk_cost, uint64_t* dense_off,
                   kmp_work_item* items, uint64_t cap, uint64_t* n_items) {
    if (!n_items || !dense_off || (n && !set_len) || (cap && !items)) return KMP_EINVAL;
    if (chunk_cost == 0) chunk_cost = kChunkCost;
    dense_off[0] = 0;
    for (uint32_t p = 0; p < n; ++p) {
        if (set_len[p] > kTileCap) return KMP_EINVAL;
        dense_off[p + 1] = dense_off[p] + set_len[p];
    }
    // row tiles: greedy in index order; tiles whose sets are all empty make no items
    std::vector<uint32_t> tb, te;
    for (uint32_t r0 = 0; r0 < n;) {
        uint32_t r1 = r0;
        uint64_t tot = 0;
        while (r1 < n && r1 - r0 < kRowsMax && tot + set_len[r1] <= kTileCap) tot += set_len[r1++];
        if (tot > 0 && r0 + 1 < n) {
            tb.push_back(r0);
            te.push_back(r1);
        }
        r0 = r1;
    }
    // column chunks (cost counts one per protein so empty runs still split); chunk-major items
    uint64_t m = 0;
    for (uint32_t c0 = 0; c0 < n;) {
        uint32_t c1 = c0;
        uint64_t cost = 0;
        while (c1 < n && (cost < chunk_cost || c1 == c0)) cost += set_len[c1++] + 1;
        for (size_t t = 0; t < tb.size() && tb[t] + 1 < c1; ++t) {
            if (m < cap) items[m] = kmp_work_item{tb[t], te[t], c0, c1};
            ++m;
        }
        c0 = c1;
    }
    *n_items = m;
    return m > cap ? KMP_EOVERFLOW : KMP_OK;
}

int kmp_order_items_xcd(const kmp_work_item* in, uint64_t n, kmp_work_item* out, uint64_t cap, uint64_t* n_out) {
    if (!n_out || (n && !in) || (cap && !out)) return KMP_EINVAL;
    constexpr uint32_t kXcds = 8;
    // consecutive items of one chunk share col_beg; chunk g -> XCD list g % 8
    std::vector<std::vector<kmp_work_item>> lists(kXcds);
    uint64_t g = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (i > 0 && in[i].col_beg != in[i - 1].col_beg) ++g;
        lists[g % kXcds].push_back(in[i]);
    }
    size_t longest = 0;
    for (auto& l : lists) longest = std::max(longest, l.size());
    // slot 8*s + x <- lists[x][s]; a short list is padded with empty items (no-ops)
    const uint64_t m = (uint64_t)longest * kXcds;
    *n_out = m;
    if (m > cap) return KMP_EOVERFLOW;
    for (size_t s = 0; s < longest; ++s)
        for (uint32_t x = 0; x < kXcds; ++x)
            out[s * kXcds + x] = s < lists[x].size() ? lists[x][s] : kmp_work_item{0, 0, 0, 0};
    return KMP_OK;
}

uint32_t kmp_pair_col_window(const uint32_t* set_len, uint32_t n) {
    if (!set_len || n == 0) return 0;
    // smallest window class that holds >= 97 % of the non-empty columns (the rest are deferred)
    const uint32_t classes[3] = {192, 384, 768};
    uint64_t nonempty = 0, fit[3] = {0, 0, 0};
    for (uint32_t p = 0; p < n; ++p) {
        if (set_len[p] == 0) continue;
        ++nonempty;
        for (int c = 0; c < 3; ++c) fit[c] += set_len[p] <= classes[c];
    }
    for (int c = 0; c < 3; ++c)
        if (fit[c] * 100 >= nonempty * 97) return classes[c];
    return classes[2];
}

int kmp_dev_pack_dense(const uint32_t* d_rep, const uint64_t* d_res_off, const uint64_t* d_dense_off, uint32_t n,
                       uint32_t* d_dense, void* stream) {
    if (n == 0) return KMP_OK;
    if (!d_rep || !d_res_off || !d_dense_off || !d_dense) return KMP_EINVAL;
    pack_dense_kernel<<<n, 256, 0, as_stream(stream)>>>(d_rep, d_res_off, d_dense_off, d_dense);
    return hip_status(hipGetLastError());
}

int kmp_dev_pairs(const uint32_t* d_dense, const uint64_t* d_dense_off, const uint16_t* d_class, uint32_t n,
                  const kmp_work_item* d_items, uint64_t n_items, uint32_t col_window, uint32_t min_shared,
                  int require_class_diff, uint32_t* d_p, uint32_t* d_q, uint32_t* d_w, uint64_t cap,
                  unsigned long long* d_count, void* stream) {
    (void)n;
    if (n_items == 0) return KMP_OK;
    if (!d_dense || !d_dense_off || !d_class || !d_items || !d_count || (cap && (!d_p || !d_q || !d_w)))
        return KMP_EINVAL;
    if (n_items > 0x7FFFFFFFull) return KMP_EINVAL;
    if (min_shared < 1) min_shared = 1;
    const dim3 grid((uint32_t)n_items), block(kPairThreads);
    hipStream_t st = as_stream(stream);
#define KMP_PAIR_LAUNCH(CC, BB)                                                                             \
    pair_kernel<CC, BB><<<grid, block, 0, st>>>(d_dense, d_dense_off, d_class, d_items, min_shared,          \
                                                require_class_diff, d_p, d_q, d_w, cap, d_count)
    // register window: 64*C k-mers per column, B columns per batch (2*B*C VGPRs in flight)
    const uint32_t w = col_window <= 192 ? 3u : col_window <= 384 ? 6u : 12u;
    if (w == 3) KMP_PAIR_LAUNCH(3, 8);
    else if (w == 6) KMP_PAIR_LAUNCH(6, 3);
    else KMP_PAIR_LAUNCH(12, 1);
#undef KMP_PAIR_LAUNCH
    return hip_status(hipGetLastError());
}

int kmp_dev_pairs_long(const uint32_t* d_rep, const uint32_t* d_rep_len, const uint64_t* d_res_off,
                       const uint16_t* d_class, uint32_t n, const uint32_t* d_long_ids, uint32_t n_long,
                       uint32_t min_shared, int require_class_diff, uint32_t* d_p, uint32_t* d_q, uint32_t* d_w,
                       uint64_t cap, unsigned long long* d_count, void* stream) {
    if (n_long == 0 || n == 0) return KMP_OK;
    if (!d_rep || !d_rep_len || !d_res_off || !d_class || !d_long_ids || !d_count || (cap && (!d_p || !d_q || !d_w)))
        return KMP_EINVAL;
    if (n_long > 65535) return KMP_EINVAL;
    if (min_shared < 1) min_shared = 1;
    const dim3 grid((n + kLongCols - 1) / kLongCols, n_long);
    pair_long_kernel<<<grid, kLongPairThreads, 0, as_stream(stream)>>>(d_rep, d_rep_len, d_res_off, d_class, d_long_ids,
                                                                      kTileCap, n, min_shared, require_class_diff,
                                                                      d_p, d_q, d_w, cap, d_count);
    return hip_status(hipGetLastError());
}

uint64_t kmp_dev_sort_edges_tmp_bytes(uint64_t n, uint32_t n_proteins) {
    return sort_layout(n, n_proteins ? n_proteins : 1).total;
}

int kmp_dev_sort_edges(uint32_t* d_p, uint32_t* d_q, uint32_t* d_w, uint64_t n, uint32_t n_proteins, void* d_tmp,
                       uint64_t tmp_bytes, void* stream) {
    if (n == 0) return KMP_OK;
    if (!d_p || !d_q || !d_w || !d_tmp || n_proteins == 0) return KMP_EINVAL;
    const SortLayout l = sort_layout(n, n_proteins);
    if (tmp_bytes < l.total) return KMP_EINVAL;
    hipStream_t st = as_stream(stream);
    char* base = (char*)align_up((uint64_t)(uintptr_t)d_tmp, 256) ;
    if ((uint64_t)(base - (char*)d_tmp) + l.total - 256 > tmp_bytes) return KMP_EINVAL;
    auto* kin = reinterpret_cast<unsigned long long*>(base + l.keys_in);
    auto* kout = reinterpret_cast<unsigned long long*>(base + l.keys_out);
    auto* vout = reinterpret_cast<uint32_t*>(base + l.vals_out);
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((n + 255) / 256, 8192);
    pack_edges_kernel<<<blocks, 256, 0, st>>>(d_p, d_q, n, n_proteins, kin);
    size_t prim = l.prim_bytes;
    const unsigned end_bit = bits_for((uint64_t)n_proteins * n_proteins);
    hipError_t e = rocprim::radix_sort_pairs(base + l.prim, prim, kin, kout, d_w, vout, (size_t)n, 0u, end_bit, st);
    if (e != hipSuccess) return KMP_EDEVICE;
    unpack_edges_kernel<<<blocks, 256, 0, st>>>(kout, n, n_proteins, d_p, d_q);
    e = hipMemcpyAsync(d_w, vout, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) return KMP_EDEVICE;
    return hip_status(hipGetLastError());
}

}  // extern "C"
