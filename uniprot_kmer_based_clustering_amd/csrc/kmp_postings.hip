// kmp_postings.hip — the postings engine: the reference's own pair algorithm restated for the
// GPU as sort / expand / reduce.
//
//   reference (file:line)                                  here
//   Protein::new windows + codes (protein.rs:82-94)        residue_keys_chunk_kernel: one key per window
//   per-protein sort + dedup (main.rs:99-101,187-189)             duplicates of (k-mer, p) end up adjacent
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

#include <rocprim/block/block_radix_sort.hpp>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_reduce_by_key.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>
#include <rocprim/iterator/transform_iterator.hpp>
#include <rocprim/device/device_run_length_encode.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <chrono>
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

// compute units of the current device (persistent grids), looked up once per device and thread
uint32_t device_cus() {
    static thread_local int dev = -1;
    static thread_local uint32_t cus = 256;
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess) return cus;
    if (d != dev) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess && v > 0)
            cus = (uint32_t)v;
        dev = d;
    }
    return cus;
}


// rocprim 4.2 (ROCm 7.2): with the default config, radix_sort_keys on fewer than 1M keys takes a
// merge-sort path that returns unsorted, non-permuted data for bit ranges [b, 64) with b > 0
// (tools/sort_check.hip reproduces it).  Onesweep (merge-sort limit 0) is correct for every range
// and size, so every sort here uses it.
using SortCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                           rocprim::default_config, 0>;
// Pair keys (p * N + q, 34 bits at N = 100k): 9-bit digits in 1024 x 8 workgroups take 4 onesweep
// passes instead of 5 (tools/radix_bits_bench.hip: 0.209 vs 0.269 ms for 5.4 M keys); 10-bit
// digits are slower and 11 bits exceed the LDS.  Merge-sort limit 0, as for SortCfg.
using PairSortCfg = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<512, 12>, rocprim::kernel_config<1024, 8>, 9,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;
constexpr unsigned kClsBits = 16;

// Two key layouts (u64, kNoKey = all ones is the padding of every layout):
//   flat     [ code | class (16 bits, when it fits) | p ]       sorted on the code bits (stable)
//   bucketed [ 0 | h(code) (32) | p | class (cb bits) ]         h(code) = code * A mod 2^32 is a
//            bijection, so h identifies the k-mer; bucket = top bbits of h (equal k-mers share a
//            bucket); keys are sorted on bits [bucket .. 64): the zero top bit makes the padding
//            sort last.  cb = 31 - pbits (16 at most); a class id that does not fit sends the
//            call to the flat layout.
struct Layout {
    unsigned pbits;    // protein index bits
    unsigned cbits;    // code bits
    unsigned shift;    // flat: code starts here
    bool cls_in_key;   // flat: class bits between code and p
    bool bucketed;
    unsigned bbits;    // bucketed: bucket index bits
    unsigned clsbits;  // bucketed: class bits (bits [0, clsbits))
    unsigned hshift;   // bucketed: h(code) starts here (= pbits + clsbits)
    unsigned sort_lo, sort_hi;  // radix-sorted bit range
    uint32_t mean_keys;         // bucketed: expected keys per bucket (windows / buckets)
};

#ifndef KMP_BUCKET_TARGET
#define KMP_BUCKET_TARGET 1024
#endif
constexpr uint32_t kBucketTarget = KMP_BUCKET_TARGET;  // mean keys per bucket
constexpr uint32_t kHashA = 0x9E3779B1u;  // odd: code -> h(code) is a bijection of u32

Layout make_layout(uint32_t n, int k, uint64_t slots, bool bucketed) {
    Layout l{};
    l.pbits = bits_for(n);
    l.cbits = bits_for(pow21(k));
    if (bucketed && l.pbits <= 30) {
        unsigned bb = 1;
        while (bb < 20 && (slots >> bb) > kBucketTarget) ++bb;  // bb + sub bits <= 32
        l.bucketed = true;
        l.bbits = bb;
        l.clsbits = std::min(16u, 31u - l.pbits);
        l.hshift = l.pbits + l.clsbits;
        l.sort_lo = l.hshift + 32 - bb;
        l.sort_hi = 64;
        // a protein's slot region (L + 4 slots and more) holds L - k + 1 windows: k + 3 slots at
        // least hold none, so this is an upper bound of the mean
        const uint64_t spare = (uint64_t)(k + 3) * n;
        l.mean_keys = (uint32_t)((slots > spare ? slots - spare : 0ull) >> bb);
        return l;
    }
    l.cls_in_key = l.pbits + kClsBits + l.cbits <= 64;
    l.shift = l.pbits + (l.cls_in_key ? kClsBits : 0);
    l.sort_lo = l.shift;
    l.sort_hi = l.shift + l.cbits;
    return l;
}

__device__ __forceinline__ unsigned long long make_key(uint32_t code, uint16_t c, uint32_t p, const Layout& l) {
    if (l.bucketed)
        return ((unsigned long long)(code * kHashA) << l.hshift) | ((unsigned long long)p << l.clsbits) |
               (c & ((1u << l.clsbits) - 1));
    unsigned long long x = ((unsigned long long)code << l.shift) | p;
    if (l.cls_in_key) x |= (unsigned long long)c << l.pbits;
    return x;
}

// class ids wider than the bucketed layout's class field -> flat layout
__device__ __forceinline__ void check_class(uint16_t c, const Layout& l, uint32_t* flags) {
    if (l.bucketed && l.clsbits < 16 && (c >> l.clsbits)) flags[1] = 1;
}

// keys of the unfiltered K(p) slots: K(p)[t] for t < |K(p)|, kNoKey for the rest of the region;
// block n fills the tail of the buffer past the last region (no memset needed)
__global__ __launch_bounds__(256) void set_keys_kernel(const uint32_t* __restrict__ set,
                                                       const uint32_t* __restrict__ set_len,
                                                       const uint64_t* __restrict__ res_off,
                                                       const uint16_t* __restrict__ cls, uint32_t n, uint64_t slots,
                                                       Layout lay, unsigned long long* __restrict__ keys,
                                                       uint32_t* __restrict__ flags) {
    const uint32_t p = blockIdx.x;
    if (p == n) {
        for (uint64_t i = set_base(res_off[n], n) + threadIdx.x; i < slots; i += 256) keys[i] = kNoKey;
        return;
    }
    const uint64_t b = set_base(res_off[p], p), e = set_base(res_off[p + 1], p + 1);
    const uint32_t len = set_len[p];
    const uint16_t c = cls[p];
    if (threadIdx.x == 0) check_class(c, lay, flags);
    for (uint64_t i = b + threadIdx.x; i < e; i += 256) {
        const uint64_t o = i - b;
        keys[i] = o < len ? make_key(set[i], c, p, lay) : kNoKey;
    }
}

// one key per window straight from the residues (Protein::new, protein.rs:82-94: window j of
// protein p is residues [j, j+k), radix-21, first residue most significant), same slot layout.
// Workgroup g owns slots [slot_begin + g*kKeyChunk, ... + kKeyChunk) of proteins
// [p_lo, p_hi) (about 13 proteins per chunk at L ~ 300).  It finds them by binary search on
// set_base, recodes just the residue span its windows need into LDS (byte -> code), and writes the
// chunk's keys coalesced; slots past a protein's windows (and past the last region) get kNoKey.
// keys[i - slot_begin] for slot i.
constexpr int kKeyThreads = 256;
constexpr uint32_t kKeyChunk = 4096;
constexpr uint32_t kKeyProtMax = kKeyChunk / 4 + 2;                // a region spans >= 4 slots
// residues a chunk can need: a protein's region is longer than its residue count, so the span is
// at most the chunk plus the last window's k - 1 residues
constexpr uint32_t kKeyResMax = kKeyChunk + 64;

// first[c] = the protein whose region holds the chunk's first slot (p_hi: the tail past the last
// region); one thread per protein writes the chunk starts that fall in its region
__global__ void chunk_first_kernel(const uint64_t* __restrict__ res_off, uint32_t p_lo, uint32_t p_hi,
                                   uint64_t slot_begin, uint64_t slot_end, uint32_t n_chunks,
                                   uint32_t* __restrict__ first) {
    const uint32_t p = p_lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (p > p_hi) return;
    const uint64_t b = set_base(res_off[p], p) - slot_begin;
    const uint64_t e = (p < p_hi ? set_base(res_off[p + 1], p + 1) : slot_end) - slot_begin;
    for (uint64_t c = (b + kKeyChunk - 1) / kKeyChunk; c * kKeyChunk < e && c < n_chunks; ++c) first[c] = p;
}

// chunk_first_kernel (proteins [0, p_hi]) fused with the clear of the cursor level 2's bucket
// counts (one launch less per step)
__global__ void chunk_first_clear_kernel(const uint64_t* __restrict__ res_off, uint32_t p_hi, uint64_t slot_end,
                                         uint32_t n_chunks, uint32_t* __restrict__ first,
                                         uint32_t* __restrict__ cur, uint32_t ncur) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    for (uint32_t i = t; i < ncur; i += gridDim.x * blockDim.x) cur[i] = 0;
    const uint32_t p = t;
    if (p > p_hi) return;
    const uint64_t b = set_base(res_off[p], p);
    const uint64_t e = p < p_hi ? set_base(res_off[p + 1], p + 1) : slot_end;
    for (uint64_t c = (b + kKeyChunk - 1) / kKeyChunk; c * kKeyChunk < e && c < n_chunks; ++c) first[c] = p;
}

// LDS state of one key chunk: residue codes of the chunk's span and its proteins' geometry
struct KeyChunk {
    uint8_t lut[256];
    __attribute__((aligned(16))) uint8_t rc[kKeyResMax + 32];  // residue codes from a0 = r0 & ~15
    uint32_t pb[kKeyProtMax + 1];   // region start of each protein, relative to c0 (may wrap)
    int32_t pr[kKeyProtMax];        // LDS index of the protein's residue 0 (may be < 0)
    uint32_t pw[kKeyProtMax];       // window count
    uint16_t pc[kKeyProtMax];       // class
    uint32_t np;
    uint64_t r0, r1;
};

// Stage chunk [c0, c1) of proteins [first, p_hi): the proteins whose regions overlap it and the
// residue span their windows need, recoded into LDS.  Ends with a barrier.
template <uint32_t kThr = kKeyThreads>
__device__ __forceinline__ void key_chunk_load(KeyChunk& s, const uint8_t* __restrict__ res,
                                               const uint64_t* __restrict__ res_off,
                                               const uint16_t* __restrict__ cls, int k, uint32_t p_hi,
                                               uint64_t c0, uint64_t c1, uint32_t first, const Layout& lay,
                                               uint32_t* __restrict__ flags) {
    const int tid = threadIdx.x;
    if (tid < 256) s.lut[tid] = c_lut.v[tid];
    if (tid == 0) {
        s.np = 0;
        s.r0 = s.r1 = 0;
    }
    __syncthreads();
    // the chunk's proteins: first + t while its region starts before c1 (one parallel round)
    for (uint32_t t = tid; t < kKeyProtMax && first + t < p_hi; t += kThr) {
        const uint32_t p = first + t;
        const uint64_t off = res_off[p], L = res_off[p + 1] - off;
        const uint64_t b = set_base(off, p);
        if (b >= c1) break;
        const uint32_t nw = L >= (uint64_t)k ? (uint32_t)(L - k + 1) : 0u;
        s.pb[t] = (uint32_t)(b - c0);  // wraps for the first protein when it starts before c0
        s.pw[t] = nw;
        s.pc[t] = cls[p];
        check_class(s.pc[t], lay, flags);
        atomicMax(&s.np, t + 1);
        const uint64_t j0 = c0 > b ? c0 - b : 0;
        const uint64_t j1 = min<uint64_t>(nw, c1 - b);
        if (t == 0) s.r0 = off + min<uint64_t>(j0, L);
        if (j1 > j0) atomicMax((unsigned long long*)&s.r1, (unsigned long long)(off + j1 + k - 1));
    }
    __syncthreads();
    const uint32_t np = s.np;
    const uint64_t r0 = s.r0, r1 = max(s.r0, s.r1);
    // stage the span with independent 16-byte loads (byte loads where a vector would pass the end
    // of the range's residues or the base is unaligned), recoded through the LUT, one 16-byte LDS
    // store per vector
    const uint64_t a0 = r0 & ~15ull, res_end = res_off[p_hi];
    const bool vec_ok = ((uintptr_t)res & 15u) == 0;
    const uint32_t nv = (uint32_t)((r1 - a0 + 15) >> 4);
    for (uint32_t v = tid; v < nv; v += kThr) {
        const uint64_t g = a0 + 16ull * v;
        uint32_t w[4];
        if (vec_ok && g + 16 <= res_end) {
            const uint4 q = *reinterpret_cast<const uint4*>(res + g);
            w[0] = q.x, w[1] = q.y, w[2] = q.z, w[3] = q.w;
        } else {
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                w[d] = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const uint64_t i = g + 4 * d + b;
                    w[d] |= (uint32_t)(i < res_end ? res[i] : 0) << (8 * b);
                }
            }
        }
        auto code4 = [&](uint32_t x) {
            return (uint32_t)s.lut[x & 255u] | (uint32_t)s.lut[(x >> 8) & 255u] << 8 |
                   (uint32_t)s.lut[(x >> 16) & 255u] << 16 | (uint32_t)s.lut[x >> 24] << 24;
        };
        *reinterpret_cast<uint4*>(s.rc + 16 * v) =
            make_uint4(code4(w[0]), code4(w[1]), code4(w[2]), code4(w[3]));
    }
    for (uint32_t t = tid; t < np; t += kThr) s.pr[t] = (int32_t)((int64_t)res_off[first + t] - (int64_t)a0);
    __syncthreads();
}

// key of chunk slot c0 + i (kNoKey past a protein's windows)
__device__ __forceinline__ unsigned long long key_chunk_key(const KeyChunk& s, uint32_t i, int k, uint32_t first,
                                                            const Layout& lay) {
    const uint32_t np = s.np;
    if (!np) return kNoKey;
    // protein of slot c0 + i: last t with region start <= c0 + i (t = 0 may start before c0)
    uint32_t a = 0, b = np;
    while (a + 1 < b) {
        const uint32_t mid = (a + b) >> 1;
        if (s.pb[mid] <= i) a = mid;
        else b = mid;
    }
    const uint32_t j = i - s.pb[a];  // window index (pb[0] wraps: i - pb[0] = c0 + i - b0)
    if (j >= s.pw[a]) return kNoKey;
    const uint8_t* w = s.rc + (s.pr[a] + (int32_t)j);
    uint32_t v = 0;
    for (int t = 0; t < k; ++t) v = v * kRadix + w[t];
    return make_key(v, s.pc[a], first + a, lay);
}

// The kPer consecutive chunk slots i0 .. i0 + kPer - 1: one binary search, then the protein's
// state in registers (reloaded at a region start: regions are >= 4 slots, so at most one per
// slot) and the radix-21 code rolled window to window (two LDS reads instead of k).
// emit(e, valid, h, lo) per slot: h = h(code), lo = the key's p | class bits; the key is
// (u64)h << hshift | lo.  pw21 = 21^(k-1).
template <uint32_t kPer, class Emit>
__device__ __forceinline__ void key_chunk_run(const KeyChunk& s, uint32_t i0, uint32_t n_slots, int k, uint32_t pw21,
                                              uint32_t first, const Layout& lay, Emit emit) {
    const uint32_t np = s.np;
    if (!np) {
#pragma unroll
        for (uint32_t e = 0; e < kPer; ++e) emit(e, false, 0u, 0ull);
        return;
    }
    uint32_t a = 0, b = np;
    while (a + 1 < b) {
        const uint32_t mid = (a + b) >> 1;
        if (s.pb[mid] <= i0) a = mid;
        else b = mid;
    }
    const uint32_t cmask = (1u << lay.clsbits) - 1;
    uint32_t nxt = a + 1 < np ? s.pb[a + 1] : 0xFFFFFFFFu;  // first slot of protein a + 1
    uint32_t j = i0 - s.pb[a];                              // window index (pb[0] may wrap)
    uint32_t nw = s.pw[a];
    int32_t r = s.pr[a] + (int32_t)j;                       // LDS index of window j's first residue
    unsigned long long lo = ((unsigned long long)(first + a) << lay.clsbits) | (s.pc[a] & cmask);
    uint32_t v = 0;
    bool have = false;  // v holds the code of window j - 1
#pragma unroll
    for (uint32_t e = 0; e < kPer; ++e) {
        const uint32_t i = i0 + e;
        if (i == nxt) {
            ++a;
            nxt = a + 1 < np ? s.pb[a + 1] : 0xFFFFFFFFu;
            j = 0;
            nw = s.pw[a];
            r = s.pr[a];
            lo = ((unsigned long long)(first + a) << lay.clsbits) | (s.pc[a] & cmask);
            have = false;
        }
        const bool valid = j < nw && i < n_slots;
        if (valid) {
            if (have) {
                v = (v - s.rc[r - 1] * pw21) * kRadix + s.rc[r + k - 1];
            } else {
                v = 0;
                for (int t = 0; t < k; ++t) v = v * kRadix + s.rc[r + t];
            }
        }
        have = valid;
        emit(e, valid, v * kHashA, lo);
        ++j;
        ++r;
    }
}

__global__ __launch_bounds__(kKeyThreads) void residue_keys_chunk_kernel(
    const uint8_t* __restrict__ res, const uint64_t* __restrict__ res_off, const uint16_t* __restrict__ cls,
    int k, uint32_t p_hi, uint64_t slot_begin, uint64_t slot_end, const uint32_t* __restrict__ chunk_first,
    Layout lay, unsigned long long* __restrict__ keys, uint32_t* __restrict__ flags) {
    __shared__ KeyChunk s;
    const uint64_t c0 = slot_begin + (uint64_t)blockIdx.x * kKeyChunk;
    const uint64_t c1 = min(c0 + kKeyChunk, slot_end);
    const uint32_t first = chunk_first[blockIdx.x];
    key_chunk_load(s, res, res_off, cls, k, p_hi, c0, c1, first, lay, flags);
    for (uint32_t i = threadIdx.x; i < (uint32_t)(c1 - c0); i += kKeyThreads)
        keys[c0 + i - slot_begin] = key_chunk_key(s, i, k, first, lay);
}

enum : int { kStSumS, kStDistinct, kStRepeat, kStCdf2, kStMaxDf, kStHeavy, kStInc, kStN };

constexpr int kExpThreads = 256;
constexpr int kExpRounds = 8;
constexpr uint64_t kExpChunk = (uint64_t)kExpThreads * kExpRounds;  // keys per workgroup

__device__ __forceinline__ unsigned long long stat_op(int t, unsigned long long a, unsigned long long b) {
    return t == kStMaxDf ? (a > b ? a : b) : a + b;
}

// Wave64 inclusive scans on DPP (VALU only, no LDS crossbar round trips): row_shr 1/2/4/8 scan
// each 16-lane row (bound_ctrl: a source before the row start reads 0), then row_bcast 15 / 31
// carry the row totals into the later rows (rows outside the row mask keep the old value, 0).
// Every lane of the wave must be active.
template <int kCtrl, int kRowMask = 0xF>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kCtrl, kRowMask, 0xF, true);
}
__device__ __forceinline__ uint32_t wave_iscan(uint32_t x) {
    x += dpp_mov<0x111>(x);
    x += dpp_mov<0x112>(x);
    x += dpp_mov<0x114>(x);
    x += dpp_mov<0x118>(x);
    x += dpp_mov<0x142, 0xA>(x);
    x += dpp_mov<0x143, 0xC>(x);
    return x;
}
// the wave's maximum (every lane; values are unsigned, so the 0 of an invalid source is neutral)
__device__ __forceinline__ uint32_t wave_max(uint32_t x) {
    x = max(x, dpp_mov<0x111>(x));
    x = max(x, dpp_mov<0x112>(x));
    x = max(x, dpp_mov<0x114>(x));
    x = max(x, dpp_mov<0x118>(x));
    x = max(x, dpp_mov<0x142, 0xA>(x));
    x = max(x, dpp_mov<0x143, 0xC>(x));
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_iscan(x), 63);
}

// exclusive scan of one value per thread over the workgroup; returns (prefix, total)
__device__ __forceinline__ void block_scan(uint32_t v, uint32_t& excl, uint32_t& total, uint32_t* wave_tot) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t x = wave_iscan(v);
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

// ---------------------------------------------------------------- bucketed layout ----------
// Bucket b occupies [bstart[b], bstart[b+1]) of the keys sorted on bits [sort_lo, 64); the
// padding starts at bstart[nb].
__global__ void bucket_bounds_kernel(const unsigned long long* __restrict__ k, uint64_t slots, unsigned sort_lo,
                                     uint32_t nb, uint32_t* __restrict__ bstart) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b > nb) return;
    uint64_t lo = 0, hi = slots;  // first key whose field >= b
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if ((k[mid] >> sort_lo) < b) lo = mid + 1;
        else hi = mid;
    }
    bstart[b] = (uint32_t)lo;
}

constexpr uint32_t kHeavySub = 128;  // larger sub-buckets (very frequent k-mers) -> flat layout

// ---- BLOSUM score carried in the pair key (a build extension) ----
// A scored call writes every (k-mer, pair) incidence as (pair << sb) | sor | s(x): s(x) = Σ_i
// B62[x_i][x_i] over the k residues of the shared k-mer x (the BLOSUM62 diagonal of blosum.rs:8-30
// in residue-code order, code 20 scored 0; at most 7 x 11 = 77, kScoreBits bits) and sor the call's
// k-index bit (kmp_pairs_multi_k's fused union: bit kScoreBits marks the second k).  The row-block
// tail then sums s over each pair's run (score = Σ_{x in K(p) ∩ K(q)} s(x)) and counts the marked
// entries (w of the second k), so no per-edge intersection runs at all.  h(code) = code * kHashA
// is a bijection of u32: the k-mer's code is h * kHashAInv.
constexpr unsigned kScoreBits = 7;
constexpr uint32_t kHashAInv = 0x0E8B2F51u;  // kHashA^-1 mod 2^32
__constant__ uint8_t c_b62_self[21] = {9, 4, 5, 4, 6, 7, 6, 5, 5, 6, 8, 5, 5, 5, 4, 4, 4, 11, 7, 6, 0};
__device__ __forceinline__ uint32_t kmer_self_score(uint32_t h, int k) {
    uint32_t x = h * kHashAInv, sc = 0;
    for (int i = 0; i < k; ++i) {
        const uint32_t q = x / 21u;
        sc += c_b62_self[x - q * 21u];
        x = q;
    }
    return sc;
}
constexpr int kShards = 64;          // output cursors (one per bucket residue mod kShards)
static_assert(kShards == 64, "the heavy tiles hash to a shard with a 6-bit shift");
// device flags of a step (ws->flags): a coarse bin above its level-2 tile budget, a class id too
// wide for the key, the large-bucket list count, row blocks above the LDS capacity, the tile
// budget an overflowing bin needs, a cursor-partition region overflow
enum : uint32_t { kFlBin = 0, kFlClass = 1, kFlList = 2, kFlOvf = 3, kFlBinTiles = 4, kFlCur = 5, kFlSegs = 6, kFlSegMax = 7, kFlN = 8 };

template <int kThreads>
__device__ __forceinline__ void block_scan_n(uint32_t v, uint32_t& excl, uint32_t& total, uint32_t* wave_tot) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t x = wave_iscan(v);
    if (lane == 63) wave_tot[w] = x;
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kThreads / 64; ++i) {
        const uint32_t t = wave_tot[i];
        before += i < w ? t : 0;
        tot += t;
    }
    __syncthreads();
    excl = before + x - v;
    total = tot;
}

// exclusive scan of lh[0, nb) in place (kThreads threads); ends with a barrier
template <int kThreads = kKeyThreads>
__device__ __forceinline__ void lds_bins_scan(uint32_t* lh, uint32_t nb, uint32_t* wave_tot) {
    const uint32_t q = (nb + kThreads - 1) / kThreads, b0 = threadIdx.x * q;
    uint32_t v = 0;
    for (uint32_t t = 0; t < q; ++t)
        if (b0 + t < nb) v += lh[b0 + t];
    uint32_t excl, total;
    block_scan_n<kThreads>(v, excl, total, wave_tot);  // barriers inside
    for (uint32_t t = 0; t < q; ++t)
        if (b0 + t < nb) {
            const uint32_t c = lh[b0 + t];
            lh[b0 + t] = excl;
            excl += c;
        }
    __syncthreads();
}

constexpr uint32_t kSplitMax = 64;  // ranks of the k-mer split
struct SplitRows {
    uint32_t start[kSplitMax + 1];  // row range of rank d: [start[d], start[d+1])
    uint32_t parts;
};

// Arguments of the bucket kernels (one struct, passed by value).
//   out / shard_cap / cursor: kShards pair-key regions; a workgroup reserves its range on
//     cursor[b % kShards] and writes the keys min(p,q) * mul + max(p,q) (writes past shard_cap are
//     dropped, the cursor still counts them: the caller grows the regions and reruns);
//   gstats: kShards x 8 statistics accumulators (kSt* slots);
//   list / list_count: buckets above the small kernel's capacity (the large kernel takes them);
//   spill / spill_cap / spill_cursor: the keys of heavy groups (more than kHeavySub keys: a
//     frequent k-mer) and of buckets above the large capacity, one region of spill_cap keys per
//     shard; the heavy path (heavy_* below) expands them.  spill == nullptr: heavy groups are
//     skipped (an earlier pass of the same keys spilled them already);
//   row_lo / row_hi (kRows): emit only the pairs whose smaller protein lies in [row_lo, row_hi)
//     (a pass or a rank of the row split).
//   capb: 0 -> bucket b is [bstart[b], bstart[b+1]) of sorted; else (cursor partition) bucket b
//     is the region [b * capb, b * capb + bstart[b]) (bstart holds the counts), or, with a learned
//     layout (vreg), [vreg[b], vreg[b] + bstart[b])
struct BucketArgs {
    const unsigned long long* sorted;
    const uint32_t* bstart;
    uint32_t capb;
    const uint32_t* vreg;
    Layout lay;
    uint32_t mul;
    int require_diff;
    uint32_t heavy_df;
    uint32_t row_lo, row_hi;
    unsigned long long* out;
    uint64_t shard_cap;
    unsigned long long* cursor;
    unsigned long long* gstats;
    uint32_t* flags;
    uint32_t* list;
    uint32_t* list_count;
    unsigned long long* spill;
    uint64_t spill_cap;
    unsigned long long* spill_cursor;
    // spill segments (a heavy group, or a whole bucket): spill index | keys << 40, counted in
    // flags[kFlSegs], the largest in flags[kFlSegMax]; the heavy path sorts each in LDS
    unsigned long long* seg;
    uint32_t seg_cap;
    // scored calls (kScore kernels): pair keys (pair << sb) | sor | s(x), s(x) of the group's k-mer
    int k;
    unsigned sb;
    uint32_t sor;
    // k-mer split, routed (send != nullptr): each pair key goes straight to the send region of the
    // rank owning its row (rows), sub-region `shard` of send_sub keys, reserved on
    // dcur[rank * kShards + shard]; no shard regions, no route kernel (unscored calls only)
    unsigned long long* send;
    uint64_t send_cap, send_sub;
    unsigned long long* dcur;
    SplitRows rows;
    // the passes of one batch with the row-driven heavy expansion (heavy_flat_kernel): every bucket
    // goes to the heavy path whole on the first pass, so later passes launch no bucket kernel
    int spill_all;
};

// descriptor: spill index (40 bits) | keys (23 bits) << 40 | whole bucket (several k-mers) << 63
__device__ __forceinline__ void spill_segment(const BucketArgs& a, uint64_t pos, uint32_t keys, bool whole) {
    const uint32_t s = atomicAdd(&a.flags[kFlSegs], 1u);
    if (s < a.seg_cap)
        a.seg[s] = pos | (unsigned long long)min(keys, 0x7FFFFFu) << 40 | (unsigned long long)whole << 63;
    atomicMax(&a.flags[kFlSegMax], keys);
}

// One workgroup per bucket with size <= kCap (the bucket: keys with the same top bbits of
// h(code)).  In LDS:
//   A. exact k-mer groups: an open-addressing table on h (kTab >= kCap slots, the empty mark can
//      not be an h of this bucket) gives every key its group slot; LDS atomics rank it in the group;
//   B. groups are laid out by size, largest first (a counting sort over the size classes), so the
//      lanes of a wave walk groups of equal size in the loops below; singletons walk none; a group
//      above kHeavySub keys (a frequent k-mer) is spilled whole to the heavy path instead;
//   C. scatter: Bl[pos] = p << cb | class, and per position its group (start << 8 | size);
//   D. duplicate windows of one protein (same p twice in a group) count once (main.rs:99-100);
//   E. df = distinct proteins of the group; every element pairs with the later non-duplicate
//      elements of its group (vertex.rs:103-137), class test fused (mod.rs:580-587).  kRows:
//      instead every element pairs with the group's elements of a LARGER protein, and only
//      elements whose protein lies in [row_lo, row_hi) emit (the row filter of a pass / rank);
//   F. output: the workgroup reserves its range on cursor[b % kShards] and writes the pair keys.
// Thread tid owns positions tid + e*kThreads in C-F, so its per-position state stays in
// registers.  Statistics -> gstats[b % kShards] (heavy groups: the heavy path's).
// kMerge (bucket field >= kMergeMinBits): one slot word holds h's low 32 - bbits bits and the group
// count above them (the top bits of h are the bucket, equal for every key), so the table of h
// and the count table share H, and T shrinks to the per-position array: 18.9 KB of LDS at the
// small geometry, 8 workgroups (32 waves) per CU instead of 6
constexpr unsigned kMergeMinBits = 11;
// KMP_CLASS_RUNS: groups of kRunMin+ keys laid out by class (step C'), partners past the element's
// class run taken without a test.  Off: measured slower at config 3 (group_expand 0.222 -> 0.238 ms:
// the extra barrier and LDS) and at config 1 (0.443 -> 0.452 ms), whose time is not in the tests
#ifndef KMP_CLASS_RUNS
#define KMP_CLASS_RUNS 0
#endif
// KMP_BS_CUT (A/B timing builds only, wrong results): the small kernel returns after step
// 1 = A, 2 = B, 3 = C, 4 = D, 5 = E + statistics (no output)
#ifndef KMP_BS_CUT
#define KMP_BS_CUT 0
#endif
constexpr uint32_t kRunMin = 32;  // groups of at least this many keys are laid out in class runs (LDS: 640 B at 1,280 keys)
template <int kCap, int kThreads, int kTabBits, bool kMerge, bool kRows, bool kScore>
__device__ __forceinline__ void process_bucket(const uint32_t b, const BucketArgs& a, bool small) {
    constexpr int kE = kCap / kThreads;
    constexpr uint32_t kTab = 1u << kTabBits;
    constexpr int kPer = kTab / kThreads;
    constexpr int kMaxHeavy = kCap / (kHeavySub + 1) + 1;
    static_assert(kE * kThreads == kCap && kPer % 4 == 0 && kTab >= (uint32_t)kCap, "geometry");
    static_assert(!kMerge || kCap < (1 << kMergeMinBits) - 1, "merged count field");
    // T: (unmerged) A: table of h; C-E: per position start<<8|size
    __shared__ __attribute__((aligned(16))) uint32_t T[kMerge ? kCap : kTab];
    // H: per slot: (merged: h low bits | count << hb) / group size, then start<<8|size
    __shared__ __attribute__((aligned(16))) uint32_t H[kTab];
    __shared__ uint32_t Bl[kCap + 4];  // per position: p << cb | class (+4: the forward walk reads past a group)
    __shared__ uint32_t dupw[kCap / 32];   // per position: a later occurrence of a protein in its group
    __shared__ uint32_t gdupw[kCap / 32];  // per group start: the group holds such a duplicate
    __shared__ uint32_t SZ[kHeavySub + 1];
    __shared__ uint32_t wave_tot[kThreads / 64];
    __shared__ uint32_t red[kThreads / 64][kStN];  // per wave: the statistics, unpacked
    __shared__ unsigned long long sbase;
    __shared__ unsigned long long hbase[kMaxHeavy];  // spill offset of each heavy group
    __shared__ uint32_t nheavy, hkeys;
    __shared__ uint32_t anydup;  // some group of the bucket holds a duplicate window (gdupw nonzero)
    // class runs (step C): per group of at least kRunMin keys (indexed by its start / kRunMin, unique
    // since such groups start kRunMin apart) the keys of each of up to 16 classes, 8 bits a class
    __shared__ uint32_t CC[kCap / kRunMin * 4];
    uint64_t s0;
    uint32_t n;
    if (a.vreg) {
        s0 = a.vreg[b];
        n = min(a.bstart[b], a.vreg[b + 1] - a.vreg[b]);  // a larger count raised kFlCur: the call reruns
    } else if (a.capb) {
        s0 = (uint64_t)b * a.capb;
        n = min(a.bstart[b], a.capb);  // a larger count raised kFlCur: the call reruns
    } else {
        s0 = a.bstart[b];
        n = a.bstart[b + 1] - (uint32_t)s0;
    }
    const int tid = threadIdx.x;
    const Layout& lay = a.lay;
    if (n == 0) return;
    const uint32_t shard = b % kShards;
    if (n > (uint32_t)kCap || a.spill_all) {
        if (small && !a.spill_all) {
            if (tid == 0) a.list[atomicAdd(a.list_count, 1u)] = b;  // the large kernel takes it
            return;
        }
        // above every LDS capacity: the whole bucket goes to the heavy path
        if (!a.spill) return;
        __syncthreads();
        if (tid == 0) {
            sbase = atomicAdd(&a.spill_cursor[shard], (unsigned long long)n);
            spill_segment(a, (uint64_t)shard * a.spill_cap + sbase, n, true);
        }
        __syncthreads();
        unsigned long long* dst = a.spill + (uint64_t)shard * a.spill_cap;
        for (uint32_t i = tid; i < n; i += kThreads)
            if (sbase + i < a.spill_cap) dst[sbase + i] = a.sorted[s0 + i];
        return;
    }
    // the bucket's keys, every load issued before any is used (one HBM round trip per wave, not
    // one per key slot: a load inside the insert loop below waited on each in turn)
    unsigned long long xk[kE];
#pragma unroll
    for (int e = 0; e < kE; ++e) {
        const uint32_t i = tid + e * kThreads;
        xk[e] = i < n ? a.sorted[s0 + i] : 0ull;
    }
    __syncthreads();  // LDS reuse across the buckets of one workgroup
    const unsigned hshift = lay.hshift, cb = lay.clsbits;
    const uint32_t lmask = (1u << hshift) - 1, cmask = (1u << cb) - 1;
    const uint32_t empty = ~b << (32 - lay.bbits);  // top bits differ from every h of bucket b
    const unsigned hb = 32 - lay.bbits;             // merged: low h bits kept in a slot
    const uint32_t hm = (1u << hb) - 1;
    constexpr uint32_t kFree = 0xFFFFFFFFu;          // merged empty slot (count field never all ones)
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        if (!kMerge) T[tid * kPer + q] = empty;
        H[tid * kPer + q] = kMerge ? kFree : 0u;
    }
    for (uint32_t i = tid; i < kCap / 32; i += kThreads) dupw[i] = gdupw[i] = 0;
    for (uint32_t i = tid; i <= kHeavySub; i += kThreads) SZ[i] = 0;
    // class runs: the class filter on, at most 16 classes, every pair of a group (not kRows)
    const bool runs_on = KMP_CLASS_RUNS && !kRows && a.require_diff && cb >= 1 && cb <= 4;
    if (runs_on)
        for (uint32_t i = tid; i < kCap / kRunMin * 4; i += kThreads) CC[i] = 0;
    if (tid == 0) nheavy = hkeys = anydup = 0;
    __syncthreads();
    // A. group slot + rank of every key (the keys were loaded before the table clear).  (Issuing
    // every key's first probe before using any result, then the collisions, then the counts, was
    // measured slower: 643 -> 651 VALU per wave, group_expand 0.176 -> 0.180 ms at config 3)
    uint32_t xl[kE], sl[kE], rk[kE];
#pragma unroll
    for (int e = 0; e < kE; ++e) {
        const uint32_t i = tid + e * kThreads;
        const unsigned long long x = xk[e];
        const uint32_t h = (uint32_t)(x >> hshift);
        xl[e] = (uint32_t)x & lmask;
        sl[e] = 0;
        rk[e] = 0;
        if (i < n) {
            uint32_t slot = (h * 0x85EBCA6Bu) >> (32 - kTabBits);
            if (kMerge) {
                // a new k-mer goes in with its count already 1 (one atomic: most keys are the
                // first or only one of their k-mer); a later key of it adds to the count
                // (inserting a new k-mer with its count already 1 saves an atomic for most keys but
                // measured 6 % slower: the divergent two-exit loop)
                const uint32_t hl = h & hm;
                for (;;) {
                    const uint32_t old = atomicCAS(&H[slot], kFree, hl);
                    if (old == kFree || (old & hm) == hl) break;
                    slot = (slot + 1) & (kTab - 1);
                }
                rk[e] = atomicAdd(&H[slot], 1u << hb) >> hb;
                sl[e] = slot;
            } else {
                for (;;) {
                    const uint32_t old = atomicCAS(&T[slot], empty, h);
                    if (old == empty || old == h) break;
                    slot = (slot + 1) & (kTab - 1);
                }
                sl[e] = slot;
                rk[e] = atomicAdd(&H[slot], 1u);
            }
        }
    }
    __syncthreads();
    if (KMP_BS_CUT == 1 && small) return;
    // B. size classes, largest first.  Each group's first key (rank 0) stands for it (count from
    // its slot word, size-class rank, position rewrite), so the pass is per key, not over all kTab
    // table slots (measured 6 % faster); singleton groups (most) take no rank and no position.
    // A heavy group's first key reserves its spill range (one returning atomic per bucket).
    uint32_t single = 0;
    uint32_t cn[kE], rr[kE];
#pragma unroll
    for (int e = 0; e < kE; ++e) {
        cn[e] = rr[e] = 0;
        if (tid + e * kThreads >= n) continue;
        if (rk[e] != 0) {  // a later key of a group of two or more: step C's word gives its size
            cn[e] = 2;
            continue;
        }
        const uint32_t w = H[sl[e]];
        cn[e] = kMerge ? w >> hb : w;
        if (cn[e] > kHeavySub) {
            if (a.spill) {
                rr[e] = atomicAdd(&nheavy, 1u);
                hbase[rr[e]] = atomicAdd(&hkeys, cn[e]);  // offset inside the bucket's spill range
            }
        } else if (cn[e] == 1) {
            ++single;
        } else {
            rr[e] = atomicAdd(&SZ[cn[e]], 1u);
        }
    }
    __syncthreads();
    if (tid == 0 && hkeys) sbase = atomicAdd(&a.spill_cursor[shard], (unsigned long long)hkeys);
    uint32_t nm;  // keys in groups of two or more: positions [0, nm)
    {
        const bool cls = tid + 2 <= (int)kHeavySub;                       // classes kHeavySub .. 2
        const uint32_t m = cls ? kHeavySub - tid : 0;
        const uint32_t v = cls ? m * SZ[m] : 0u;
        uint32_t excl;
        block_scan_n<kThreads>(v, excl, nm, wave_tot);  // barriers: sbase visible after it
        if (cls) SZ[m] = excl;  // first position of size class m
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < kE; ++e)
        if (rk[e] == 0 && cn[e] >= 2) {
            // start << 8 | size (start < 4,096: 20 bits); scored: s(x) of the group's k-mer in bits
            // 24-30; a heavy group: bit 31 | its index in hbase
            const uint32_t sc = kScore && cn[e] <= kHeavySub ? kmer_self_score((uint32_t)(xk[e] >> hshift), a.k) << 24 : 0u;
            H[sl[e]] = cn[e] > kHeavySub ? 0x80000000u | rr[e] : ((SZ[cn[e]] + rr[e] * cn[e]) << 8) | cn[e] | sc;
        }
    __syncthreads();
    if (KMP_BS_CUT == 2 && small) return;
    // C. scatter (T now holds, per position, its group's start << 8 | size); heavy groups' keys
    // go to the spill region
    unsigned long long* spill_dst = a.spill ? a.spill + (uint64_t)shard * a.spill_cap : nullptr;
#pragma unroll
    for (int e = 0; e < kE; ++e) {
        const uint32_t i = tid + e * kThreads;
        if (i >= n || cn[e] < 2) continue;  // singleton
        const uint32_t g = H[sl[e]];
        if (g >> 31) {  // heavy
            if (spill_dst) {
                const unsigned long long pos = sbase + hbase[g & 0x7FFFFFFFu] + rk[e];
                if (pos < a.spill_cap) spill_dst[pos] = xk[e];
                if (rk[e] == 0) spill_segment(a, (uint64_t)shard * a.spill_cap + pos, cn[e], false);
            }
            cn[e] = kHeavySub + 1;
            continue;
        }
        cn[e] = g & 255u;
        const uint32_t gs = kScore ? (g >> 8) & 0xFFFFu : g >> 8;
        T[gs + rk[e]] = g;
        if (runs_on && cn[e] >= kRunMin) {  // its rank in its class; placed below by class
            const uint32_t c = xl[e] & cmask, sh = 8 * (c & 3);
            rr[e] = (atomicAdd(&CC[gs / kRunMin * 4 + (c >> 2)], 1u << sh) >> sh) & 0xFFu;
        } else {
            Bl[gs + rk[e]] = xl[e];
        }
    }
    __syncthreads();
    if (KMP_BS_CUT == 3 && small) return;
    // keys of classes below c in the group starting at gs (class-run mode), and of class c
    auto run_of = [&](uint32_t gs, uint32_t c, uint32_t& below, uint32_t& same) {
        const uint32_t* cc = CC + gs / kRunMin * 4;
        below = 0;
#pragma unroll
        for (uint32_t w = 0; w < 4; ++w) {
            const uint32_t x = cc[w];
#pragma unroll
            for (uint32_t t = 0; t < 4; ++t)
                if (w * 4 + t < c) below += (x >> (8 * t)) & 0xFFu;
        }
        same = (cc[c >> 2] >> (8 * (c & 3))) & 0xFFu;
    };
    if (runs_on) {
        // C'. a group of at least kRunMin keys laid out by class (ascending): an element's
        // cross-class partners after it are then exactly the positions past its class run, so E
        // counts them without a test and F writes them without one (config 1: 258M partners
        // tested for 5.3M kept)
#pragma unroll
        for (int e = 0; e < kE; ++e) {
            const uint32_t i = tid + e * kThreads;
            if (i >= n || cn[e] < kRunMin || cn[e] > kHeavySub) continue;
            const uint32_t g = H[sl[e]];
            const uint32_t gs = kScore ? (g >> 8) & 0xFFFFu : g >> 8;
            uint32_t below, same;
            run_of(gs, xl[e] & cmask, below, same);
            Bl[gs + below + rr[e]] = xl[e];
        }
        __syncthreads();
    }
    // D. per position: group bounds, duplicate flag (same protein earlier in the group: the same
    // p << cb | class word); a group holding one marks its start in gdupw.
    // fwd (every pair of a group, no class runs): one forward walk over the partners after i does
    // both D and E's partner test — the kept partners go to cnt (a bit mask in a group of at most 33
    // keys, else their count) and an equal word j > i marks j as a duplicate (rare: the group then
    // takes E's walk over the whole group).  No separate backward duplicate scan (config 3: 62 VALU
    // instructions per wave).
    uint32_t s[kE], en[kE], cnt[kE];
    constexpr bool kMask = kThreads <= 256;  // the large kernel measured slower with it (74 -> 80 us, config 1)
    const bool fwd = !kRows && !runs_on;
#pragma unroll
    for (int e = 0; e < kE; ++e) {
        const uint32_t i = tid + e * kThreads;
        s[e] = en[e] = cnt[e] = 0;
        if (i >= nm) continue;
        const uint32_t g = T[i];
        s[e] = kScore ? (g >> 8) & 0xFFFFu : g >> 8;
        en[e] = s[e] + (g & 255u);
        xl[e] = Bl[i];
        if (fwd) {
            uint32_t acc = 0;
            auto mark = [&](uint32_t j) {
                atomicOr(&dupw[j >> 5], 1u << (j & 31));
                atomicOr(&gdupw[s[e] >> 5], 1u << (s[e] & 31));
                anydup = 1;
            };
            if (kMask && en[e] - s[e] <= 33u) {
                // four partners per step (two ds_read2 of consecutive words; words past en are read
                // and masked off: Bl is followed by other LDS arrays, never out of the allocation)
                const uint32_t span = en[e] - 1 - i;
                for (uint32_t j = i + 1; j < en[e]; j += 4) {
                    const uint32_t l0 = Bl[j], l1 = Bl[j + 1], l2 = Bl[j + 2], l3 = Bl[j + 3];
                    const uint32_t d = j - i - 1;
                    auto kp = [&](uint32_t lj) { return (uint32_t)(!a.require_diff || ((lj ^ xl[e]) & cmask) != 0u); };
                    acc |= (kp(l0) | kp(l1) << 1 | kp(l2) << 2 | kp(l3) << 3) << d;
                    if ((l0 == xl[e]) | (l1 == xl[e]) | (l2 == xl[e]) | (l3 == xl[e])) {
                        if (l0 == xl[e]) mark(j);
                        if (l1 == xl[e] && j + 1 < en[e]) mark(j + 1);
                        if (l2 == xl[e] && j + 2 < en[e]) mark(j + 2);
                        if (l3 == xl[e] && j + 3 < en[e]) mark(j + 3);
                    }
                }
                acc &= span >= 32u ? ~0u : (1u << span) - 1u;
            } else {
                for (uint32_t j = i + 1; j < en[e]; ++j) {
                    const uint32_t lj = Bl[j];
                    acc += !a.require_diff || ((lj ^ xl[e]) & cmask) != 0u;
                    if (lj == xl[e]) mark(j);
                }
            }
            cnt[e] = acc;
            continue;
        }
        uint32_t j0 = s[e];
        if (runs_on && en[e] - s[e] >= kRunMin) {  // a duplicate shares the class: its run only
            uint32_t below, same;
            run_of(s[e], xl[e] & cmask, below, same);
            j0 = s[e] + below;
        }
        for (uint32_t j = j0; j < i; ++j)
            if (Bl[j] == xl[e]) {
                atomicOr(&dupw[i >> 5], 1u << (i & 31));
                atomicOr(&gdupw[s[e] >> 5], 1u << (s[e] & 31));
                anydup = 1;
                break;
            }
    }
    __syncthreads();
    if (KMP_BS_CUT == 4 && small) return;
    auto is_dup = [&](uint32_t j) { return (dupw[j >> 5] >> (j & 31)) & 1u; };
    // E. df, head, kept-partner count.  A group without duplicates (almost all) has df = its size
    // and counts its partners after i only; a group with one walks the whole group.  In a group of
    // at most 33 keys without duplicates (nearly all), cnt holds the kept partners as a bit mask
    // (bit t: position i + 1 + t) instead of their count, so F visits only the kept partners (at
    // config 3 they are 5.3M of the 22.5M partners the class test looks at) without re-reading and
    // re-testing the others.  The mode follows from s, en and gd (no register), and is the same for
    // a whole group, so a wave walking one large group does not run both loops of F (deciding it per
    // element, by the partners after i, measured 5 % slower at config 1).
    bool gd[kE];
    // kRows: bit t = position s + t (every partner of a larger protein, anywhere in the group)
    auto run_mode = [&](int e) { return runs_on && !gd[e] && en[e] - s[e] >= kRunMin; };
    auto mask_mode = [&](int e) { return kMask && !gd[e] && en[e] - s[e] <= (kRows ? 32u : 33u) && !run_mode(e); };
    const bool anyd = anydup;  // (uniform) most buckets hold no duplicate window: no gdupw reads
    uint32_t st_sum = single, st_dist = single, st_rep = 0, st_cdf2 = 0, st_max = single ? 1u : 0u, st_heavy = 0,
             mine = 0;
#pragma unroll
    for (int e = 0; e < kE; ++e) {
        const uint32_t i = tid + e * kThreads;
        const uint32_t pre = cnt[e];  // fwd: D's kept partners (mask or count)
        cnt[e] = 0;
        gd[e] = false;
        if (i >= nm) continue;
        gd[e] = anyd && ((gdupw[s[e] >> 5] >> (s[e] & 31)) & 1u);
        if (gd[e] && is_dup(i)) continue;
        uint32_t f, c = 0, bits = 0;
        if (kRows) {
            // df, and the partners of a larger protein when this element's protein is in the rows
            const uint32_t p = xl[e] >> cb;
            const bool emit = p >= a.row_lo && p < a.row_hi;
            f = gd[e] ? 0u : en[e] - s[e];
            if (emit || gd[e])
                for (uint32_t j = s[e]; j < en[e]; ++j) {
                    if (gd[e] && is_dup(j)) continue;
                    f += gd[e];
                    const uint32_t lj = Bl[j];
                    const bool k = emit && (lj >> cb) > p && (!a.require_diff || ((lj ^ xl[e]) & cmask));
                    c += k;
                    if (kMask && j - s[e] < 32u) bits |= (uint32_t)k << (j - s[e]);
                }
        } else if (run_mode(e)) {  // class runs: the positions past its run, all kept
            f = en[e] - s[e];
            uint32_t below, same;
            run_of(s[e], xl[e] & cmask, below, same);
            c = en[e] - (s[e] + below + same);
        } else if (fwd && !gd[e]) {
            f = en[e] - s[e];
            if (kMask && en[e] - s[e] <= 33u) {
                bits = pre;
                c = __popc(bits);
            } else {
                c = pre;
            }
        } else if (!gd[e]) {
            f = en[e] - s[e];
            const uint32_t span = en[e] - 1 - i;
            if (kMask && en[e] - s[e] <= 33u) {
                if (a.require_diff) {
                    for (uint32_t j = i + 1; j < en[e]; ++j)
                        bits |= (uint32_t)(((Bl[j] ^ xl[e]) & cmask) != 0u) << (j - i - 1);
                } else {
                    bits = span == 32u ? ~0u : (1u << span) - 1u;
                }
                c = __popc(bits);
            } else if (a.require_diff) {
                for (uint32_t j = i + 1; j < en[e]; ++j) c += ((Bl[j] ^ xl[e]) & cmask) != 0u;
            } else {
                c = span;
            }
        } else {
            f = 0;
            for (uint32_t j = s[e]; j < en[e]; ++j) {
                if (is_dup(j)) continue;
                ++f;
                if (j > i && (!a.require_diff || ((Bl[j] ^ xl[e]) & cmask))) ++c;
            }
        }
        if (f > a.heavy_df) c = bits = 0;
        st_sum += 1;
        if (i == s[e]) {  // the group's first position is never a duplicate
            st_dist += 1;
            st_rep += f >= 2;
            if (f <= a.heavy_df) st_cdf2 += f * (f - 1) / 2;
            else st_heavy += f;
            st_max = max(st_max, f);
        }
        cnt[e] = mask_mode(e) ? bits : c;
        mine += c;
    }
    // statistics: three wave reductions of packed words (per workgroup every count is at most
    // kCap, so 16-bit fields cannot carry; C(df,2) and the incidences stay below 2^32), wave
    // partials -> red, then kStN threads unpack, sum and post one (sharded) atomic each.  They
    // ride on the output scan's barriers; the last wave reserves the output range meanwhile.
    {
        // DPP wave sums of packed fields (the incidences are the output scan's total).  kCap below
        // 2^11: Σ|K| | distinct << 11 | repeat << 22 (each at most kCap, repeat at most kCap / 2)
        // and C(df,2) | heavy << 17 (at most kCap / 128 groups of C(128,2) < 2^17) in two sums;
        // else 16-bit fields in three
        const uint32_t mx = wave_max(st_max);
        uint32_t v0, v1, v2, v3, v4;  // Σ|K|, distinct, repeat, heavy, C(df,2)
        if (kCap < 2048) {
            const uint32_t s0 = wave_sum(st_sum | st_dist << 11 | st_rep << 22);
            const uint32_t s1 = wave_sum(st_cdf2 | st_heavy << 17);
            v0 = s0 & 0x7FFu, v1 = (s0 >> 11) & 0x7FFu, v2 = s0 >> 22, v3 = s1 >> 17, v4 = s1 & 0x1FFFFu;
        } else {
            const uint32_t s0 = wave_sum(st_sum | st_dist << 16), s1 = wave_sum(st_rep | st_heavy << 16);
            v0 = s0 & 0xFFFFu, v1 = s0 >> 16, v2 = s1 & 0xFFFFu, v3 = s1 >> 16, v4 = wave_sum(st_cdf2);
        }
        if ((tid & 63) == 0) {
            uint32_t* rw = red[tid >> 6];
            rw[kStSumS] = v0, rw[kStDistinct] = v1, rw[kStRepeat] = v2, rw[kStHeavy] = v3, rw[kStCdf2] = v4;
            rw[kStMaxDf] = mx, rw[kStInc] = 0;
        }
    }
    uint32_t excl, total;
    block_scan_n<kThreads>(mine, excl, total, wave_tot);
    if (tid == kThreads - 64 && !a.send) sbase = total ? atomicAdd(&a.cursor[shard], (unsigned long long)total) : 0ull;
    if (tid < kStN) {
        uint32_t v = 0;
#pragma unroll
        for (int w = 0; w < kThreads / 64; ++w) {
            const uint32_t x = red[w][tid];
            v = tid == kStMaxDf ? max(v, x) : v + x;
        }
        if (tid == kStInc) v = total;
        unsigned long long* g = a.gstats + (uint64_t)shard * 8 + tid;  // sharded: no hot word
        if (tid == kStMaxDf) atomicMax(g, (unsigned long long)v);
        else if (v) atomicAdd(g, (unsigned long long)v);
    }
    __syncthreads();
    if (KMP_BS_CUT == 5 && small) return;
    // F. write the pair keys.  When the bucket's keys fit (almost always) they are staged in LDS
    // (H is dead after C) at each element's scanned offset and copied out coalesced; each lane
    // writing its own short run straight to HBM cost one memory transaction per key (a bucket
    // kernel without the partner loops ran 151 us instead of 236 us at config 3).
    unsigned long long* dst = a.out + (uint64_t)shard * a.shard_cap;
    auto partners = [&](auto put) {
#pragma unroll
        for (int e = 0; e < kE; ++e) {
            if (!cnt[e]) continue;
            const uint32_t i = tid + e * kThreads;
            const uint32_t p = xl[e] >> cb;
            // scored: every key of the element carries its k-mer's self-score and the call's k bit
            const uint32_t sfield = kScore ? a.sor | T[s[e]] >> 24 : 0u;
            auto pkey = [&](uint32_t q) {
                const unsigned long long pk = (unsigned long long)min(p, q) * a.mul + max(p, q);
                return kScore ? pk << a.sb | sfield : pk;
            };
            if (run_mode(e)) {
                uint32_t below, same;
                run_of(s[e], xl[e] & cmask, below, same);
                for (uint32_t j = s[e] + below + same; j < en[e]; ++j) put(pkey(Bl[j] >> cb));
                continue;
            }
            if (mask_mode(e)) {
                const uint32_t base = kRows ? s[e] : i + 1;
                for (uint32_t m = cnt[e]; m; m &= m - 1) {
                    const uint32_t q = Bl[base + __builtin_ctz(m)] >> cb;
                    put(pkey(q));
                }
                continue;
            }
            for (uint32_t j = kRows ? s[e] : i + 1; j < en[e]; ++j) {
                if (gd[e] && is_dup(j)) continue;
                const uint32_t lj = Bl[j];
                if (a.require_diff && !((lj ^ xl[e]) & cmask)) continue;
                const uint32_t q = lj >> cb;
                if (kRows && q <= p) continue;
                put(pkey(q));
            }
        }
    };
    constexpr uint32_t kStage = kTab / 2;
    if (!kScore && a.send) {  // the k-mer split: straight to the row owners' send sub-regions
        // (SZ and CC are dead after step C: per-destination counts / row starts, and bases)
        uint32_t* dcnt = SZ;
        uint32_t* rst = SZ + 64;
        uint32_t* dbase = CC;
        static_assert(kHeavySub + 1 >= 64 + kSplitMax + 1 && kCap / kRunMin * 4 >= kSplitMax, "route tables");
        const uint32_t parts = a.rows.parts;
        if (tid < (int)parts) dcnt[tid] = 0;
        if (tid <= (int)parts) rst[tid] = a.rows.start[tid];
        const unsigned pb = lay.pbits;
        auto dest = [&](unsigned long long key) {  // the rank owning row min(p, q)
            const uint32_t p = (uint32_t)(key >> pb);
            uint32_t lo = 0, hi = parts;  // last d with rst[d] <= p
            while (lo + 1 < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (rst[mid] <= p) lo = mid;
                else hi = mid;
            }
            return lo;
        };
        auto reserve = [&]() {
            if (tid < (int)parts)
                dbase[tid] = dcnt[tid] ? (uint32_t)atomicAdd(&a.dcur[tid * kShards + shard], (unsigned long long)dcnt[tid])
                                       : 0u;
        };
        auto put = [&](uint32_t d, uint32_t pos, unsigned long long key) {
            if (pos < a.send_sub) a.send[d * a.send_cap + (uint64_t)shard * a.send_sub + pos] = key;
        };
        if (total <= kStage) {  // staged: ranked per destination in LDS, one reservation each
            unsigned long long* stage = reinterpret_cast<unsigned long long*>(H);
            uint32_t lpos = excl;
            if (mine) partners([&](unsigned long long key) { stage[lpos++] = key; });
            __syncthreads();
            constexpr uint32_t kSt = kStage / kThreads;
            uint32_t dr[kSt];
#pragma unroll
            for (uint32_t j = 0; j < kSt; ++j) {
                const uint32_t t = tid + j * kThreads;
                dr[j] = ~0u;
                if (t < total) {
                    const uint32_t d = dest(stage[t]);
                    dr[j] = d << 24 | atomicAdd(&dcnt[d], 1u);
                }
            }
            __syncthreads();
            reserve();
            __syncthreads();
#pragma unroll
            for (uint32_t j = 0; j < kSt; ++j)
                if (dr[j] != ~0u) put(dr[j] >> 24, dbase[dr[j] >> 24] + (dr[j] & 0xFFFFFFu), stage[tid + j * kThreads]);
        } else {  // a bucket above the staging: count, reserve, then write with LDS cursors
            __syncthreads();
            if (mine) partners([&](unsigned long long key) { atomicAdd(&dcnt[dest(key)], 1u); });
            __syncthreads();
            reserve();
            __syncthreads();
            if (tid < (int)parts) dcnt[tid] = 0;
            __syncthreads();
            if (mine)
                partners([&](unsigned long long key) {
                    const uint32_t d = dest(key);
                    put(d, dbase[d] + atomicAdd(&dcnt[d], 1u), key);
                });
        }
        return;
    }
    if (total <= kStage) {  // uniform over the workgroup
        unsigned long long* stage = reinterpret_cast<unsigned long long*>(H);
        uint32_t lpos = excl;
        if (mine) partners([&](unsigned long long key) { stage[lpos++] = key; });
        __syncthreads();
        for (uint32_t t = tid; t < total; t += kThreads)
            if (sbase + t < a.shard_cap) dst[sbase + t] = stage[t];
    } else if (mine) {
        unsigned long long pos = sbase + excl;
        partners([&](unsigned long long key) {
            if (pos < a.shard_cap) dst[pos] = key;
            ++pos;
        });
    }
}

// KMP_BS_WAVES: an occupancy floor for the small kernel (waves per SIMD; 0: the compiler's choice)
#ifndef KMP_BS_WAVES
#define KMP_BS_WAVES 8  // 64 VGPRs: 8 workgroups per CU (LDS allows 8); group_expand 0.238 -> 0.222 ms at config 3
#endif
template <int kCap, int kThreads, int kTabBits, bool kMerge, bool kRows, bool kScore>
__global__ __launch_bounds__(kThreads, KMP_BS_WAVES ? KMP_BS_WAVES * 256 / kThreads : 1) void bucket_small_kernel(BucketArgs a, uint32_t b0) {
    process_bucket<kCap, kThreads, kTabBits, kMerge, kRows, kScore>(b0 + blockIdx.x, a, true);
}

// the buckets the small kernel listed (above its capacity), a grid-stride loop over the list
template <int kCap, int kThreads, int kTabBits, bool kRows, bool kScore>
__global__ __launch_bounds__(kThreads) void bucket_large_kernel(BucketArgs a) {
    const uint32_t m = *a.list_count;
    for (uint32_t i = blockIdx.x; i < m; i += gridDim.x)
        process_bucket<kCap, kThreads, kTabBits, false, kRows, kScore>(a.list[i], a, false);
}


// ------------------------------------------------------------- heavy path ------------------
// Frequent k-mers (a group above kHeavySub keys) and buckets above every LDS capacity are
// spilled by the bucket kernels (their keys, unchanged) and expanded here, with no cap on df:
//   1. the spilled keys, gathered, are radix sorted on (h, p) (bits [clsbits, 63)): one run per
//      k-mer, its proteins ascending, duplicate windows of one protein adjacent;
//   2. heavy_scan / heavy_compact (4,096-key tiles + a scan of the tile counts): the distinct
//      (k-mer, protein) elements E = p << cb | class, and each k-mer's start GS[g] in E;
//      df(g) = GS[g+1] - GS[g] (main.rs:77-122 restated on the spill);
//   3. heavy_plan (one thread per k-mer): statistics, the element range [i0, i1) whose proteins
//      lie in the call's rows, and the tile count: element blocks of kHvI rows x partner chunks
//      of kHvJ (the upper triangle of the k-mer's C(df,2) pairs, vertex.rs:103-137);
//   4. heavy_expand (one workgroup per tile): the partner chunk in LDS, one row per thread, the
//      class test (mod.rs:580-587) on every pair (p_i, p_j), j > i; a workgroup scan and one
//      cursor reservation place the pair keys p_i * mul + p_j in the shard regions the bucket
//      kernels fill.  A k-mer of df 10^4 is ~400 tiles: no workgroup walks a long posting list.
constexpr uint32_t kHvTile = 4096, kHvThreads = 256, kHvPer = kHvTile / kHvThreads;
constexpr uint32_t kHvI = 256, kHvJ = 256, kHvMW = kHvJ / 32;
constexpr uint32_t kHvSpread = 64 * 256;  // a tile with this many pairs spreads them over the shards
// flat tiles (class order, every pair kept, a k-mer of at most kHvFlatRuns class runs): the
// k-mer's cross-class pairs (row of run r, any element past r's end) numbered run by run, row by
// row, cut into kHvFlat-pair tiles: every tile full, nothing per row to plan
constexpr uint32_t kHvFlat = 1024, kHvFlatRuns = 64, kHvFlatMark = 0xFFFFFFFFu;

// Heavy key order.  Plain: the spilled keys [h | p | class] sorted on (h, p).  Class order (the
// class test is on): gather_shards rewrites them to [h | class | p] and the sort is on every bit,
// so each k-mer's elements come in class runs, proteins ascending inside a run.  A pair of
// different classes is then (row i, partner j) with j past the end of i's run: the expansion
// walks only those — at k = 5 on uniprot_arg 98% of a frequent k-mer's pairs share a class and
// were enumerated and tested one by one in the plain order.
struct HeavyOrder {
    unsigned cb, hshift, pbits;  // class bits, h shift, protein bits (hshift - cb)
    int cls;                     // class order
    uint32_t hj;                 // partners per tile (<= kHvJ)
    // element-distinct test shift: plain keys drop the class (a function of p), class-ordered keys
    // compare whole
    __host__ __device__ unsigned eshift() const { return cls ? 0u : cb; }
    // E value (p << cb | class) of a sorted key
    __device__ uint32_t elem(unsigned long long v) const {
        const unsigned long long lmask = (1ull << hshift) - 1;
        if (!cls) return (uint32_t)(v & lmask);
        const uint32_t pm = (uint32_t)((1ull << pbits) - 1), cm = (1u << cb) - 1;
        return ((uint32_t)v & pm) << cb | ((uint32_t)(v >> pbits) & cm);
    }
};

// spill shard regions -> one contiguous array (shard order); class order: keys rewritten to
// [h | class | p]
__global__ void gather_shards_kernel(const unsigned long long* __restrict__ src, uint64_t shard_cap,
                                     const unsigned long long* __restrict__ cursor, HeavyOrder ho,
                                     unsigned long long* __restrict__ dst) {
    const int s = blockIdx.y;
    unsigned long long off = 0;
    for (int t = 0; t < s; ++t) off += cursor[t];
    const unsigned long long m = cursor[s];
    const unsigned long long cm = (1ull << ho.cb) - 1, hm = ~((1ull << ho.hshift) - 1);
    for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < m;
         i += (unsigned long long)gridDim.x * blockDim.x) {
        const unsigned long long v = src[(uint64_t)s * shard_cap + i];
        dst[off + i] = ho.cls ? (v & hm) | (v & cm) << ho.pbits | ((v & ~hm) >> ho.cb) : v;
    }
}

// The spill is a list of segments (BucketArgs::seg): one heavy group (one k-mer) or one whole
// bucket, each holding every key of its k-mers.  Each sorted alone, in LDS, and written where the
// gather would have put it, is the whole sort the heavy path needs (k-mers contiguous, each
// sorted): no global radix sort (eight onesweep passes over 1M keys at k = 5, 0.3 ms).  One
// workgroup per segment.  Above kSegSmall keys: a block radix sort (rocprim, 8-bit digits,
// 1,024 threads) of the key bits that differ — [0, hshift) for one k-mer (protein and class: four
// passes instead of eight), every bit for a whole bucket (0.057 ms at config 1 against 0.074 ms
// for a bitonic sort).
constexpr uint32_t kSegSmall = 2048, kSegLarge = 8192, kSegItems = 8;
template <uint32_t kLo, uint32_t kN>
__global__ __launch_bounds__(kN / kSegItems) void heavy_segsort_kernel(const unsigned long long* __restrict__ spill,
                                                                       uint64_t spill_cap,
                                                                       const unsigned long long* __restrict__ cursor,
                                                                       const unsigned long long* __restrict__ seg,
                                                                       HeavyOrder ho,
                                                                       unsigned long long* __restrict__ out) {
    constexpr uint32_t kThreads = kN / kSegItems;
    using Sort = rocprim::block_radix_sort<unsigned long long, kThreads, kSegItems>;
    __shared__ typename Sort::storage_type st;
    const unsigned long long sd = seg[blockIdx.x];
    const uint32_t cnt = (uint32_t)(sd >> 40) & 0x7FFFFFu;
    if (cnt <= kLo || cnt > kN) return;
    const bool whole = sd >> 63;
    if (ho.cls && !whole) return;  // heavy_segclass_kernel
    const uint64_t pos = sd & ((1ull << 40) - 1), shard = pos / spill_cap;
    uint64_t dst = pos - shard * spill_cap;
    for (uint64_t t = 0; t < shard; ++t) dst += cursor[t];
    const unsigned long long cm = (1ull << ho.cb) - 1, hm = ~((1ull << ho.hshift) - 1);
    unsigned long long k[kSegItems];  // blocked: thread t holds keys t * kSegItems + e
#pragma unroll
    for (uint32_t e = 0; e < kSegItems; ++e) {
        const uint32_t i = threadIdx.x * kSegItems + e;
        unsigned long long v = ~0ull;  // padding: after every key (the sort is stable)
        if (i < cnt) {
            v = spill[pos + i];
            if (ho.cls) v = (v & hm) | (v & cm) << ho.pbits | ((v & ~hm) >> ho.cb);
        }
        k[e] = v;
    }
    Sort().sort(k, st, 0, whole ? 64u : ho.hshift);
#pragma unroll
    for (uint32_t e = 0; e < kSegItems; ++e) {
        const uint32_t i = threadIdx.x * kSegItems + e;
        if (i < cnt) out[dst + i] = k[e];
    }
}

// Class order, one k-mer per segment (a heavy group, not a whole bucket): what the compaction and the
// class-order expansion need is class runs in ascending class, each protein once per run — not its
// proteins ascending (only plain order, the ranged calls', searches by protein).  So: a counting sort
// by class in LDS, a protein's later windows dropped through an LDS hash set on p (vertex.rs:59-140
// counts a protein once per k-mer), and the segment's tail (as many slots as windows dropped) filled
// with copies of its last key, which the compaction sees as duplicates of their neighbour.  O(n) per
// segment with four barriers, instead of a bitonic sort (66 compare-exchange rounds at 2,048 keys) or
// a 4-pass block radix sort.  A segment whose classes reach kScClasses sorts its keys in LDS (bitonic)
// instead.
constexpr uint32_t kScThreads = 512, kScItems = kSegLarge / kScThreads, kScClasses = 256, kScSlots = 2 * kSegLarge;
__global__ __launch_bounds__(kScThreads) void heavy_segclass_kernel(const unsigned long long* __restrict__ spill,
                                                                    uint64_t spill_cap,
                                                                    const unsigned long long* __restrict__ cursor,
                                                                    const unsigned long long* __restrict__ seg,
                                                                    HeavyOrder ho, unsigned long long* __restrict__ out) {
    __shared__ union {
        uint32_t P[kScSlots];            // hash set of the segment's proteins (64 KB)
        unsigned long long K[kSegLarge]; // the fallback's keys
    } u;
    __shared__ uint32_t CH[kScClasses];  // keys per class, then each class run's start
    __shared__ uint32_t wave_tot[kScThreads / 64];
    __shared__ uint32_t s_maxc;
    __shared__ unsigned long long s_last;
    const unsigned long long sd = seg[blockIdx.x];
    const uint32_t cnt = (uint32_t)(sd >> 40) & 0x7FFFFFu;
    if ((sd >> 63) || cnt > kSegLarge) return;  // a whole bucket, or above the LDS: the sorts
    const uint32_t tid = threadIdx.x;
    const uint64_t pos = sd & ((1ull << 40) - 1), shard = pos / spill_cap;
    uint64_t dst = pos - shard * spill_cap;
    for (uint64_t t = 0; t < shard; ++t) dst += cursor[t];
    const unsigned long long cm = (1ull << ho.cb) - 1, hm = ~((1ull << ho.hshift) - 1);
    const uint32_t pm = (uint32_t)((1ull << ho.pbits) - 1);
    unsigned long long v[kScItems];
    uint32_t mc = 0;
#pragma unroll
    for (uint32_t e = 0; e < kScItems; ++e) {
        const uint32_t i = tid + e * kScThreads;
        v[e] = ~0ull;
        if (i < cnt) {
            const unsigned long long x = spill[pos + i];
            v[e] = (x & hm) | (x & cm) << ho.pbits | ((x & ~hm) >> ho.cb);  // [h | class | p]
            mc = max(mc, (uint32_t)(v[e] >> ho.pbits) & (uint32_t)cm);
        }
    }
    for (uint32_t i = tid; i < kScSlots; i += kScThreads) u.P[i] = 0xFFFFFFFFu;
    for (uint32_t i = tid; i < kScClasses; i += kScThreads) CH[i] = 0;
    if (tid == 0) s_maxc = 0;
    __syncthreads();
    const uint32_t wm = wave_max(mc);
    if ((tid & 63) == 0) atomicMax(&s_maxc, wm);
    __syncthreads();
    if (s_maxc >= kScClasses) {  // (uniform) many classes: a bitonic sort of the segment
        uint32_t N = 1;
        while (N < cnt) N <<= 1;
        __syncthreads();  // P is dead: K reuses it
        for (uint32_t i = tid; i < N; i += kScThreads) u.K[i] = ~0ull;
        __syncthreads();
#pragma unroll
        for (uint32_t e = 0; e < kScItems; ++e) {
            const uint32_t i = tid + e * kScThreads;
            if (i < cnt) u.K[i] = v[e];
        }
        __syncthreads();
        for (uint32_t k = 2; k <= N; k <<= 1)
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t i = tid; i < N / 2; i += kScThreads) {
                    const uint32_t lo = 2 * j * (i / j) + (i % j), hi = lo + j;
                    const unsigned long long x = u.K[lo], y = u.K[hi];
                    if ((x > y) == !(lo & k)) {
                        u.K[lo] = y;
                        u.K[hi] = x;
                    }
                }
                __syncthreads();
            }
        for (uint32_t i = tid; i < cnt; i += kScThreads) out[dst + i] = u.K[i];
        return;
    }
    // a protein's first window in the segment keeps its key, later ones are dropped; each kept key
    // ranked in its class
    uint32_t rk[kScItems];
#pragma unroll
    for (uint32_t e = 0; e < kScItems; ++e) {
        rk[e] = ~0u;
        if (v[e] == ~0ull) continue;
        const uint32_t p = (uint32_t)v[e] & pm;
        uint32_t sl = (p * 0x9E3779B1u) >> (32 - 14);  // kScSlots = 2^14
        bool first = false;
        while (true) {
            const uint32_t old = atomicCAS(&u.P[sl], 0xFFFFFFFFu, p);
            if (old == 0xFFFFFFFFu) {
                first = true;
                break;
            }
            if (old == p) break;
            sl = (sl + 1) & (kScSlots - 1);
        }
        if (first) rk[e] = atomicAdd(&CH[(uint32_t)(v[e] >> ho.pbits) & (uint32_t)cm], 1u);
    }
    __syncthreads();
    lds_bins_scan<kScThreads>(CH, kScClasses, wave_tot);  // CH: run starts; the kept count below
    uint32_t kept = 0;
#pragma unroll
    for (uint32_t e = 0; e < kScItems; ++e)
        if (rk[e] != ~0u) {
            const uint32_t at = CH[(uint32_t)(v[e] >> ho.pbits) & (uint32_t)cm] + rk[e];
            out[dst + at] = v[e];
            ++kept;
        }
    // the segment's last kept key: the largest (class, position) — the highest class run's last slot
    uint32_t D, excl;
    block_scan_n<kScThreads>(kept, excl, D, wave_tot);
#pragma unroll
    for (uint32_t e = 0; e < kScItems; ++e)
        if (rk[e] != ~0u && CH[(uint32_t)(v[e] >> ho.pbits) & (uint32_t)cm] + rk[e] == D - 1) s_last = v[e];
    __syncthreads();
    const unsigned long long last = s_last;
    for (uint32_t i = D + tid; i < cnt; i += kScThreads) out[dst + i] = last;
}

// the small segments (<= kSegSmall keys): a bitonic sort of the next power of two, 256 threads
// (the radix sort's four passes measured 0.081 ms there against 0.064 ms)
template <uint32_t kN, uint32_t kThreads>
__global__ __launch_bounds__(kThreads) void heavy_segsort_bitonic_kernel(
    const unsigned long long* __restrict__ spill, uint64_t spill_cap, const unsigned long long* __restrict__ cursor,
    const unsigned long long* __restrict__ seg, HeavyOrder ho, unsigned long long* __restrict__ out) {
    __shared__ unsigned long long K[kN];
    const unsigned long long sd = seg[blockIdx.x];
    const uint32_t cnt = (uint32_t)(sd >> 40) & 0x7FFFFFu;
    if (cnt > kN || (ho.cls && !(sd >> 63))) return;  // one k-mer in class order: heavy_segclass_kernel
    const uint64_t pos = sd & ((1ull << 40) - 1), shard = pos / spill_cap;
    uint64_t dst = pos - shard * spill_cap;
    for (uint64_t t = 0; t < shard; ++t) dst += cursor[t];
    uint32_t N = 1;
    while (N < cnt) N <<= 1;
    const unsigned long long cm = (1ull << ho.cb) - 1, hm = ~((1ull << ho.hshift) - 1);
    for (uint32_t i = threadIdx.x; i < N; i += kThreads) {
        unsigned long long v = ~0ull;  // padding sorts last
        if (i < cnt) {
            v = spill[pos + i];
            if (ho.cls) v = (v & hm) | (v & cm) << ho.pbits | ((v & ~hm) >> ho.cb);
        }
        K[i] = v;
    }
    __syncthreads();
    for (uint32_t k = 2; k <= N; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < N / 2; i += kThreads) {
                const uint32_t lo = 2 * j * (i / j) + (i % j), hi = lo + j;
                const unsigned long long x = K[lo], y = K[hi];
                if ((x > y) == !(lo & k)) {
                    K[lo] = y;
                    K[hi] = x;
                }
            }
            __syncthreads();
        }
    for (uint32_t i = threadIdx.x; i < cnt; i += kThreads) out[dst + i] = K[i];
}

// per tile: distinct (h, p) elements, k-mer heads and (class order) class-run heads
__global__ __launch_bounds__(kHvThreads) void heavy_scan_kernel(const unsigned long long* __restrict__ x, uint64_t m,
                                                                HeavyOrder ho, uint32_t* __restrict__ ecnt,
                                                                uint32_t* __restrict__ gcnt,
                                                                uint32_t* __restrict__ rcnt) {
    __shared__ uint32_t s_e, s_g, s_r;
    if (threadIdx.x == 0) s_e = s_g = s_r = 0;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * kHvTile;
    const unsigned es = ho.eshift();
    uint32_t ne = 0, ng = 0, nr = 0;
    for (uint32_t r = 0; r < kHvPer; ++r) {
        const uint64_t i = t0 + r * kHvThreads + threadIdx.x;
        if (i >= m) break;
        const unsigned long long v = x[i], u = i ? x[i - 1] : ~0ull;
        ne += (v >> es) != (u >> es);
        ng += (v >> ho.hshift) != (u >> ho.hshift);
        nr += (v >> ho.pbits) != (u >> ho.pbits);
    }
    if (ne) atomicAdd(&s_e, ne);
    if (ng) atomicAdd(&s_g, ng);
    if (nr && ho.cls) atomicAdd(&s_r, nr);
    __syncthreads();
    if (threadIdx.x == 0) {
        ecnt[blockIdx.x] = s_e;
        gcnt[blockIdx.x] = s_g;
        if (ho.cls) rcnt[blockIdx.x] = s_r;
    }
}

// per tile: the elements at eoff[t] + their rank, the k-mer starts at goff[t] + rank; class order:
// the class-run starts at roff[t] + rank (RH) and every element's run (RUN)
__global__ __launch_bounds__(kHvThreads) void heavy_compact_kernel(const unsigned long long* __restrict__ x,
                                                                   uint64_t m, HeavyOrder ho,
                                                                   const uint64_t* __restrict__ eoff,
                                                                   const uint64_t* __restrict__ goff,
                                                                   const uint64_t* __restrict__ roff,
                                                                   uint32_t* __restrict__ E,
                                                                   uint64_t* __restrict__ GS,
                                                                   uint32_t* __restrict__ RUN,
                                                                   uint64_t* __restrict__ RH,
                                                                   uint32_t* __restrict__ GH,
                                                                   uint32_t* __restrict__ KG) {
    __shared__ uint32_t wave_tot[kHvThreads / 64];
    const uint64_t t0 = (uint64_t)blockIdx.x * kHvTile;
    uint64_t eb = eoff[blockIdx.x], gb = goff[blockIdx.x], rb = ho.cls ? roff[blockIdx.x] : 0;
    const unsigned es = ho.eshift();
    for (uint32_t r = 0; r < kHvPer; ++r) {
        const uint64_t i = t0 + r * kHvThreads + threadIdx.x;
        bool ke = false, kg = false, kr = false;
        unsigned long long v = 0;
        if (i < m) {
            v = x[i];
            const unsigned long long u = i ? x[i - 1] : ~0ull;
            ke = (v >> es) != (u >> es);
            kg = (v >> ho.hshift) != (u >> ho.hshift);
            kr = (v >> ho.pbits) != (u >> ho.pbits);
        }
        uint32_t xe, te, xg, tg;
        block_scan_n<kHvThreads>(ke, xe, te, wave_tot);
        block_scan_n<kHvThreads>(kg, xg, tg, wave_tot);
        if (ke) E[eb + xe] = ho.elem(v);
        if (ke && KG) KG[eb + xe] = (uint32_t)(gb + xg + kg - 1);  // its k-mer (the last head up to it)
        if (kg) {
            GS[gb + xg] = eb + xe;  // a k-mer head is always a new element
            GH[gb + xg] = (uint32_t)(v >> ho.hshift);  // the k-mer's h (scored calls: its self-score)
        }
        if (ho.cls) {
            uint32_t xr, tr;
            block_scan_n<kHvThreads>(kr, xr, tr, wave_tot);
            if (kr) RH[rb + xr] = eb + xe;  // a run head too
            if (ke) RUN[eb + xe] = (uint32_t)(rb + xr + kr - 1);
            rb += tr;
        }
        eb += te;
        gb += tg;
    }
}

// Row blocks of kHvI elements: k-mer g's blocks are entries [bbase(g), bbase(g) + nblk) of the
// block tables (GS[g] / kHvI + g: disjoint for consecutive k-mers), BT = the k-mer's tiles before
// the block, BP = the block's partner start (its first row's).
__device__ __forceinline__ uint64_t heavy_bbase(uint64_t gs, uint64_t g) { return gs / kHvI + g; }

// a row's partner start (local index): past its class run (class order) or past itself
__device__ __forceinline__ uint32_t heavy_pstart(uint32_t i, uint64_t b, const HeavyOrder& ho,
                                                 const uint32_t* __restrict__ RUN,
                                                 const uint64_t* __restrict__ RH) {
    return ho.cls ? (uint32_t)(RH[RUN[b + i] + 1] - b) : i + 1;
}

// per k-mer: statistics (stats != 0), rows [i0, i1) of the call, the block tables and the tile
// count.  Plain order: the rows whose protein lies in [row_lo, row_hi) (a contiguous range);
// class order: every element (a ranged call tests each pair's smaller protein instead).
__global__ __launch_bounds__(256) void heavy_plan_kernel(const uint32_t* __restrict__ E,
                                                         const uint64_t* __restrict__ GS, uint64_t ngb,
                                                         const unsigned long long* __restrict__ ng_dev,
                                                         HeavyOrder ho, const uint32_t* __restrict__ RUN,
                                                         const uint64_t* __restrict__ RH, int flat_ok,
                                                         uint32_t row_lo, uint32_t row_hi, uint32_t heavy_df,
                                                         int stats, int tiles_on,
                                                         unsigned long long* __restrict__ gstats,
                                                         uint32_t* __restrict__ gi, uint32_t* __restrict__ BT,
                                                         uint32_t* __restrict__ BP,
                                                         unsigned long long* __restrict__ tcount) {
    const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t ng = *ng_dev;  // k-mers; threads up to the bound ngb write empty plans
    const unsigned cb = ho.cb;
    unsigned long long st[kStN] = {0, 0, 0, 0, 0, 0, 0};
    if (g >= ng && g < ngb) {
        if (tiles_on) {
            gi[2 * g] = gi[2 * g + 1] = 0;
            tcount[g] = 0;
        }
    }
    if (g < ng) {
        const uint64_t b = GS[g];
        const uint32_t d = (uint32_t)(GS[g + 1] - b);
        auto lower = [&](uint32_t row) {  // first element whose protein >= row
            uint32_t lo = 0, hi = d;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if ((E[b + mid] >> cb) < row) lo = mid + 1;
                else hi = mid;
            }
            return lo;
        };
        uint32_t i0 = 0, i1 = 0;
        unsigned long long tiles = 0;
        const uint32_t nruns = ho.cls && d ? RUN[b + d - 1] - RUN[b] + 1 : 0u;
        if (!tiles_on) {
            // statistics only
        } else if (d >= 2 && d <= heavy_df && flat_ok && nruns <= kHvFlatRuns) {
            // flat: the k-mer's cross-class pairs as one index space, cut into kHvFlat-pair tiles
            const uint32_t ra = RUN[b];
            unsigned long long pairs = 0;
            for (uint32_t r = 0; r < nruns; ++r) {
                const uint64_t rs = RH[ra + r], re = RH[ra + r + 1];
                pairs += (re - rs) * (b + d - re);
            }
            i0 = kHvFlatMark;
            i1 = nruns;
            tiles = (pairs + kHvFlat - 1) / kHvFlat;
        } else if (d >= 2 && d <= heavy_df) {
            i0 = ho.cls ? 0u : lower(row_lo);
            i1 = ho.cls ? d : lower(row_hi);
            const uint64_t bb = heavy_bbase(b, g);
            for (uint32_t r = i0, k = 0; r < i1; r += kHvI, ++k) {
                const uint32_t ps = heavy_pstart(r, b, ho, RUN, RH);
                BT[bb + k] = (uint32_t)tiles;
                BP[bb + k] = ps;
                tiles += ps < d ? (d - ps + ho.hj - 1) / ho.hj : 0u;
            }
        }
        if (tiles_on) gi[2 * g] = i0;
        if (tiles_on) {
            gi[2 * g + 1] = i1;
            tcount[g] = tiles;
        }
        st[kStSumS] = d;
        st[kStDistinct] = 1;
        st[kStRepeat] = d >= 2;
        if (d <= heavy_df) st[kStCdf2] = (unsigned long long)d * (d - 1) / 2;
        else st[kStHeavy] = d;
        st[kStMaxDf] = d;
    }
    if (!stats) return;
    __shared__ unsigned long long red[4][kStN];
#pragma unroll
    for (int t = 0; t < kStN; ++t) {
        unsigned long long v = st[t];
        for (int s = 32; s > 0; s >>= 1) v = stat_op(t, v, __shfl_down(v, s));
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][t] = v;
    }
    __syncthreads();
    if (threadIdx.x < kStN && threadIdx.x != kStInc) {
        const int t = threadIdx.x;
        unsigned long long v = red[0][t];
        for (int w = 1; w < 4; ++w) v = stat_op(t, v, red[w][t]);
        unsigned long long* gp = gstats + (uint64_t)(blockIdx.x % kShards) * 8 + t;
        if (t == kStMaxDf) atomicMax(gp, v);
        else if (v) atomicAdd(gp, v);
    }
}

// one workgroup per tile (grid-stride): rows i of block k of k-mer g against partner chunk
// [j0, j0 + kHvJ).  Plain order: partners j > i, the class test per pair when require_diff.
// Class order: partners past i's class run (every one of another class); a ranged call keeps the
// pairs whose smaller protein lies in [row_lo, row_hi).  Keys min(p) * mul + max(p).
__global__ __launch_bounds__(kHvI) void heavy_expand_kernel(const uint32_t* __restrict__ E,
                                                            const uint64_t* __restrict__ GS,
                                                            const uint32_t* __restrict__ gi,
                                                            const uint32_t* __restrict__ BT,
                                                            const uint32_t* __restrict__ BP,
                                                            const uint32_t* __restrict__ RUN,
                                                            const uint64_t* __restrict__ RH,
                                                            const unsigned long long* __restrict__ toff,
                                                            const unsigned long long* __restrict__ ng_dev,
                                                            HeavyOrder ho, uint32_t mul, int require_diff, int ranged,
                                                            uint32_t row_lo, uint32_t row_hi,
                                                            unsigned long long* __restrict__ out, uint64_t shard_cap,
                                                            unsigned long long* __restrict__ cursor,
                                                            unsigned long long* __restrict__ gstats,
                                                            const uint32_t* __restrict__ GH, int k, unsigned sb,
                                                            uint32_t sor) {
    __shared__ uint32_t J[kHvJ];
    __shared__ uint32_t s_ex[kHvI + 1], s_js[kHvI], s_p[kHvI];
    __shared__ uint32_t s_m[kHvI * kHvMW];  // filtered tile: each row's kept partners (bit j - j0)
    __shared__ unsigned long long s_sb[kShards];  // spread tile: shard base minus its first output
    __shared__ uint32_t f_s[kHvFlatRuns], f_e[kHvFlatRuns];  // flat tile: the k-mer's runs (local)
    __shared__ unsigned long long f_c[kHvFlatRuns + 1];       // ... and their first pair's index
    __shared__ uint32_t wave_tot[kHvI / 64];
    __shared__ unsigned long long sbase;
    const uint64_t ng = *ng_dev;
    const unsigned long long T = toff[ng];
    const unsigned cb = ho.cb;
    const uint32_t cmask = (1u << cb) - 1;
    const bool test_cls = require_diff && !ho.cls, test_row = ho.cls && ranged;
    // workgroup w takes the consecutive tiles [w * per, (w + 1) * per): one binary search for its
    // first tile's k-mer, then the k-mer and row block advance (a search per tile was a chain of
    // ~15 dependent loads, the bulk of a tile's time)
    const unsigned long long per = (T + gridDim.x - 1) / gridDim.x, tb = blockIdx.x * per;
    const unsigned long long te = min(T, tb + per);
    uint64_t g = 0;
    if (tb < te) {
        uint64_t lo = 0, hi = ng;  // the last k-mer with toff[g] <= tb
        while (lo + 1 < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (toff[mid] <= tb) lo = mid;
            else hi = mid;
        }
        g = lo;
    }
    uint32_t klo = 0;
    for (unsigned long long t = tb; t < te; ++t) {
        if (toff[g + 1] <= t) {  // the next k-mer with tiles (toff[ng] = T > t)
            do ++g;
            while (toff[g + 1] <= t);
            klo = 0;
        }
        const uint64_t b = GS[g];
        const uint32_t d = (uint32_t)(GS[g + 1] - b), i0 = gi[2 * g], i1 = gi[2 * g + 1];
        const uint32_t local = (uint32_t)(t - toff[g]);
        // pair key; scored (sb > 0): (pair << sb) | sor | s(x) of this k-mer
        const uint32_t sfield = sb ? sor | kmer_self_score(GH[g], k) : 0u;
        auto mk = [&](uint32_t pa, uint32_t pb) {
            return ((unsigned long long)min(pa, pb) * mul + max(pa, pb)) << sb | sfield;
        };
        if (i0 == kHvFlatMark) {  // flat tile (uniform over the workgroup)
            const uint32_t nr = i1, ra = RUN[b];
            __syncthreads();  // the run table's reuse
            unsigned long long pr = 0;
            if (threadIdx.x < nr) {
                const uint32_t rs = (uint32_t)(RH[ra + threadIdx.x] - b), re = (uint32_t)(RH[ra + threadIdx.x + 1] - b);
                f_s[threadIdx.x] = rs;
                f_e[threadIdx.x] = re;
                pr = (unsigned long long)(re - rs) * (d - re);
            }
            if (threadIdx.x < 64) {  // exclusive scan of the runs' pair counts (nr <= 64: one wave)
                unsigned long long incl = pr;
                for (int sh = 1; sh < 64; sh <<= 1) {
                    const unsigned long long y = __shfl_up(incl, sh);
                    if ((int)threadIdx.x >= sh) incl += y;
                }
                if (threadIdx.x < nr) f_c[threadIdx.x] = incl - pr;
                if (threadIdx.x == nr - 1) f_c[nr] = incl;
            }
            __syncthreads();
            const unsigned long long o0 = (unsigned long long)local * kHvFlat, o1 = min(f_c[nr], o0 + kHvFlat);
            const uint32_t total = (uint32_t)(o1 - o0);
            uint32_t hx = (GH[g] * 0x9E3779B1u) ^ (local * 0xC2B2AE35u) ^ 0x27D4EB2Fu;
            hx ^= hx >> 16;
            const uint32_t shard = (hx * 0x7FEB352Du) >> 26;
            if (threadIdx.x == 0) {
                sbase = atomicAdd(&cursor[shard], (unsigned long long)total);
                atomicAdd(&gstats[(uint64_t)shard * 8 + kStInc], (unsigned long long)total);
            }
            __syncthreads();
            unsigned long long* dst = out + (uint64_t)shard * shard_cap;
            for (uint32_t u = threadIdx.x; u < total; u += kHvI) {
                const unsigned long long o = o0 + u;
                uint32_t r = 0, hi = nr;  // the last run with f_c[r] <= o
                while (r + 1 < hi) {
                    const uint32_t mid = (r + hi) >> 1;
                    if (f_c[mid] <= o) r = mid;
                    else hi = mid;
                }
                const unsigned long long off = o - f_c[r];
                const uint32_t part = d - f_e[r];
                const uint32_t row = f_s[r] + (uint32_t)(off / part), j = f_e[r] + (uint32_t)(off % part);
                const uint32_t pa = E[b + row] >> cb, pj = E[b + j] >> cb;
                const unsigned long long pos = sbase + u;
                if (pos < shard_cap) dst[pos] = mk(pa, pj);
            }
            continue;
        }
        // row block: the last with BT <= local (blocks without tiles share the next one's BT)
        const uint64_t bb = heavy_bbase(b, g);
        const uint32_t nblk = (i1 - i0 + kHvI - 1) / kHvI;
        if (t == tb) {  // entered mid-k-mer: search
            uint32_t khi = nblk;
            while (klo + 1 < khi) {
                const uint32_t mid = (klo + khi) >> 1;
                if (BT[bb + mid] <= local) klo = mid;
                else khi = mid;
            }
        }
        while (klo + 1 < nblk && BT[bb + klo + 1] <= local) ++klo;
        const uint32_t r = i0 + klo * kHvI;
        const uint32_t j0 = BP[bb + klo] + (local - BT[bb + klo]) * ho.hj, j1 = min(d, j0 + ho.hj);
        __syncthreads();  // J reuse
        for (uint32_t j = j0 + threadIdx.x; j < j1; j += kHvI) J[j - j0] = E[b + j];
        const uint32_t i = r + threadIdx.x;
        const bool row = i < i1;
        const uint32_t xi = row ? E[b + i] : 0u;
        const uint32_t js = row ? max(heavy_pstart(i, b, ho, RUN, RH), j0) : j1;
        const uint32_t pi = xi >> cb;
        __syncthreads();
        auto keep = [&](uint32_t xj) {
            if (test_cls) return ((xj ^ xi) & cmask) != 0u;
            if (test_row) {
                const uint32_t pm = min(pi, xj >> cb);
                return pm >= row_lo && pm < row_hi;
            }
            return true;
        };
        uint32_t c = 0;
        if (test_cls || test_row) {
            // the row's kept partners as a bit mask over the chunk (hj <= kHvJ): the emit below
            // writes the tile's output coalesced (a row writing its own run, one lane per row, cost
            // one memory transaction per key)
            uint32_t* mrow = s_m + threadIdx.x * kHvMW;
#pragma unroll
            for (uint32_t w = 0; w < kHvMW; ++w) {
                uint32_t bits = 0;
                const uint32_t jw = j0 + w * 32;
                if (jw < j1 && jw + 32 > js)
                    for (uint32_t t = 0; t < 32; ++t) {
                        const uint32_t j = jw + t;
                        if (j >= js && j < j1 && keep(J[j - j0])) bits |= 1u << t;
                    }
                mrow[w] = bits;
                c += __popc(bits);
            }
        } else {
            c = js < j1 ? j1 - js : 0u;
        }
        uint32_t excl, total;
        block_scan_n<kHvI>(c, excl, total, wave_tot);
        // Shards, which size the next call's regions: a large unfiltered tile spreads its output
        // evenly over all of them (output o in shard 64 o / total); another tile takes one shard from
        // what it is (its k-mer's h, block, chunk) — not from t: the k-mers' order in E
        // follows the spill's (atomic) order, and the shard loads must not
        const bool spread = !(test_cls || test_row) && total >= kHvSpread;
        // the k-mer's h, not its first element: class runs come in LDS-atomic order
        // (heavy_segclass), so E[b] varied between calls and so did the fullest region (8 %)
        uint32_t hx = (GH[g] * 0x9E3779B1u) ^ (klo * 0x85EBCA6Bu) ^ (local * 0xC2B2AE35u);
        hx ^= hx >> 16;
        const uint32_t shard = (hx * 0x7FEB352Du) >> 26;  // the top bits: kShards = 64
        if (spread) {
            if (threadIdx.x < kShards) {
                const uint32_t sh = threadIdx.x;
                const uint64_t a0 = ((uint64_t)sh * total + kShards - 1) / kShards;
                const uint64_t a1 = ((uint64_t)(sh + 1) * total + kShards - 1) / kShards;
                s_sb[sh] = atomicAdd(&cursor[sh], (unsigned long long)(a1 - a0)) - a0;  // pos = s_sb + o
                if (a1 > a0) atomicAdd(&gstats[(uint64_t)sh * 8 + kStInc], (unsigned long long)(a1 - a0));
            }
        } else if (threadIdx.x == 0) {
            sbase = total ? atomicAdd(&cursor[shard], (unsigned long long)total) : 0ull;
            if (total) atomicAdd(&gstats[(uint64_t)shard * 8 + kStInc], (unsigned long long)total);
        }
        __syncthreads();
        unsigned long long* dst = out + (uint64_t)shard * shard_cap;
        if (test_cls || test_row) {
            // filtered tile: output o of row i (the last with s_ex[i] <= o) is the row's
            // (o - s_ex[i])-th kept partner, selected from its mask; consecutive lanes write
            // consecutive keys
            s_ex[threadIdx.x] = excl;
            s_p[threadIdx.x] = pi;
            if (threadIdx.x == 0) s_ex[kHvI] = total;
            __syncthreads();
            uint32_t i = 0, hi = kHvI;
            if (threadIdx.x < total) {
                while (i + 1 < hi) {
                    const uint32_t mid = (i + hi) >> 1;
                    if (s_ex[mid] <= threadIdx.x) i = mid;
                    else hi = mid;
                }
            }
            for (uint32_t o = threadIdx.x; o < total; o += kHvI) {
                while (s_ex[i + 1] <= o) ++i;
                uint32_t rk = o - s_ex[i], w = 0, x = s_m[i * kHvMW];
                while (rk >= (uint32_t)__popc(x)) {  // the word holding it
                    rk -= __popc(x);
                    x = s_m[i * kHvMW + ++w];
                }
                uint32_t bit = 0;  // the rk-th set bit of x
                for (uint32_t half = 16; half; half >>= 1) {
                    const uint32_t low = __popc(x & ((1u << half) - 1));
                    if (rk >= low) {
                        rk -= low;
                        x >>= half;
                        bit += half;
                    }
                }
                const uint32_t pj = J[w * 32 + bit] >> cb;
                const unsigned long long pos = sbase + o;
                if (pos < shard_cap) dst[pos] = mk(s_p[i], pj);
            }
        } else {
            // every partner kept: the tile's output [0, total) in coalesced order, output o of row
            // i (the last with s_ex[i] <= o) = partner js_i + o - s_ex[i]; a thread's rows only move
            // forward as o grows
            s_ex[threadIdx.x] = excl;
            s_js[threadIdx.x] = js;
            s_p[threadIdx.x] = pi;
            if (threadIdx.x == 0) s_ex[kHvI] = total;
            __syncthreads();
            uint32_t i = 0, hi = kHvI;
            if (threadIdx.x < total) {
                while (i + 1 < hi) {
                    const uint32_t mid = (i + hi) >> 1;
                    if (s_ex[mid] <= threadIdx.x) i = mid;
                    else hi = mid;
                }
            }
            // spread: output o's shard sh = 64 o / total, advanced as o grows (total < 2^26)
            uint32_t sh = spread ? threadIdx.x * kShards / total : 0u;
            uint32_t sh_end = spread ? ((sh + 1) * total + kShards - 1) / kShards : 0u;
            for (uint32_t o = threadIdx.x; o < total; o += kHvI) {
                while (s_ex[i + 1] <= o) ++i;
                const uint32_t pa = s_p[i], pj = J[s_js[i] + (o - s_ex[i]) - j0] >> cb;
                const unsigned long long key = mk(pa, pj);
                if (spread) {
                    while (o >= sh_end) {
                        ++sh;
                        sh_end = ((sh + 1) * total + kShards - 1) / kShards;
                    }
                    const unsigned long long pos = s_sb[sh] + o;
                    if (pos < shard_cap) out[(uint64_t)sh * shard_cap + pos] = key;
                } else {
                    const unsigned long long pos = sbase + o;
                    if (pos < shard_cap) dst[pos] = key;
                }
            }
        }
    }
}

// Ranged calls in plain order (the passes of a streamed batch): the rows of a pass, not its
// k-mers, drive the expansion.  A per-protein index of the compacted elements (PE: element
// indices grouped by protein, PO: each protein's start; built once per compaction) makes a pass's
// active elements the contiguous range PE[PO[row_lo], PO[row_hi]); each pairs with the later
// elements of its k-mer (E is sorted by protein within a k-mer, so every partner's protein is
// larger: the pair's smaller protein is the active row).  One workgroup per 256 active elements:
// their candidate counts scanned in LDS, the candidates split into one contiguous slice per wave,
// the class test counted (pass 1), one cursor reservation for the workgroup, and the kept keys
// written compacted by ballot (pass 2; consecutive lanes read consecutive partners).  No per-k-mer
// plan, tile table or search: the work is the pass's own pairs.
constexpr uint32_t kHfThreads = 256, kHfWaves = kHfThreads / 64;
__global__ __launch_bounds__(kHfThreads) void heavy_flat_kernel(
        const uint32_t* __restrict__ E, const uint64_t* __restrict__ GS, const uint32_t* __restrict__ KG,
        const uint32_t* __restrict__ GH, const uint32_t* __restrict__ PE, uint32_t a0, uint32_t a1, unsigned cb,
        uint32_t mul, int require_diff, uint32_t heavy_df, int k, unsigned sb, uint32_t sor,
        unsigned long long* __restrict__ out, uint64_t shard_cap, unsigned long long* __restrict__ cursor,
        unsigned long long* __restrict__ gstats) {
    __shared__ uint32_t s_ex[kHfThreads + 1], s_e[kHfThreads], s_x[kHfThreads], s_f[kHfThreads];
    __shared__ uint32_t wave_tot[kHfWaves], s_wk[kHfWaves];
    __shared__ unsigned long long s_base;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t a = a0 + blockIdx.x * kHfThreads + tid;
    uint32_t cand = 0, e = 0, x = 0, f = 0;
    if (a < a1) {
        e = PE[a];
        const uint32_t g = KG[e];
        const uint64_t gs0 = GS[g], gs1 = GS[g + 1];
        x = E[e];
        if (gs1 - gs0 <= heavy_df) cand = (uint32_t)(gs1 - e - 1);
        f = sb ? sor | kmer_self_score(GH[g], k) : 0u;
    }
    uint32_t ex, total;
    block_scan_n<kHfThreads>(cand, ex, total, wave_tot);
    s_ex[tid] = ex;
    s_e[tid] = e;
    s_x[tid] = x;
    s_f[tid] = f;
    if (tid == 0) s_ex[kHfThreads] = total;
    __syncthreads();
    if (total == 0) return;  // (uniform)
    const uint32_t S = (total + kHfWaves - 1) / kHfWaves;
    const uint32_t c0 = min(total, wv * S), c1 = min(total, c0 + S);
    const uint32_t cmask = (1u << cb) - 1;
    auto search = [&](uint32_t o) {  // the last row with s_ex[i] <= o (o < total: a row with candidates)
        uint32_t lo = 0, hi = kHfThreads;
        while (lo + 1 < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_ex[mid] <= o) lo = mid;
            else hi = mid;
        }
        return lo;
    };
    uint32_t kept = 0;
    if (require_diff) {
        uint32_t i = c0 + lane < c1 ? search(c0 + lane) : 0u;
        for (uint32_t o = c0 + lane; o < c1; o += 64) {
            while (s_ex[i + 1] <= o) ++i;
            const uint32_t j = s_e[i] + 1 + (o - s_ex[i]);
            kept += ((E[j] ^ s_x[i]) & cmask) != 0u;
        }
        kept = wave_sum(kept);
    } else {
        kept = c1 - c0;
    }
    if (lane == 0) s_wk[wv] = kept;
    __syncthreads();
    uint32_t before = 0, K = 0;
#pragma unroll
    for (uint32_t w = 0; w < kHfWaves; ++w) {
        before += w < wv ? s_wk[w] : 0u;
        K += s_wk[w];
    }
    uint32_t hx = (blockIdx.x * 0x9E3779B1u) ^ (a0 * 0x85EBCA6Bu);
    hx ^= hx >> 16;
    const uint32_t shard = (hx * 0x7FEB352Du) >> 26;
    if (tid == 0) {
        s_base = K ? atomicAdd(&cursor[shard], (unsigned long long)K) : 0ull;
        if (K) atomicAdd(&gstats[(uint64_t)shard * 8 + kStInc], (unsigned long long)K);
    }
    __syncthreads();
    unsigned long long* dst = out + (uint64_t)shard * shard_cap;
    uint64_t run = s_base + before;
    uint32_t i = c0 + lane < c1 ? search(c0 + lane) : 0u;
    for (uint32_t o0 = c0; o0 < c1; o0 += 64) {  // uniform over the wave (ballot)
        const uint32_t o = o0 + lane;
        bool keep = false;
        unsigned long long key = 0;
        if (o < c1) {
            while (s_ex[i + 1] <= o) ++i;
            const uint32_t j = s_e[i] + 1 + (o - s_ex[i]), xj = E[j], xi = s_x[i];
            keep = !require_diff || ((xj ^ xi) & cmask) != 0u;
            key = ((unsigned long long)(xi >> cb) * mul + (xj >> cb)) << sb | s_f[i];
        }
        const unsigned long long m = __ballot(keep);
        if (keep) {
            const uint64_t pos = run + __popcll(m & ((1ull << lane) - 1));
            if (pos < shard_cap) dst[pos] = key;
        }
        run += __popcll(m);
    }
}

// per-protein index of the compacted elements: counts, then (after a scan into PO) the scatter
__global__ void heavy_pcount_kernel(const uint32_t* __restrict__ E, const unsigned long long* __restrict__ tot,
                                    unsigned cb, uint32_t* __restrict__ cnt) {
    const uint64_t ne = tot[0];
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < ne; e += (uint64_t)gridDim.x * blockDim.x)
        atomicAdd(&cnt[E[e] >> cb], 1u);
}
__global__ void heavy_pscatter_kernel(const uint32_t* __restrict__ E, const unsigned long long* __restrict__ tot,
                                      unsigned cb, const uint32_t* __restrict__ PO, uint32_t* __restrict__ cur,
                                      uint32_t* __restrict__ PE) {
    const uint64_t ne = tot[0];
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < ne; e += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t p = E[e] >> cb;
        PE[PO[p] + atomicAdd(&cur[p], 1u)] = (uint32_t)e;
    }
}

// bucket kernels: capacity (keys), threads, log2 of the k-mer table (>= capacity)
#ifndef KMP_SMALL_GEOM
#define KMP_SMALL_GEOM 1280, 256, 11
#endif
constexpr int kSmallGeom[3] = {KMP_SMALL_GEOM};
constexpr int kBucketSmallCap = kSmallGeom[0], kBucketSmallThreads = kSmallGeom[1], kBucketSmallTab = kSmallGeom[2];
// larger buckets (up to 4,096 keys: four per thread, no register spills) take the large kernel;
// above that the whole bucket goes to the heavy path
constexpr int kBucketLargeCap = 4096, kBucketLargeThreads = 1024, kBucketLargeTab = 12;
// the large kernel grid-strides the list of large buckets (usually empty at config 3; most
// buckets of a k = 5 batch of real proteins): four workgroups per CU (one per CU measured 8 % slower)
constexpr int kBucketLargeGrid = 1024;
#ifndef KMP_VREG_TRIES
#define KMP_VREG_TRIES 3
#endif
constexpr uint32_t kVregTries = KMP_VREG_TRIES;  // learned bucket layouts in a row before the counting partition

// ------------------------------------------------------------- bucket partition ------------
// The residue path groups its keys by bucket (the top bbits of h) with two counting passes
// instead of materialising every key and radix sorting it (0.09 ms of key writes + 0.46 ms of
// onesweep at config 3): bucket = digit1 (high d1 bits) : digit2 (low d2 bits).
//   level 1 (bp_hist1 -> column scan -> bp_scatter1): each 4,096-slot key chunk computes its keys
//     from the residues twice, once to count them per digit1 and once to write them, ranked in
//     LDS, as one contiguous run per digit1 at the offset the column scan gave that (digit, chunk);
//     padding slots are dropped.  Output: keys grouped by digit1 ("coarse bins"), in ws->keys.
//   level 2 (bp_hist2 -> per-coarse-bin scan -> bp_scatter2): 4,096-key tiles of each coarse bin,
//     counted and scattered the same way on digit2.  Output: keys grouped by bucket, in
//     ws->sorted, and bstart[] for the bucket kernels straight from the scan.
// Order inside a bucket is unspecified (LDS atomics rank the keys); the bucket kernel does not
// need one.  A coarse bin above its tile budget (a k-mer with ~10^5 copies) raises flags[0] and
// records the tiles it needs in flags[4]; the step reruns with that budget.
constexpr uint32_t kBpTile = 4096;            // level-2 tile (level 1 uses the key chunk, also 4,096)
constexpr uint32_t kBpPer = kBpTile / kKeyThreads;
constexpr uint32_t kBpMaxBins = 1024;         // digit widths <= 10 bits
constexpr uint32_t kBpRowGroup = 64;          // rows per partial sum of the level-1 column scan
constexpr uint32_t kBpAlign = 16;             // coarse bins start on 128-B lines of the level-1 array
static_assert(kKeyChunk == kBpTile, "one tile geometry for both levels");

struct BpDigits {
    unsigned sh1, sh2;   // digit1 = x >> sh1; digit2 = (x >> sh2) & m2
    uint32_t nb1, nb2, m2;
};

BpDigits bp_digits(const Layout& lay) {
    BpDigits d{};
    const unsigned d2 = lay.bbits / 2, d1 = lay.bbits - d2;
    d.sh2 = lay.sort_lo;
    d.sh1 = lay.sort_lo + d2;
    d.nb1 = 1u << d1;
    d.nb2 = 1u << d2;
    d.m2 = d.nb2 - 1;
    return d;
}


// sum of x[i * stride], i < m, with the loads issued in batches of 8 (an accumulation loop would
// otherwise wait on every load in turn)
__device__ __forceinline__ uint32_t col_sum(const uint32_t* __restrict__ x, uint64_t stride, uint32_t m) {
    uint32_t s = 0;
    for (uint32_t i = 0; i < m; i += 8) {
        uint32_t v[8];
#pragma unroll
        for (uint32_t t = 0; t < 8; ++t) v[t] = i + t < m ? x[(i + t) * stride] : 0u;
#pragma unroll
        for (uint32_t t = 0; t < 8; ++t) s += v[t];
    }
    return s;
}

// in place: x[i * stride] <- run + (exclusive prefix of x[0 .. i)), for i < m; returns the end
// value.  Loads go out in batches of 8 ahead of the stores (the in-place stores would otherwise
// serialise every load behind the previous store).
__device__ __forceinline__ uint32_t col_prefix_inplace(uint32_t* __restrict__ x, uint64_t stride, uint32_t m,
                                                       uint32_t run) {
    for (uint32_t i = 0; i < m; i += 8) {
        uint32_t v[8];
#pragma unroll
        for (uint32_t t = 0; t < 8; ++t) v[t] = i + t < m ? x[(i + t) * stride] : 0u;
#pragma unroll
        for (uint32_t t = 0; t < 8; ++t)
            if (i + t < m) {
                x[(i + t) * stride] = run;
                run += v[t];
            }
    }
    return run;
}

// level 1, pass 1: per-chunk digit1 histogram -> H1[chunk][digit]
__global__ __launch_bounds__(kKeyThreads) void bp_hist1_kernel(
    const uint8_t* __restrict__ res, const uint64_t* __restrict__ res_off, const uint16_t* __restrict__ cls, int k,
    uint32_t p_hi, uint64_t slots, const uint32_t* __restrict__ chunk_first, Layout lay, BpDigits dg, uint32_t pw21,
    uint32_t dlo, uint32_t dhi, uint32_t* __restrict__ H1, uint32_t* __restrict__ flags) {
    __shared__ KeyChunk s;
    __shared__ uint32_t lh[kBpMaxBins];
    const uint64_t c0 = (uint64_t)blockIdx.x * kKeyChunk, c1 = min(c0 + kKeyChunk, slots);
    for (uint32_t d = threadIdx.x; d < dg.nb1; d += kKeyThreads) lh[d] = 0;
    const uint32_t first = chunk_first[blockIdx.x];
    key_chunk_load(s, res, res_off, cls, k, p_hi, c0, c1, first, lay, flags);
    const unsigned hs1 = dg.sh1 - lay.hshift;  // digit1 = the top d1 bits of h
    key_chunk_run<kBpPer>(s, threadIdx.x * kBpPer, (uint32_t)(c1 - c0), k, pw21, first, lay,
                          [&](uint32_t, bool valid, uint32_t h, unsigned long long) {
                              const uint32_t d = h >> hs1;
                              if (valid && d >= dlo && d < dhi) atomicAdd(&lh[d], 1u);
                          });
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < dg.nb1; d += kKeyThreads) H1[(uint64_t)blockIdx.x * dg.nb1 + d] = lh[d];
}

// column scan of a [rows][cols] count matrix, 1 of 3: R[g][c] = sum of M[r][c] over the
// kBpRowGroup rows of group g (grid: groups x ceil(cols / 256))
__global__ __launch_bounds__(256) void bp_colsum_kernel(const uint32_t* __restrict__ M, uint32_t rows, uint32_t cols,
                                                        uint32_t* __restrict__ R) {
    const uint32_t r0 = blockIdx.x * kBpRowGroup, r1 = min(rows, r0 + kBpRowGroup);
    for (uint32_t c = blockIdx.y * 256 + threadIdx.x; c < cols; c += gridDim.y * 256) {
        R[(uint64_t)blockIdx.x * cols + c] = col_sum(M + (uint64_t)r0 * cols + c, cols, r1 - r0);
    }
}

// 2 of 3 (one workgroup): per column an exclusive scan down the groups; the column totals
// scanned across columns twice: rounded up to kBpAlign keys -> colstart[c] (where column c's run
// starts in the level-1 array, added to every R[g][c]) and exact -> colstart[cols + 1 + c]
// (compact starts; [cols] and [2 cols + 1] are the grand totals).
// cols is a power of two <= 1024; each column's groups are split over 1024 / cols threads.
constexpr int kColThreads = 1024;
__global__ __launch_bounds__(kColThreads) void bp_colscan_kernel(uint32_t* __restrict__ R, uint32_t groups,
                                                                 uint32_t cols, uint32_t* __restrict__ colstart) {
    __shared__ uint32_t part[kColThreads];
    __shared__ uint32_t tot[kBpMaxBins], cmp[kBpMaxBins];
    __shared__ uint32_t wave_tot[kColThreads / 64];
    const uint32_t splits = max(1u, kColThreads / cols);
    const uint32_t c = threadIdx.x % cols, sp = threadIdx.x / cols;
    const bool act = sp < splits;
    const uint32_t gq = (groups + splits - 1) / splits, g0 = min(groups, sp * gq), g1 = min(groups, g0 + gq);
    const uint32_t v = act ? col_sum(R + (uint64_t)g0 * cols + c, cols, g1 - g0) : 0u;
    part[threadIdx.x] = v;
    __syncthreads();
    uint32_t before = 0;  // this split's offset inside its column
    if (act) {
        uint32_t t = 0;
        for (uint32_t s = 0; s < splits; ++s) {
            const uint32_t y = part[s * cols + c];
            before += s < sp ? y : 0u;
            t += y;
        }
        if (sp == 0) {
            tot[c] = (t + kBpAlign - 1) & ~(kBpAlign - 1);
            cmp[c] = t;
        }
    }
    __syncthreads();
    uint32_t last = 0, last_c = 0;
    if (threadIdx.x == 0) {
        last = tot[cols - 1];
        last_c = cmp[cols - 1];
    }
    lds_bins_scan<kColThreads>(tot, cols, wave_tot);
    lds_bins_scan<kColThreads>(cmp, cols, wave_tot);
    if (act) {
        if (sp == 0) {
            colstart[c] = tot[c];
            colstart[cols + 1 + c] = cmp[c];
        }
        col_prefix_inplace(R + (uint64_t)g0 * cols + c, cols, g1 - g0, tot[c] + before);
    }
    if (threadIdx.x == 0) {
        colstart[cols] = tot[cols - 1] + last;
        colstart[2 * cols + 1] = cmp[cols - 1] + last_c;
    }
}

// 3 of 3: P[r][c] = R[group(r)][c] + the rows of the group before r
__global__ __launch_bounds__(256) void bp_colprefix_kernel(const uint32_t* __restrict__ M, uint32_t rows,
                                                           uint32_t cols, const uint32_t* __restrict__ R,
                                                           uint32_t* __restrict__ P) {
    const uint32_t r0 = blockIdx.x * kBpRowGroup, r1 = min(rows, r0 + kBpRowGroup);
    for (uint32_t c = blockIdx.y * 256 + threadIdx.x; c < cols; c += gridDim.y * 256) {
        uint32_t run = R[(uint64_t)blockIdx.x * cols + c];
#pragma unroll 8
        for (uint32_t r = r0; r < r1; ++r) {
            P[(uint64_t)r * cols + c] = run;
            run += M[(uint64_t)r * cols + c];
        }
    }
}

// the tile's row of run offsets (P1 / P2), digit tid + t * kKeyThreads in pre[t]: loaded at the
// start of the scatter kernels so the load's latency hides behind the tile's own work (loaded
// where it was used, after the tile scan, every workgroup waited on it)
constexpr uint32_t kBpQ = kBpMaxBins / kKeyThreads;
__device__ __forceinline__ void bp_prow_load(const uint32_t* __restrict__ prow, uint32_t nb, uint32_t (&pre)[kBpQ]) {
#pragma unroll
    for (uint32_t t = 0; t < kBpQ; ++t) {
        const uint32_t d = threadIdx.x + t * kKeyThreads;
        pre[t] = d < nb ? prow[d] : 0u;
    }
}

// rank every key of the workgroup's tile by digit in LDS (x[e] = element tid + e*kKeyThreads),
// place the tile digit-major into S and write each digit's run at base[digit] (global offset of
// the tile's run, from the scan; pre = bp_prow_load of it).  lh holds the tile histogram on
// entry (zeroed, then counted by the caller's ranks); shared by both scatter levels.
template <class Digit>
__device__ __forceinline__ void bp_place(const unsigned long long (&x)[kBpPer], const uint32_t (&r)[kBpPer],
                                         uint32_t n_in, uint32_t nb, Digit digit, uint32_t* lh, uint32_t* wave_tot,
                                         unsigned long long* S, const uint32_t (&pre)[kBpQ],
                                         unsigned long long* __restrict__ out) {
    lds_bins_scan(lh, nb, wave_tot);
#pragma unroll
    for (uint32_t e = 0; e < kBpPer; ++e)
        if (x[e] != kNoKey) S[lh[digit(x[e])] + r[e]] = x[e];
    __syncthreads();
    // lh[d] -> global base of the digit's run minus its tile start: out[lh[d] + i] for S[i]
#pragma unroll
    for (uint32_t t = 0; t < kBpQ; ++t) {
        const uint32_t d = threadIdx.x + t * kKeyThreads;
        if (d < nb) lh[d] = pre[t] - lh[d];
    }
    __syncthreads();
    // pairs (i, i+1), i even: one 16-byte store when both keys belong to the same run and its
    // destination is 16-byte aligned (S is 16-byte aligned, i even), else two 8-byte stores
    for (uint32_t i = 2 * threadIdx.x; i < n_in; i += 2 * kKeyThreads) {
        if (i + 1 < n_in) {
            const ulonglong2 y = *reinterpret_cast<const ulonglong2*>(S + i);
            const uint32_t d0 = digit(y.x), d1 = digit(y.y);
            const uint64_t a0 = (uint64_t)lh[d0] + i;
            if (d0 == d1 && !(a0 & 1)) {
                *reinterpret_cast<ulonglong2*>(out + a0) = y;
            } else {
                out[a0] = y.x;
                out[(uint64_t)lh[d1] + i + 1] = y.y;
            }
        } else {
            const unsigned long long y = S[i];
            out[lh[digit(y)] + i] = y;
        }
    }
}

// level 1, pass 2: the chunk's keys again, grouped by digit1 at P1[chunk][digit]
__global__ __launch_bounds__(kKeyThreads) void bp_scatter1_kernel(
    const uint8_t* __restrict__ res, const uint64_t* __restrict__ res_off, const uint16_t* __restrict__ cls, int k,
    uint32_t p_hi, uint64_t slots, const uint32_t* __restrict__ chunk_first, Layout lay, BpDigits dg, uint32_t pw21,
    uint32_t dlo, uint32_t dhi, const uint32_t* __restrict__ P1, unsigned long long* __restrict__ out,
    uint32_t* __restrict__ flags) {
    __shared__ union {
        KeyChunk kc;
        unsigned long long S[kKeyChunk];
    } u;
    __shared__ uint32_t lh[kBpMaxBins];
    __shared__ uint32_t wave_tot[kKeyThreads / 64];
    __shared__ uint32_t s_n;
    const uint64_t c0 = (uint64_t)blockIdx.x * kKeyChunk, c1 = min(c0 + kKeyChunk, slots);
    uint32_t pre[kBpQ];
    bp_prow_load(P1 + (uint64_t)blockIdx.x * dg.nb1, dg.nb1, pre);
    for (uint32_t d = threadIdx.x; d < dg.nb1; d += kKeyThreads) lh[d] = 0;
    if (threadIdx.x == 0) s_n = 0;
    const uint32_t first = chunk_first[blockIdx.x];
    key_chunk_load(u.kc, res, res_off, cls, k, p_hi, c0, c1, first, lay, flags);
    unsigned long long x[kBpPer];
    uint32_t r[kBpPer], nk = 0;
    auto digit = [&](unsigned long long y) { return (uint32_t)(y >> dg.sh1); };
    const unsigned hs1 = dg.sh1 - lay.hshift;
    key_chunk_run<kBpPer>(u.kc, threadIdx.x * kBpPer, (uint32_t)(c1 - c0), k, pw21, first, lay,
                          [&](uint32_t e, bool valid, uint32_t h, unsigned long long lo) {
                              const uint32_t d = h >> hs1;
                              const bool mine = valid && d >= dlo && d < dhi;  // the call's coarse bins
                              x[e] = mine ? ((unsigned long long)h << lay.hshift) | lo : kNoKey;
                              r[e] = mine ? atomicAdd(&lh[d], 1u) : 0u;
                              nk += mine;
                          });
    if (nk) atomicAdd(&s_n, nk);
    __syncthreads();  // the chunk's staging (u.kc) is dead from here: u.S reuses it
    bp_place(x, r, s_n, dg.nb1, digit, lh, wave_tot, u.S, pre, out);
}

// level-2 tile (j, c) of coarse bin c: keys [a + j*kBpTile, a + min(n, (j+1)*kBpTile)) of the
// level-1 array, a = C1[c] (aligned start), n = the bin's key count (compact starts C1[nb1+1+c]);
// false past the bin's last tile, and for every tile of a bin above its budget of J tiles
__device__ __forceinline__ bool bp_tile(const uint32_t* __restrict__ C1, uint32_t nb1, uint32_t c, uint32_t j,
                                        uint32_t J, uint32_t& t0, uint32_t& tn) {
    const uint32_t n = C1[nb1 + 2 + c] - C1[nb1 + 1 + c];
    if (n > J * kBpTile || j * kBpTile >= n) return false;
    t0 = C1[c] + j * kBpTile;
    tn = min(kBpTile, n - j * kBpTile);
    return true;
}

// level 2, pass 1: per-tile digit2 histogram -> H2[c][j][digit]
__global__ __launch_bounds__(kKeyThreads) void bp_hist2_kernel(const unsigned long long* __restrict__ in,
                                                               const uint32_t* __restrict__ C1, uint32_t J,
                                                               BpDigits dg, uint32_t* __restrict__ H2,
                                                               uint32_t c0) {
    __shared__ uint32_t lh[kBpMaxBins];
    const uint32_t j = blockIdx.x, c = c0 + blockIdx.y;
    uint32_t t0, tn;
    if (!bp_tile(C1, dg.nb1, c, j, J, t0, tn)) return;
    for (uint32_t d = threadIdx.x; d < dg.nb2; d += kKeyThreads) lh[d] = 0;
    __syncthreads();
    // t0 is even (aligned bins): two keys per 16-byte load
    for (uint32_t i = 2 * threadIdx.x; i < tn; i += 2 * kKeyThreads) {
        if (i + 1 < tn) {
            const ulonglong2 y = *reinterpret_cast<const ulonglong2*>(in + t0 + i);
            atomicAdd(&lh[(uint32_t)(y.x >> dg.sh2) & dg.m2], 1u);
            atomicAdd(&lh[(uint32_t)(y.y >> dg.sh2) & dg.m2], 1u);
        } else {
            atomicAdd(&lh[(uint32_t)(in[t0 + i] >> dg.sh2) & dg.m2], 1u);
        }
    }
    __syncthreads();
    uint32_t* row = H2 + ((uint64_t)c * J + j) * dg.nb2;
    for (uint32_t d = threadIdx.x; d < dg.nb2; d += kKeyThreads) row[d] = lh[d];
}

// level-2 scan, one workgroup per coarse bin c: per digit the total over the bin's tiles, scanned
// across digits -> bstart of buckets c*nb2 .. c*nb2 + nb2 - 1; then per digit an exclusive scan
// down the tiles, in place (H2 -> P2).  A bin with more tiles than J raises flags[0].
__global__ __launch_bounds__(kKeyThreads) void bp_scan2_kernel(uint32_t* __restrict__ H2,
                                                               const uint32_t* __restrict__ C1, uint32_t J,
                                                               BpDigits dg, uint32_t* __restrict__ bstart,
                                                               uint32_t* __restrict__ flags, uint32_t c0) {
    __shared__ uint32_t tot[kBpMaxBins];
    __shared__ uint32_t wave_tot[kKeyThreads / 64];
    const uint32_t c = c0 + blockIdx.x;
    const uint32_t b0 = C1[dg.nb1 + 1 + c], n = C1[dg.nb1 + 2 + c] - b0;  // compact start, key count
    const uint32_t nt = (n + kBpTile - 1) / kBpTile;
    if (nt > J) {  // no tile of this bin was written: its buckets read as empty, the call reruns
        if (threadIdx.x == 0) {
            flags[0] = 1;
            atomicMax(&flags[4], nt);  // the budget the rerun needs
        }
        for (uint32_t d = threadIdx.x; d < dg.nb2; d += kKeyThreads) bstart[c * dg.nb2 + d] = b0;
        if (threadIdx.x == 0) bstart[(c + 1) * dg.nb2] = b0 + n;  // the bin's end (= the next bin's start)
        return;
    }
    uint32_t* base = H2 + (uint64_t)c * J * dg.nb2;
    for (uint32_t d = threadIdx.x; d < dg.nb2; d += kKeyThreads) {
        tot[d] = col_sum(base + d, dg.nb2, nt);
    }
    __syncthreads();
    lds_bins_scan(tot, dg.nb2, wave_tot);
    for (uint32_t d = threadIdx.x; d < dg.nb2; d += kKeyThreads) {
        const uint32_t run = b0 + tot[d];
        bstart[c * dg.nb2 + d] = run;
        col_prefix_inplace(base + d, dg.nb2, nt, run);
    }
    // the bin's end, which the next bin's scan writes too (same value)
    if (threadIdx.x == 0) bstart[(c + 1) * dg.nb2] = b0 + n;
}

// level 2, pass 2: the tile's keys grouped by digit2 at P2[c][j][digit]
__global__ __launch_bounds__(kKeyThreads) void bp_scatter2_kernel(const unsigned long long* __restrict__ in,
                                                                  const uint32_t* __restrict__ C1, uint32_t J,
                                                                  BpDigits dg, const uint32_t* __restrict__ P2,
                                                                  unsigned long long* __restrict__ out, uint32_t c0) {
    __shared__ __attribute__((aligned(16))) unsigned long long S[kBpTile];
    __shared__ uint32_t lh[kBpMaxBins];
    __shared__ uint32_t wave_tot[kKeyThreads / 64];
    const uint32_t j = blockIdx.x, c = c0 + blockIdx.y;
    uint32_t t0, tn;
    if (!bp_tile(C1, dg.nb1, c, j, J, t0, tn)) return;
    uint32_t pre[kBpQ];
    bp_prow_load(P2 + ((uint64_t)c * J + j) * dg.nb2, dg.nb2, pre);
    for (uint32_t d = threadIdx.x; d < dg.nb2; d += kKeyThreads) lh[d] = 0;
    __syncthreads();
    unsigned long long x[kBpPer];
    uint32_t r[kBpPer];
    auto digit = [&](unsigned long long y) { return (uint32_t)(y >> dg.sh2) & dg.m2; };
#pragma unroll
    for (uint32_t e = 0; e < kBpPer; e += 2) {  // t0 is even: two keys per 16-byte load
        const uint32_t i = 2 * threadIdx.x + e * kKeyThreads;
        if (i + 1 < tn) {
            const ulonglong2 y = *reinterpret_cast<const ulonglong2*>(in + t0 + i);
            x[e] = y.x;
            x[e + 1] = y.y;
        } else {
            x[e] = i < tn ? in[t0 + i] : kNoKey;
            x[e + 1] = kNoKey;
        }
    }
#pragma unroll
    for (uint32_t e = 0; e < kBpPer; ++e) r[e] = x[e] != kNoKey ? atomicAdd(&lh[digit(x[e])], 1u) : 0u;
    __syncthreads();
    bp_place(x, r, tn, dg.nb2, digit, lh, wave_tot, S, pre, out);
}

// ------------------------------------------------------------- cursor level 2 --------------
// Level 2 without its counting passes (bp_hist2 + bp_scan2, 45 us at config 3): every bucket
// owns a fixed-capacity region of capb keys, and the workgroup that writes a run reserves it with
// one returning atomic on the bucket's cursor (its count).  A bucket receives runs from ~30 tiles,
// so the cursors see no queueing; order inside a bucket is unspecified, as with the counting
// partition.  A run that would pass its region's end is dropped and raises kFlCur: the call
// reruns with the counting level 2 (a skewed batch: a very frequent k-mer fills one bucket).
// Regions are sized from the hash-uniform mean (capb ~ 2.6 x mean_keys: 0.6 GB at config 3).
// Measured and rejected: the same reservation at level 1 (per-chunk runs into fixed-capacity
// segments of each coarse bin, 8 / 32 / 64 cursor shards per bin instead of bp_hist1 and the
// column scan): bp_scatter1 went from 139 us to 206 / 173 / 189 us — each of the 7,430
// workgroups waits on its 256 returning atomics before it can write, which costs more than
// the counting pass it replaces.
struct CurGeom {
    uint32_t capb;         // keys per bucket region
    const uint32_t* vreg;  // learned layout (nullptr: fixed): bucket b's region [vreg[b], vreg[b + 1])
    // bucket b's region and capacity; the level-2 kernels take kVreg as a template argument: a
    // run-time choice per key cost bp_scatter2g 138 -> 230 us at config 3
    template <bool kVreg>
    __device__ __forceinline__ uint32_t region(uint32_t b) const { return kVreg ? vreg[b] : b * capb; }
    template <bool kVreg>
    __device__ __forceinline__ uint32_t cap(uint32_t b) const { return kVreg ? vreg[b + 1] - vreg[b] : capb; }
};

// lh holds the tile's digit histogram and r[e] every key's rank in its digit: reserve each digit's
// run on cursor(d) (start of its region: region(d), cap keys), place the tile digit-major into S
// and write each run at its reservation; keys past their region's end are dropped (kFlCur)
template <uint32_t kPer, class Digit, class Cursor, class Region, class Cap, uint32_t kThr = kKeyThreads>
__device__ __forceinline__ void bp_place_cur(const unsigned long long (&x)[kPer], const uint32_t (&r)[kPer],
                                             uint32_t n_in, uint32_t nb, Digit digit, Cursor cursor, Region region,
                                             Cap cap, uint32_t* lh, uint32_t* wave_tot, unsigned long long* S,
                                             unsigned long long* __restrict__ out, uint32_t* __restrict__ flags) {
    constexpr uint32_t kQ = kBpMaxBins / kThr;
    const uint32_t q = (nb + kThr - 1) / kThr, b0 = threadIdx.x * q;
    uint32_t c[kQ], base[kQ], v = 0;
#pragma unroll
    for (uint32_t t = 0; t < kQ; ++t) {
        c[t] = t < q && b0 + t < nb ? lh[b0 + t] : 0u;
        base[t] = c[t] ? atomicAdd(cursor(b0 + t), c[t]) : 0u;
        v += c[t];
    }
    uint32_t excl, total;
    block_scan_n<kThr>(v, excl, total, wave_tot);
#pragma unroll
    for (uint32_t t = 0; t < kQ; ++t)
        if (t < q && b0 + t < nb) {
            lh[b0 + t] = excl;
            excl += c[t];
        }
    __syncthreads();
#pragma unroll
    for (uint32_t e = 0; e < kPer; ++e)
        if (x[e] != kNoKey) S[lh[digit(x[e])] + r[e]] = x[e];
    __syncthreads();
    // lh[d] -> global start of the digit's run minus its tile start; a run that does not fit
    // starts at its region's end, so every one of its keys is dropped below
    bool over = false;
#pragma unroll
    for (uint32_t t = 0; t < kQ; ++t)
        if (t < q && b0 + t < nb) {
            const uint32_t cp = cap(b0 + t);
            const bool fits = base[t] + c[t] <= cp;
            over |= !fits;
            lh[b0 + t] = region(b0 + t) + (fits ? base[t] : cp) - lh[b0 + t];
        }
    if (over) flags[kFlCur] = 1;
    __syncthreads();
    for (uint32_t i = 2 * threadIdx.x; i < n_in; i += 2 * kThr) {
        const ulonglong2 y = *reinterpret_cast<const ulonglong2*>(S + i);
        const uint32_t d0 = digit(y.x), a0 = lh[d0] + i, e0 = region(d0) + cap(d0);
        if (i + 1 < n_in) {
            const uint32_t d1 = digit(y.y), a1 = lh[d1] + i + 1;
            if (d0 == d1 && !(a0 & 1) && a1 < e0) {
                *reinterpret_cast<ulonglong2*>(out + a0) = y;
            } else {
                if (a0 < e0) out[a0] = y.x;
                if (a1 < region(d1) + cap(d1)) out[a1] = y.y;
            }
        } else if (a0 < e0) {
            out[a0] = y.x;
        }
    }
}

// level 2, cursor variant: tile (j, c) of coarse bin c as bp_scatter2, each digit's run reserved
// in its bucket's region; bcur[b] counts bucket b
template <bool kVreg>
__global__ __launch_bounds__(kKeyThreads) void bp_scatter2c_kernel(const unsigned long long* __restrict__ in,
                                                                   const uint32_t* __restrict__ C1, uint32_t J,
                                                                   BpDigits dg, CurGeom cg,
                                                                   uint32_t* __restrict__ bcur,
                                                                   unsigned long long* __restrict__ out,
                                                                   uint32_t* __restrict__ flags, uint32_t c0) {
    __shared__ __attribute__((aligned(16))) unsigned long long S[kBpTile];
    __shared__ uint32_t lh[kBpMaxBins];
    __shared__ uint32_t wave_tot[kKeyThreads / 64];
    const uint32_t j = blockIdx.x, c = c0 + blockIdx.y;
    uint32_t t0, tn;
    if (!bp_tile(C1, dg.nb1, c, j, J, t0, tn)) {
        // a bin above its tile budget: no tile of it is written; its buckets are incomplete
        if (j == 0 && threadIdx.x == 0 && C1[dg.nb1 + 2 + c] - C1[dg.nb1 + 1 + c] > J * kBpTile) {
            flags[kFlBin] = 1;
            atomicMax(&flags[kFlBinTiles], (C1[dg.nb1 + 2 + c] - C1[dg.nb1 + 1 + c] + kBpTile - 1) / kBpTile);
        }
        return;
    }
    for (uint32_t d = threadIdx.x; d < dg.nb2; d += kKeyThreads) lh[d] = 0;
    __syncthreads();
    unsigned long long x[kBpPer];
    uint32_t r[kBpPer];
    auto digit = [&](unsigned long long y) { return (uint32_t)(y >> dg.sh2) & dg.m2; };
#pragma unroll
    for (uint32_t e = 0; e < kBpPer; e += 2) {  // t0 is even: two keys per 16-byte load
        const uint32_t i = 2 * threadIdx.x + e * kKeyThreads;
        if (i + 1 < tn) {
            const ulonglong2 y = *reinterpret_cast<const ulonglong2*>(in + t0 + i);
            x[e] = y.x;
            x[e + 1] = y.y;
        } else {
            x[e] = i < tn ? in[t0 + i] : kNoKey;
            x[e + 1] = kNoKey;
        }
    }
#pragma unroll
    for (uint32_t e = 0; e < kBpPer; ++e) r[e] = x[e] != kNoKey ? atomicAdd(&lh[digit(x[e])], 1u) : 0u;
    __syncthreads();
    const uint32_t bb = c * dg.nb2;
    bp_place_cur(
        x, r, tn, dg.nb2, digit, [&](uint32_t d) { return &bcur[bb + d]; },
        [&](uint32_t d) { return cg.region<kVreg>(bb + d); }, [&](uint32_t d) { return cg.cap<kVreg>(bb + d); }, lh,
        wave_tot, S,
        out, flags);
}

// learned bucket regions: vreg[b] = Σ_{c < b} cap(c), cap(c) = count(c) + count(c) / 8 + 64 rounded
// to 16 keys (counts from the cursors of a call whose regions overflowed: they count every key,
// dropped or not); one workgroup, vreg[nb] = the total
__global__ __launch_bounds__(1024) void vreg_kernel(const uint32_t* __restrict__ counts, uint32_t nb,
                                                    uint32_t* __restrict__ vreg) {
    __shared__ uint32_t wave_tot[1024 / 64];
    uint32_t carry = 0;
    for (uint32_t base = 0; base < nb; base += 1024) {
        const uint32_t b = base + threadIdx.x;
        const uint32_t c = b < nb ? counts[b] : 0u;
        const uint32_t cap = b < nb ? (c + c / 8 + 64 + 15) / 16 * 16 : 0u;
        uint32_t excl, total;
        block_scan_n<1024>(cap, excl, total, wave_tot);
        if (b < nb) vreg[b] = carry + excl;
        carry += total;
    }
    if (threadIdx.x == 0) vreg[nb] = carry;
}

__global__ void bp_cur_clear_kernel(uint32_t* __restrict__ cur, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) cur[i] = 0;
}

// ------------------------------------------------------------- local level 1 ---------------
// With the cursor level 2 the coarse bins need not be contiguous: level 1 leaves each chunk's
// keys in its own 4,096-key segment of ws->keys, grouped by digit1 (the chunk's runs, packed
// start << 16 | count in H1[chunk][digit]), and a level-2 tile gathers the runs of one coarse bin
// over a range of T chunks.  That drops bp_hist1 (every key computed a second time) and the
// column scan, and level 1 writes whole segments.  The cursor level 2 is the only consumer; the
// counting fallback (kFlCur) reruns with the counting level 1.
constexpr uint32_t kBpGatherMax = 1024;  // chunks per level-2 tile (T)
constexpr uint32_t kBpGatherTile = 4096;  // keys per round of a level-2 tile

// KMP_L1_THREADS: workgroup size of the local level 1 (a 4,096-slot chunk either way; 512 threads
// own 8 slots each: twice the waves per CU at the same LDS; keys_level1 0.139 -> 0.127 ms at config 3)
#ifndef KMP_L1_THREADS
#define KMP_L1_THREADS 512
#endif

// Chunk descriptors of the local level 1: desc[c] = {first, last, r0, r1} = the proteins whose
// regions overlap chunk c ([first, last]; n is the tail past the last region) and the residue span
// [r0, r1) its windows read.  One thread per protein p <= n writes the chunks that start in its
// region (first, r0) and those that end in it (last, r1); the grid also clears the cursor level 2's
// bucket counts (one launch less per step).  Residue offsets fit u32 (bp_level1 checks slots).
// StepClear: the step's flags and statistics (and extra words: the k-mer split's send cursors),
// cleared by the first kernel of the residue front instead of a kernel of their own
struct StepClear {
    uint32_t* flags;
    uint32_t n_flags;
    unsigned long long* gstats;
    uint32_t n_gstats;
    unsigned long long* extra;
    uint32_t n_extra;
};
__global__ void chunk_desc_kernel(const uint64_t* __restrict__ res_off, uint32_t n, uint64_t slots,
                                  uint32_t n_chunks, int k, uint4* __restrict__ desc, uint32_t* __restrict__ cur,
                                  uint32_t ncur, StepClear sc) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    for (uint32_t i = t; i < ncur; i += gridDim.x * blockDim.x) cur[i] = 0;
    if (blockIdx.x == 0 && sc.flags) {
        for (uint32_t i = threadIdx.x; i < sc.n_gstats; i += blockDim.x) sc.gstats[i] = 0;
        for (uint32_t i = threadIdx.x; i < sc.n_flags; i += blockDim.x) sc.flags[i] = 0;
        for (uint32_t i = threadIdx.x; i < sc.n_extra; i += blockDim.x) sc.extra[i] = 0;
    }
    const uint32_t p = t;
    if (p > n) return;
    const uint64_t off = res_off[p], L = p < n ? res_off[p + 1] - off : 0;
    const uint64_t b = set_base(off, p), e = p < n ? set_base(res_off[p + 1], p + 1) : slots;
    for (uint64_t c = (b + kKeyChunk - 1) / kKeyChunk; c * kKeyChunk < e && c < n_chunks; ++c) {
        desc[c].x = p;
        desc[c].z = (uint32_t)(off + min<uint64_t>(c * kKeyChunk - b, L));
    }
    // chunks whose last slot min((c + 1) * kKeyChunk, slots) - 1 lies in [b, e)
    for (uint64_t c = b / kKeyChunk; c < n_chunks; ++c) {
        const uint64_t c1 = min<uint64_t>((c + 1) * kKeyChunk, slots);
        if (c1 - 1 >= e) break;
        if (c1 - 1 < b) continue;
        desc[c].y = p;
        desc[c].w = (uint32_t)(p < n ? off + min<uint64_t>(L, c1 - b + k - 1) : off);
    }
}

// waves per SIMD the persistent level 1 is compiled for (VGPR budget: 8 -> 64 registers and 24 B of
// scratch per lane, four 512-thread workgroups per CU; at 6 waves, 79 registers, a rank of the k-mer
// split at G = 8 spent 91 us in it against 86 us at 8; one GPU: the same)
#ifndef KMP_L1P_WAVES
#define KMP_L1P_WAVES 8
#endif
// Level 1, local, persistent: workgroup w takes chunks w, w + grid, ...; chunk c's keys of the
// call's digits [dlo, dhi) grouped by digit1 at out[c * kKeyChunk ...] (its own 4,096-key segment),
// its run table (start << 16 | count per own digit) in H1[c][digit - dlo].  The next chunk's
// residues and protein table are loaded into registers while this chunk is keyed, ranked and
// written (its descriptor one chunk earlier still), so the three dependent global round trips of
// a chunk (descriptor, protein offsets, residues) stay off the critical path: the one-chunk-per-
// workgroup kernel spent ~13 us per chunk waiting on them.
template <uint32_t kThr>
__global__ __launch_bounds__(kThr, KMP_L1P_WAVES) void bp_scatter1p_kernel(
    const uint8_t* __restrict__ res, const uint64_t* __restrict__ res_off, const uint16_t* __restrict__ cls, int k,
    uint32_t n, uint64_t slots, uint32_t G, const uint4* __restrict__ desc, Layout lay, BpDigits dg, uint32_t pw21,
    uint32_t dlo, uint32_t dhi, uint32_t* __restrict__ H1, unsigned long long* __restrict__ out,
    uint32_t* __restrict__ flags) {
    __shared__ union {
        KeyChunk kc;
        unsigned long long S[kKeyChunk];
    } u;
    __shared__ uint8_t lut[256];
    __shared__ uint32_t lh[kBpMaxBins];
    __shared__ uint32_t wave_tot[kThr / 64];
    __shared__ uint32_t s_n;
    constexpr uint32_t kPer = kKeyChunk / kThr, kPP = (kKeyProtMax + kThr - 1) / kThr;
    const uint32_t tid = threadIdx.x, nown = dhi - dlo;
    uint32_t c = blockIdx.x;
    if (c >= G) return;
    for (uint32_t i = tid; i < 256; i += kThr) lut[i] = c_lut.v[i];
    __syncthreads();  // the table before the first staging reads it
    const uint64_t res_end = res_off[n];
    const bool vec_ok = ((uintptr_t)res & 15u) == 0;
    // one chunk's loads, held in registers until it is staged
    uint4 pv = make_uint4(0, 0, 0, 0);
    uint32_t po[kPP], pe[kPP];  // residue offsets (< 2^32: bp_level1 checks slots)
    uint16_t pcl[kPP];
    auto span = [&](const uint4& d, uint64_t& a0, uint32_t& nv, uint32_t& np) {
        a0 = d.z & ~15u;
        nv = (uint32_t)((max(d.w, d.z) - a0 + 15) >> 4);
        np = d.x < n ? min(d.y, n - 1) + 1 - d.x : 0u;
    };
    auto issue = [&](const uint4& d) {
        uint64_t a0;
        uint32_t nv, np;
        span(d, a0, nv, np);
        if (tid < nv) {
            const uint64_t g = a0 + 16ull * tid;
            if (vec_ok && g + 16 <= res_end) {
                pv = *reinterpret_cast<const uint4*>(res + g);
            } else {
                uint32_t w[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    w[q] = 0;
#pragma unroll
                    for (int bb = 0; bb < 4; ++bb) {
                        const uint64_t i = g + 4 * q + bb;
                        w[q] |= (uint32_t)(i < res_end ? res[i] : 0) << (8 * bb);
                    }
                }
                pv = make_uint4(w[0], w[1], w[2], w[3]);
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < kPP; ++j) {
            const uint32_t t = tid + j * kThr;
            if (t < np) {
                po[j] = (uint32_t)res_off[d.x + t];
                pe[j] = (uint32_t)res_off[d.x + t + 1];
                pcl[j] = cls[d.x + t];
            }
        }
    };
    uint4 dcur = desc[c];
    uint4 dnxt = c + gridDim.x < G ? desc[c + gridDim.x] : make_uint4(0, 0, 0, 0);
    issue(dcur);
    const unsigned hs1 = dg.sh1 - lay.hshift;
    while (true) {
        const uint64_t c0 = (uint64_t)c * kKeyChunk, c1 = min(c0 + kKeyChunk, slots);
        // ---- stage chunk c from the registers ----
        {
            uint64_t a0;
            uint32_t nv, np;
            span(dcur, a0, nv, np);
            if (tid < nv) {
                auto code4 = [&](uint32_t x) {
                    return (uint32_t)lut[x & 255u] | (uint32_t)lut[(x >> 8) & 255u] << 8 |
                           (uint32_t)lut[(x >> 16) & 255u] << 16 | (uint32_t)lut[x >> 24] << 24;
                };
                *reinterpret_cast<uint4*>(u.kc.rc + 16 * tid) =
                    make_uint4(code4(pv.x), code4(pv.y), code4(pv.z), code4(pv.w));
            }
#pragma unroll
            for (uint32_t j = 0; j < kPP; ++j) {
                const uint32_t t = tid + j * kThr;
                if (t < np) {
                    const uint32_t p = dcur.x + t;
                    const uint32_t L = pe[j] - po[j];
                    u.kc.pb[t] = (uint32_t)(set_base(po[j], p) - c0);  // wraps for the first protein
                    u.kc.pw[t] = L >= (uint32_t)k ? L - k + 1 : 0u;
                    u.kc.pc[t] = pcl[j];
                    u.kc.pr[t] = (int32_t)((int64_t)po[j] - (int64_t)a0);
                    check_class(pcl[j], lay, flags);
                }
            }
            if (tid == 0) {
                u.kc.np = np;
                s_n = 0;
            }
            for (uint32_t d = tid; d < nown; d += kThr) lh[dlo + d] = 0;
        }
        __syncthreads();
        // ---- the next chunk's loads go out now; the descriptor after it too ----
        const uint32_t cn = c + gridDim.x;
        uint4 dnn = make_uint4(0, 0, 0, 0);
        if (cn < G) {
            issue(dnxt);
            if (cn + gridDim.x < G) dnn = desc[cn + gridDim.x];
        }
        // ---- key, rank by digit1, write the segment ----
        unsigned long long x[kPer];
        uint32_t r[kPer], nk = 0;
        key_chunk_run<kPer>(u.kc, tid * kPer, (uint32_t)(c1 - c0), k, pw21, dcur.x, lay,
                            [&](uint32_t e, bool valid, uint32_t h, unsigned long long lo) {
                                const uint32_t d = h >> hs1;
                                const bool mine = valid && d >= dlo && d < dhi;  // the call's coarse bins
                                x[e] = mine ? ((unsigned long long)h << lay.hshift) | lo : kNoKey;
                                r[e] = mine ? atomicAdd(&lh[d], 1u) : 0u;
                                nk += mine;
                            });
        if (nk) atomicAdd(&s_n, nk);
        __syncthreads();  // the chunk's staging (u.kc) is dead from here: u.S reuses it
        constexpr uint32_t kQ = kBpMaxBins / kThr;
        uint32_t cnt[kQ];
#pragma unroll
        for (uint32_t t = 0; t < kQ; ++t) {
            const uint32_t d = tid + t * kThr;
            cnt[t] = d < nown ? lh[dlo + d] : 0u;
        }
        lds_bins_scan<kThr>(lh + dlo, nown, wave_tot);
        uint32_t* row = H1 + (uint64_t)c * nown;
#pragma unroll
        for (uint32_t t = 0; t < kQ; ++t) {
            const uint32_t d = tid + t * kThr;
            if (d < nown) row[d] = lh[dlo + d] << 16 | cnt[t];
        }
#pragma unroll
        for (uint32_t e = 0; e < kPer; ++e)
            if (x[e] != kNoKey) u.S[lh[(uint32_t)(x[e] >> dg.sh1)] + r[e]] = x[e];
        __syncthreads();
        const uint32_t n_in = s_n;
        unsigned long long* seg = out + c0;  // c0 = chunk * kKeyChunk: 16-byte aligned
        for (uint32_t i = 2 * tid; i < n_in; i += 2 * kThr) {
            if (i + 1 < n_in)
                *reinterpret_cast<ulonglong2*>(seg + i) = *reinterpret_cast<const ulonglong2*>(u.S + i);
            else
                seg[i] = u.S[i];
        }
        if (cn >= G) break;
        __syncthreads();  // S read before the next chunk's staging overwrites it
        c = cn;
        dcur = dnxt;
        dnxt = dnn;
    }
}

// H1[G][nb1] -> H1T[digit - dlo][G] for digits [dlo, dhi) (32 x 32 tiles through LDS)
__global__ __launch_bounds__(256) void bp_h1t_kernel(const uint32_t* __restrict__ H1, uint32_t G, uint32_t nb1,
                                                     uint32_t dlo, uint32_t dhi, uint32_t* __restrict__ H1T) {
    __shared__ uint32_t tile[32][33];
    const uint32_t g0 = blockIdx.x * 32, d0 = dlo + blockIdx.y * 32;
    const uint32_t tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (uint32_t y = ty; y < 32; y += 8) {
        const uint32_t g = g0 + y, d = d0 + tx;
        tile[y][tx] = g < G && d < dhi ? H1[(uint64_t)g * nb1 + d] : 0u;
    }
    __syncthreads();
    for (uint32_t y = ty; y < 32; y += 8) {
        const uint32_t d = d0 + y, g = g0 + tx;
        if (d < dhi && g < G) H1T[(uint64_t)(d - dlo) * G + g] = tile[tx][y];
    }
}

// level 2 over the local level 1: tile (j, c) = coarse bin c's runs in chunks [j*T, j*T + T),
// read from the run table at H1T[(c - dlo) * hsb + chunk * hsc] (the transposed table: hsb = G,
// hsc = 1; the level-1 table itself for a few own bins: hsb = 1, hsc = own bins),
// gathered and reserved in the bucket regions as bp_scatter2c.  The run table (off, src) and a
// key -> run map live in S until the keys are in registers, so the loads go out coalesced
// (element tid + e*kKeyThreads, as the other scatters).  A tile above kBpTile keys (a skewed
// batch) goes in several rounds.  XCD-aware order: workgroup L runs on XCD L % 8, and XCD x
// takes the tiles [x * per, (x + 1) * per) of the bin-major tile list, so neighbouring bins' tiles
// of a chunk range (whose runs share the 128-B lines at their ends) run on one L2 at about the
// same time.
template <uint32_t kPer, uint32_t kThr, bool kVreg>
__global__ __launch_bounds__(kThr) void bp_scatter2g_kernel(const unsigned long long* __restrict__ in,
                                                                   const uint32_t* __restrict__ H1T, uint32_t G,
                                                                   uint32_t hsb, uint32_t hsc,
                                                                   uint32_t T, uint32_t ntiles, uint32_t nbins,
                                                                   BpDigits dg, CurGeom cg,
                                                                   uint32_t* __restrict__ bcur,
                                                                   unsigned long long* __restrict__ out,
                                                                   uint32_t* __restrict__ flags, uint32_t c0,
                                                                   uint32_t dlo) {
    constexpr uint32_t kTile = kPer * kThr;
    __shared__ __attribute__((aligned(16))) unsigned long long S[kTile];
    __shared__ uint32_t lh[kBpMaxBins];
    __shared__ uint32_t wave_tot[kThr / 64];
    // aliases in S, dead once the tile's keys are loaded: src[kBpGatherMax] (a run's segment
    // offset minus its tile offset, mod 2^32) | map[kBpTile] (key -> run)
    uint32_t* src = reinterpret_cast<uint32_t*>(S);
    uint16_t* map = reinterpret_cast<uint16_t*>(src + kBpGatherMax);
    static_assert(kBpGatherMax * 4 + kTile * 2 <= sizeof(S), "gather tables fit in S");
    constexpr uint32_t kQ = kBpGatherMax / kThr;
    const uint32_t total = ntiles * nbins, per = (total + 7) / 8;
    const uint32_t w = (blockIdx.x % 8) * per + blockIdx.x / 8;
    if (w >= total) return;
    const uint32_t c = c0 + w / ntiles, ch0 = (w % ntiles) * T;
    if (ch0 >= G) return;
    const uint32_t nch = min(T, G - ch0);
    const uint32_t* row = H1T + (uint64_t)(c - dlo) * hsb + (uint64_t)ch0 * hsc;
    const uint32_t q = (nch + kThr - 1) / kThr, b0 = threadIdx.x * q;
    uint32_t p[kQ], v = 0;
#pragma unroll
    for (uint32_t t = 0; t < kQ; ++t) {
        p[t] = t < q && b0 + t < nch ? row[(uint64_t)(b0 + t) * hsc] : 0u;
        v += p[t] & 0xFFFFu;
    }
    uint32_t excl0, tn;
    block_scan_n<kThr>(v, excl0, tn, wave_tot);
    auto digit = [&](unsigned long long y) { return (uint32_t)(y >> dg.sh2) & dg.m2; };
    const uint32_t bb = c * dg.nb2;
    auto cursor = [&](uint32_t d) { return &bcur[bb + d]; };
    auto region = [&](uint32_t d) { return cg.region<kVreg>(bb + d); };
    auto capof = [&](uint32_t d) { return cg.cap<kVreg>(bb + d); };
    for (uint32_t base = 0; base < tn; base += kTile) {
        if (base) __syncthreads();  // the previous round's writes have read lh and S
        const uint32_t n_in = min(kTile, tn - base);
        for (uint32_t d = threadIdx.x; d < dg.nb2; d += kThr) lh[d] = 0;
        uint32_t excl = excl0;
#pragma unroll
        for (uint32_t t = 0; t < kQ; ++t)
            if (t < q && b0 + t < nch) {
                src[b0 + t] = (ch0 + b0 + t) * kKeyChunk + (p[t] >> 16) - excl;
                excl += p[t] & 0xFFFFu;
            }
        // key -> run map of the round's window [base, base + n_in)
        excl = excl0;
#pragma unroll
        for (uint32_t t = 0; t < kQ; ++t)
            if (t < q && b0 + t < nch) {
                const uint32_t e1 = excl + (p[t] & 0xFFFFu);
                const uint32_t lo = max(excl, base), hi = min(e1, base + n_in);
                for (uint32_t i = lo; i < hi; ++i) map[i - base] = (uint16_t)(b0 + t);
                excl = e1;
            }
        __syncthreads();
        unsigned long long x[kPer];
        uint32_t r[kPer];
#pragma unroll
        for (uint32_t e = 0; e < kPer; ++e) {
            const uint32_t i = threadIdx.x + e * kThr;
            if (i < n_in) {
                x[e] = in[src[map[i]] + base + i];
            } else {
                x[e] = kNoKey;
            }
        }
#pragma unroll
        for (uint32_t e = 0; e < kPer; ++e) r[e] = x[e] != kNoKey ? atomicAdd(&lh[digit(x[e])], 1u) : 0u;
        __syncthreads();  // every key loaded: S is free for the placement
        bp_place_cur<kPer, decltype(digit), decltype(cursor), decltype(region), decltype(capof), kThr>(
            x, r, n_in, dg.nb2, digit, cursor, region, capof, lh, wave_tot, S, out, flags);
    }
}

// the small bucket kernel for this layout: merged slot words when the bucket field is wide enough;
// a 1,024-key capacity (four keys per thread) when the mean bucket is small enough that a bucket
// above it is a > 4-sigma event (the large kernel takes those)
constexpr uint32_t kBucketCap1024Mean = 800;  // at config 3 (mean 897) the 1,280 variant measured faster
// buckets [b0, b0 + nb)
template <bool kRows, bool kScore>
void launch_buckets(const BucketArgs& a, uint32_t b0, uint32_t nb, uint32_t large_grid, hipStream_t st) {
    if (a.lay.bbits >= kMergeMinBits && a.lay.mean_keys <= kBucketCap1024Mean)  // four keys per thread
        bucket_small_kernel<1024, kBucketSmallThreads, kBucketSmallTab, true, kRows, kScore>
            <<<nb, kBucketSmallThreads, 0, st>>>(a, b0);
    else if (a.lay.bbits >= kMergeMinBits)
        bucket_small_kernel<kBucketSmallCap, kBucketSmallThreads, kBucketSmallTab, true, kRows, kScore>
            <<<nb, kBucketSmallThreads, 0, st>>>(a, b0);
    else
        bucket_small_kernel<kBucketSmallCap, kBucketSmallThreads, kBucketSmallTab, false, kRows, kScore>
            <<<nb, kBucketSmallThreads, 0, st>>>(a, b0);
    if (large_grid)  // 0: the last call listed no bucket (a listed one now makes the call rerun)
        bucket_large_kernel<kBucketLargeCap, kBucketLargeThreads, kBucketLargeTab, kRows, kScore>
            <<<large_grid, kBucketLargeThreads, 0, st>>>(a);
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

// bumped on every reallocation of a workspace buffer: a captured step graph is valid only for the
// generation it was captured in.  Atomic: the ranks of a multi-GPU context reserve from one host
// thread each at the same time (kmp_api.cpp split_rank_edges / rows_rank_edges)
std::atomic<unsigned long long> g_grow_gen{0};

// the row-block tail's geometry (pt_geometry)
struct PtGeom {
    unsigned pbits, rbits;  // key = p << pbits | q; rows per block = 1 << rbits
    unsigned sbits;         // scored: the score field below the pair ((pair << sbits) | field), else 0
    int kbit;               // scored multi-k: bit kScoreBits of the field marks the second k (w1 counted)
    uint32_t nrb;           // row blocks, from row row0
    uint32_t jt;            // tiles per shard region
    uint64_t sc;            // shard region capacity
    uint32_t nshards;       // shard regions (kShards), or 1 for a flat array
    uint32_t row0;          // first row (a pass's or rank's row range)
    uint64_t flat_n;        // nonzero: one region of flat_n keys with kNoKey padding (no cursors)
    uint32_t min_shared;    // runs with w < min_shared are dropped
    uint32_t nprot;         // proteins (q < nprot): the pair range of a row block (pt_bin_sort)
    uint32_t rowend;        // the call's last row + 1
    int binsort;            // the reduce sorts by bins (pt_bin_sort), else the block radix sort
    uint32_t ftcap;         // fast tail: keys per row-block region
    int dense;              // fast tail: per-block dense histogram over (row, q) (2^(pbits + rbits) bins)
};

template <class T>
struct Grow {
    T* p = nullptr;
    size_t n = 0;
    hipError_t reserve(size_t m) {
        if (m <= n && p) return hipSuccess;
        g_grow_gen.fetch_add(1, std::memory_order_relaxed);
        const auto t0 = std::chrono::steady_clock::now();
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        // a large buffer grows with a quarter of headroom: the passes of a stream vary in size, and
        // every regrowth of a multi-GB buffer (a synchronous free + a fresh allocation) stalled the
        // device for up to seconds
        const size_t want = m > (size_t{1} << 26) ? m + m / 4 : std::max<size_t>(1, m);
        static const bool dbg = getenv("KMP_DEBUG_GROW") != nullptr;
        hipError_t e = hipMalloc(&p, want * sizeof(T));
        if (e == hipSuccess) n = want;
        if (dbg && want * sizeof(T) >= (64u << 20))
            fprintf(stderr, "kmp: grow %p to %.1f MB (%zu B elements) in %.1f ms\n", (void*)this,
                    want * sizeof(T) / 1e6, sizeof(T),
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
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
    Grow<uint32_t> w, keep, pos, small, cnt, flags;  // flags: see kFl*
    Grow<char> tmp;
    bool timing = false;
    bool bucketed = true;       // try the bucketed layout first
    bool last_bucketed = false; // layout the last call ran on
    bool last_fused = false;    // ... single-synchronisation step (else the split step)
    bool last_heavy = false;    // ... with spilled frequent k-mers
    bool last_fast = false;     // ... reduced by the fast row-block tail
    uint32_t last_ovf = 0;      // ... row blocks finished by the overflow sort
    uint64_t shard_cap = 0;     // capacity of each pair-key shard region
    uint64_t shard_floor = 0;   // ... at least (kmp_postings_set_shard_floor: a stream's planned pass size)
    uint64_t stage_floor = 0;   // tail_multi's staging capacity at least (keys; same call)
    Grow<uint32_t> chunk_first;
    Grow<uint32_t> chunk_desc;  // local level 1: per chunk {first, last, r0, r1}
    Grow<uint32_t> bp;          // bucket partition: H1 | P1 | R | C1 | H2 (see bp_level1)
    Grow<uint32_t> pt;          // row-block tail (pt_bufs)
    Grow<uint32_t> ovf;         // listed row blocks | segment starts | segment ends
    Grow<unsigned long long> ovk;  // their keys tagged, sorted, encoded (pt_finish_overflow)
    Grow<unsigned long long> ovx;  // per listed block: offset of its keys
    Grow<uint32_t> ovr;            // run lengths, kept flags and positions, first run per block
    Grow<uint32_t> ova;            // scored: per run (w, w1, score)
    Grow<uint32_t> stg2;           // scored tail: staged scores | second-k weights
    Grow<uint32_t> k2, dsc;        // fused tail's sub-blocks: keys by sub-block | descriptors, counts, offsets
    uint64_t pt_inc = 0;        // incidences of the last call (row-block sizing)
    uint64_t last_most = 0;     // expand-only call: the fullest shard region (sizes the next call's)
    // tail_multi's staged result, kept for a re-emit into larger arrays: sub-blocks, staging
    // capacity, edges, and the call it belongs to (rows, ks, n)
    uint32_t pend_nd = 0;
    uint64_t pend_total = 0, pend_ne = 0;
    std::vector<unsigned long long> pend_key;
    // the fused tail writes its edges in place (pt_reduce_count + pt_reduce_write); 0: staged runs + emit
    int direct_tail = 1;
    int flat_heavy = 1;  // ranged plain-order heavy expansion by rows (heavy_flat_kernel); 0: tiles
    int spill_all_on = 1;  // ... with every bucket spilled on the first pass (no bucket kernel after it)
    bool front_all = false;  // the current front's spill holds every bucket
    bool pend_direct = false;  // the pending re-emit reruns the in-place reduce (its keys still held)
    PtGeom pend_g{};
    Grow<unsigned long long> dlb;  // its statistics (windowed sub-blocks)
    Grow<uint32_t> doff;           // its sub-blocks' edge offsets
    Grow<unsigned long long> split_cur;  // k-mer split: per-destination send cursors
    std::vector<unsigned long long> split_shape;
    bool split_heavy = false;  // k-mer split: this batch spills, its heavy path runs on every call
    unsigned pt_rb_max = 16;    // rows-per-block bound learned from overflowing row blocks
    unsigned long long* clear_extra = nullptr;  // cleared with the step's flags (the split's send cursors)
    // the k-mer split's routed bucket output (BucketArgs.send): send buffer, capacity per rank, rows
    unsigned long long* route_send = nullptr;
    uint64_t route_cap = 0;
    SplitRows route_rows{};
    uint32_t clear_n = 0;
    uint32_t large_grid = 1024;  // workgroups of the large-bucket kernel (from the last call's list; 0: none)
    uint32_t large_used = 1024;  // ... the grid the last front launched
    bool fast_mode = true;      // kmp_postings_set_tail: the fast tail allowed
    bool dense_on = false;      // ... its dense variant too (KMP_TAIL_DENSE: measured slower on uniprot k = 5)
    bool fast_tail = true;      // unscored calls take the fast row-block tail (off for a shape whose
                                // row-block regions overflowed: kRbFast)
    uint32_t bp_J = 0;          // level-2 tiles per coarse bin ...
    uint32_t bp_J_min = 0;      // ... at least (learned from an overflowing bin)
    uint64_t bp_c1 = 0;         // offset of C1 (coarse bin starts) in ws->bp
    bool parted = false;        // ws->keys holds level-1 output (bp_level1 ran for this call)
    bool bp_local = false;      // ... in chunk segments (local level 1: H1T at bp + bp_h1t)
    bool clear_in_keys = false;  // the call's key path clears the step's flags (residue paths)
    bool defer_clear = false;    // ... and has not yet
    uint32_t bp_G = 0, bp_T = 0;
    uint32_t bp_hsb = 0, bp_hsc = 1;  // level 2's run-table strides (bin, chunk)
    uint64_t bp_h1t = 0;
    // coarse bins [bin_lo, bin_hi) of this call (bin_hi 0: all): the bucket-range share of a rank
    // of the multi-GPU k-mer split (kmp_dev_split_expand); level 1 keeps only their keys
    uint32_t bin_lo = 0, bin_hi = 0;
    // cursor level 2 (fixed-capacity bucket regions, no counting passes): tried first for a new
    // shape (cur_on), dropped for the shape after a region overflow; cur_used: the buckets in
    // ws->sorted came from it (ws->cur: bucket counts)
    bool cur_mode = true, cur_on = true, cur_used = false;
    Grow<uint32_t> cur;
    CurGeom cg{};
    // learned bucket layout of the cursor level 2 (a batch whose frequent k-mers overflow the
    // hash-uniform regions: the reference's uniprot_arg at k = 5): region starts from the last
    // call's exact bucket counts with an eighth of headroom; relearned on an overflow, the counting
    // partition after kVregTries in a row
    Grow<uint32_t> vreg;
    bool vreg_on = false;
    uint64_t vreg_total = 0;
    uint32_t vreg_tries = 0;
    // heavy path (frequent k-mers): spill regions, the gathered + sorted spill, its elements,
    // k-mer starts, per-k-mer row bounds / tile counts / tile offsets
    Grow<unsigned long long> spill, hkeys, hsorted, hGS, htc, htoff, hoff, hRH, hseg, hcur;
    bool hcur_valid = false;  // hcur holds the current front's spill cursors
    Grow<uint32_t> hE, hgi, hcnt, hrun, hblk, hGH;  // hGH: each heavy k-mer's h
    // ranged plain-order calls (heavy_flat_kernel): each element's k-mer, the per-protein index
    // (elements by protein | protein starts, host copy) and its build scratch
    Grow<uint32_t> hKG, hPE, hPO, hPC;
    std::vector<uint32_t> hPOh;
    bool h_flat_ready = false, h_kg = false;
    uint64_t h_ng = 0;  // k-mers of the compaction (read back with the index)
    uint64_t spill_cap = 0;     // keys per spill shard region
    bool heavy = false;         // this workspace's batches spill: run the split step
    bool heavy_ready = false;   // hE / hGS hold the current front's compacted spill
    uint64_t h_m = 0;                // spill keys behind hE (the bound on elements and k-mers)
    uint64_t h_segs = 0, h_segmax = 0;  // the front's spill segments: count, largest (read-back)
    int h_cls = 0;                   // hE in class order
    unsigned long long* h_tot = nullptr;  // device: elements, k-mers, class runs
    std::vector<unsigned long long> shape;  // (n, slots, code bits, bucket bits) of the last batch
    // front reuse (kmp_postings_set_reuse): a call on the same batch (front_key) keeps the keys,
    // level 2 and the heavy compaction of the last successful call and runs only the buckets,
    // the heavy expansion and the tail of its rows (the passes / ranks of one batch)
    bool reuse = false, front_ok = false;
    std::vector<unsigned long long> front_key;
    // single-synchronisation step as a HIP graph: captured on the second call with the same shape
    // (every buffer already sized), replayed after that
    bool graph_on = true;
    struct GraphSlot {  // one captured sequence: its executable and the shape it was captured for
        hipGraphExec_t gexec = nullptr;
        std::vector<unsigned long long> key, seen;
        void reset() {
            if (gexec) (void)hipGraphExecDestroy(gexec);
            gexec = nullptr;
            key.clear();
            seen.clear();
        }
    } split_g[2];  // the k-mer split's phases (expand, edges)
    hipGraphExec_t gexec = nullptr;
    hipStream_t cst = nullptr;  // capture stream
    std::vector<unsigned long long> gkey, gkey_seen;
    uint64_t graph_replays = 0;
    // read-back of a step (kRb* layout), written by the pack kernel into coherent pinned memory
    unsigned long long* hrb = nullptr;
    hipEvent_t ev[KMP_POSTINGS_STAGES + 1] = {};
    hipEvent_t mev[4] = {};  // kmp_dev_pairs_rows_multi: start, first k expanded, second k, tail done
    const uint32_t* pt_zero_p = nullptr;  // the pt allocation whose totals T were cleared
    size_t pt_zero_n = 0;
    ~kmp_postings() {
        for (auto* g : {&keys, &sorted, &inc, &inc_sorted, &uniq, &bstats, &btot, &boff, &spill, &hkeys, &hsorted,
                        &hGS, &htc, &htoff, &hoff, &hRH, &hseg, &hcur, &ovk, &ovx, &split_cur})
            g->release();
        for (auto* g : {&w, &keep, &pos, &small, &cnt, &flags, &chunk_first, &chunk_desc, &bp, &pt, &ovf, &ovr, &ova, &stg2, &k2, &dsc, &hE, &hgi, &hcnt,
                        &hrun, &hblk, &cur, &hGH})
            g->release();
        tmp.release();
        for (auto& e : ev)
            if (e) (void)hipEventDestroy(e);
        for (auto& e : mev)
            if (e) (void)hipEventDestroy(e);
        if (hrb) (void)hipHostFree(hrb);
        if (gexec) (void)hipGraphExecDestroy(gexec);
        for (auto& g : split_g) g.reset();
        if (cst) (void)hipStreamDestroy(cst);
    }
    void mark(int stage, hipStream_t st) {
        if (timing) (void)hipEventRecord(ev[stage], st);
    }
};

#define PG(x)                                                                                         \
    do {                                                                                              \
        hipError_t e_ = (x);                                                                          \
        if (e_ != hipSuccess) {                                                                       \
            if (getenv("KMP_DEBUG"))                                                                  \
                fprintf(stderr, "kmp: %s failed: %s (kmp_postings.hip:%d)\n", #x, hipGetErrorString(e_), \
                        __LINE__);                                                                    \
            return e_ == hipErrorOutOfMemory ? KMP_ENOMEM : KMP_EDEVICE;                              \
        }                                                                                             \
    } while (0)

namespace {

void fill_stats(kmp_postings_stats* stats, const unsigned long long* acc) {
    if (!stats) return;
    stats->sum_S = acc[kStSumS];
    stats->distinct = acc[kStDistinct];
    stats->repeat = acc[kStRepeat];
    stats->sum_cdf2_light = acc[kStCdf2];
    stats->max_df = acc[kStMaxDf];
    stats->heavy_entries = acc[kStHeavy];
    stats->incidences = acc[kStInc];
}

// Level 1 of the bucket partition for proteins [0, n): ws->keys = the valid keys grouped by
// digit1; C1 = coarse bin starts (C1[nb1] = key count) in ws->bp for level 2.
// the call's coarse bins [*lo, *hi)
void own_bins(const kmp_postings* ws, const BpDigits& dg, uint32_t* lo, uint32_t* hi) {
    *lo = ws->bin_hi ? ws->bin_lo : 0u;
    *hi = ws->bin_hi ? std::min(ws->bin_hi, dg.nb1) : dg.nb1;
}

__global__ void step_clear_kernel(uint32_t* __restrict__ flags, unsigned long long* __restrict__ gstats,
                                  unsigned long long* __restrict__ extra, uint32_t n_extra);

hipError_t bp_level1(kmp_postings* ws, const uint8_t* d_res, const uint64_t* d_res_off, const uint16_t* d_class,
                     int k, uint32_t n, uint64_t slots, const Layout& lay, hipStream_t st) {
    const BpDigits dg = bp_digits(lay);
    uint32_t dlo, dhi;
    own_bins(ws, dg, &dlo, &dhi);
    const uint64_t G64 = (slots + kKeyChunk - 1) / kKeyChunk;
    if (G64 * dg.nb1 > 0xFFFFFFFFull || slots > 0xFFFFFFFFull) return hipErrorInvalidValue;
    const uint32_t G = (uint32_t)G64, groups = (G + kBpRowGroup - 1) / kBpRowGroup;
    // coarse bins are hash-uniform: a budget of 1.25x the mean plus two tiles
    ws->bp_J = std::max(ws->bp_J_min, (uint32_t)((slots / dg.nb1 * 5 / 4 + kBpTile - 1) / kBpTile) + 2);
    const uint64_t h1 = (uint64_t)G * dg.nb1, r = (uint64_t)groups * dg.nb1;
    const uint64_t need = 2 * h1 + r + 2 * (dg.nb1 + 1) + (uint64_t)dg.nb1 * ws->bp_J * dg.nb2;
    hipError_t e = ws->bp.reserve(need);
    if (e == hipSuccess) e = ws->keys.reserve(slots + (uint64_t)kBpAlign * dg.nb1);  // + alignment gaps
    if (e == hipSuccess) e = ws->chunk_first.reserve(G + 1);
    if (e != hipSuccess) return e;
    uint32_t *H1 = ws->bp.p, *P1 = H1 + h1, *R = P1 + h1, *C1 = R + r;
    ws->bp_c1 = 2 * h1 + r;
    const uint32_t pw21 = (uint32_t)pow21(k - 1);
    ws->bp_local = ws->cur_used;
    const uint32_t nb = 1u << lay.bbits;
    if (ws->bp_local) e = ws->cur.reserve(nb);
    if (e != hipSuccess) return e;
    if (ws->defer_clear && !ws->bp_local) {  // no chunk descriptors on this path: the clear first
        step_clear_kernel<<<1, 256, 0, st>>>(ws->flags.p, ws->bstats.p, ws->clear_extra, ws->clear_n);
        ws->defer_clear = false;
    }
    if (ws->bp_local) {  // local level 1 for the cursor level 2: H1 (own digits) | H1T
        e = ws->chunk_desc.reserve(4ull * G);
        if (e != hipSuccess) return e;
        // descriptors + the cursor level 2's bucket counts cleared (bp_level2c does not)
        StepClear sc{};
        if (ws->defer_clear) {  // the front's clear, folded into this first kernel
            sc = StepClear{ws->flags.p, kFlN, ws->bstats.p, kShards * 10, ws->clear_extra, ws->clear_n};
            ws->defer_clear = false;
        }
        chunk_desc_kernel<<<(n + 1 + 255) / 256, 256, 0, st>>>(d_res_off, n, slots, G, k,
                                                               reinterpret_cast<uint4*>(ws->chunk_desc.p), ws->cur.p,
                                                               nb, sc);
        ws->bp_G = G;
        ws->bp_h1t = h1;
        // T chunks per level-2 tile: ~7/4 of a round at the hash-uniform mean (two rounds; kKeyChunk / nb1 keys
        // per chunk and bin)
        ws->bp_T = std::min<uint32_t>(kBpGatherMax, std::max<uint32_t>(1, kBpGatherTile * 7 / 4 * dg.nb1 / kKeyChunk));
        const uint32_t nown = dhi - dlo;
        // a few own bins (a rank's share of the k-mer split): level 2 reads the run table as level 1
        // wrote it (bp_hsc = own bins); otherwise transposed, so a bin's runs are contiguous
        const bool direct = nown <= 64 && nown < dg.nb1;
        ws->bp_hsb = direct ? 1u : G;
        ws->bp_hsc = direct ? nown : 1u;
        if (direct) ws->bp_h1t = 0;
        // persistent: as many workgroups as fit the device at once, each walking its chunks with the
        // next one's loads in flight
        static thread_local int per_cu = 0;
        if (!per_cu && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, bp_scatter1p_kernel<KMP_L1_THREADS>,
                                                                     KMP_L1_THREADS, 0) != hipSuccess ||
                        per_cu < 1))
            per_cu = 2;
        // every bin owned (one GPU): one workgroup per chunk, in order (bp_scatter1p 112 -> 103 us at
        // config 3); a share of the bins (a rank of the k-mer split, little work per chunk): persistent
#ifndef KMP_L1P_ALWAYS
#define KMP_L1P_ALWAYS 0  // A/B: the persistent grid on one GPU too
#endif
        const uint32_t grid = nown >= dg.nb1 && !KMP_L1P_ALWAYS ? G
                                                                 : std::min<uint32_t>(G, (uint32_t)per_cu * device_cus());
        if (nown) {
            bp_scatter1p_kernel<KMP_L1_THREADS><<<grid, KMP_L1_THREADS, 0, st>>>(
                d_res, d_res_off, d_class, k, n, slots, G, reinterpret_cast<const uint4*>(ws->chunk_desc.p), lay, dg,
                pw21, dlo, dhi, H1, ws->keys.p, ws->flags.p);
            if (!direct)
                bp_h1t_kernel<<<dim3((G + 31) / 32, (nown + 31) / 32), 256, 0, st>>>(H1, G, nown, 0, nown, H1 + h1);
        }
        return hipGetLastError();
    }
    chunk_first_kernel<<<(n + 1 + 255) / 256, 256, 0, st>>>(d_res_off, 0u, n, 0ull, slots, G, ws->chunk_first.p);
    bp_hist1_kernel<<<G, kKeyThreads, 0, st>>>(d_res, d_res_off, d_class, k, n, slots, ws->chunk_first.p, lay, dg,
                                                pw21, dlo, dhi, H1, ws->flags.p);
    bp_colsum_kernel<<<dim3(groups, (dg.nb1 + 255) / 256), 256, 0, st>>>(H1, G, dg.nb1, R);
    bp_colscan_kernel<<<1, kColThreads, 0, st>>>(R, groups, dg.nb1, C1);
    bp_colprefix_kernel<<<dim3(groups, (dg.nb1 + 255) / 256), 256, 0, st>>>(H1, G, dg.nb1, R, P1);
    bp_scatter1_kernel<<<G, kKeyThreads, 0, st>>>(d_res, d_res_off, d_class, k, n, slots, ws->chunk_first.p, lay, dg,
                                                   pw21, dlo, dhi, P1, ws->keys.p, ws->flags.p);
    return hipGetLastError();
}

// Level 2: ws->keys (level 1) -> ws->sorted grouped by bucket, bstart[0..nb] in ws->cnt.
int bp_level2(kmp_postings* ws, const Layout& lay, hipStream_t st) {
    const BpDigits dg = bp_digits(lay);
    uint32_t* C1 = ws->bp.p + ws->bp_c1;
    uint32_t* H2 = C1 + 2 * (dg.nb1 + 1);
    const uint32_t nb = 1u << lay.bbits, J = ws->bp_J;
    uint32_t c0, c1;
    own_bins(ws, dg, &c0, &c1);
    PG(ws->cnt.reserve(2 * (uint64_t)nb + 2));
    if (c1 > c0) {
        bp_hist2_kernel<<<dim3(J, c1 - c0), kKeyThreads, 0, st>>>(ws->keys.p, C1, J, dg, H2, c0);
        bp_scan2_kernel<<<c1 - c0, kKeyThreads, 0, st>>>(H2, C1, J, dg, ws->cnt.p, ws->flags.p, c0);
        bp_scatter2_kernel<<<dim3(J, c1 - c0), kKeyThreads, 0, st>>>(ws->keys.p, C1, J, dg, H2, ws->sorted.p, c0);
    }
    PG(hipGetLastError());
    return KMP_OK;
}

// Cursor level-2 geometry from the hash-uniform mean bucket; false when the region offsets
// would not fit the u32 arithmetic of the kernels
bool cur_geometry(const Layout& lay, CurGeom* cg) {
    const uint64_t nb = 1ull << lay.bbits;
    const uint64_t capb = (std::max<uint64_t>(2ull * lay.mean_keys + 512, 1536) + 63) / 64 * 64;
    if (nb * capb + capb >= (1ull << 32) - 2 * kBpTile) return false;
    cg->capb = (uint32_t)capb;
    cg->vreg = nullptr;  // the fixed layout (a residue call may switch to its learned one)
    return true;
}

// KMP_GATHER_THREADS: workgroup size of the level-2 gather (a 4,096-key round either way).  512
// threads x 8 keys (82 VGPRs, 6 waves per SIMD instead of 3) measured no faster at config 3
// (buckets_level2 0.159-0.164 ms vs 0.149-0.160 ms), so 256 x 16 stays
#ifndef KMP_GATHER_THREADS
#define KMP_GATHER_THREADS 256
#endif
// Level 2, cursor variant: ws->keys (level 1) -> the bucket regions of ws->sorted, counts in ws->cur.
int bp_level2c(kmp_postings* ws, const Layout& lay, hipStream_t st) {
    const BpDigits dg = bp_digits(lay);
    const uint32_t nb = 1u << lay.bbits;
    uint32_t* C1 = ws->bp.p + ws->bp_c1;
    PG(ws->cur.reserve(nb));
    PG(ws->sorted.reserve(ws->cg.vreg ? ws->vreg_total : (uint64_t)nb * ws->cg.capb));
    PG(ws->cnt.reserve(2 * (uint64_t)nb + 2));  // the large-bucket list
    uint32_t c0, c1;
    own_bins(ws, dg, &c0, &c1);
    if (!ws->bp_local)  // the local level 1 cleared the counts with its chunk_first
        bp_cur_clear_kernel<<<std::min<uint32_t>((nb + 1023) / 1024, 1024), 1024, 0, st>>>(ws->cur.p, nb);
    if (c1 > c0 && ws->bp_local) {
        const uint32_t ntiles = (ws->bp_G + ws->bp_T - 1) / ws->bp_T, per = (ntiles * (c1 - c0) + 7) / 8;
        constexpr uint32_t kGp = kBpGatherTile / KMP_GATHER_THREADS, kGt = KMP_GATHER_THREADS;
        if (ws->cg.vreg)
            bp_scatter2g_kernel<kGp, kGt, true><<<8 * per, kGt, 0, st>>>(
                ws->keys.p, ws->bp.p + ws->bp_h1t, ws->bp_G, ws->bp_hsb, ws->bp_hsc, ws->bp_T, ntiles, c1 - c0, dg, ws->cg,
                ws->cur.p, ws->sorted.p, ws->flags.p, c0, c0);
        else
            bp_scatter2g_kernel<kGp, kGt, false><<<8 * per, kGt, 0, st>>>(
                ws->keys.p, ws->bp.p + ws->bp_h1t, ws->bp_G, ws->bp_hsb, ws->bp_hsc, ws->bp_T, ntiles, c1 - c0, dg, ws->cg,
                ws->cur.p, ws->sorted.p, ws->flags.p, c0, c0);
    } else if (c1 > c0) {
        if (ws->cg.vreg)
            bp_scatter2c_kernel<true><<<dim3(ws->bp_J, c1 - c0), kKeyThreads, 0, st>>>(
                ws->keys.p, C1, ws->bp_J, dg, ws->cg, ws->cur.p, ws->sorted.p, ws->flags.p, c0);
        else
            bp_scatter2c_kernel<false><<<dim3(ws->bp_J, c1 - c0), kKeyThreads, 0, st>>>(
                ws->keys.p, C1, ws->bp_J, dg, ws->cg, ws->cur.p, ws->sorted.p, ws->flags.p, c0);
    }
    PG(hipGetLastError());
    return KMP_OK;
}

// Bucketed front: keys `in` grouped by bucket into ws->sorted, bstart[0..nb] in ws->cnt.  After
// bp_level1 (ws->parted) that is level 2; otherwise a radix sort on the bucket field and a binary
// search per bucket.  Marks 2 after the grouping.
int bucket_group(kmp_postings* ws, const unsigned long long* in, uint64_t slots, const Layout& lay, hipStream_t st) {
    const uint32_t nb = 1u << lay.bbits;
    PG(ws->sorted.reserve(slots));
    if (ws->parted && in == ws->keys.p) {
        ws->parted = false;
        int rc = ws->cur_used ? bp_level2c(ws, lay, st) : bp_level2(ws, lay, st);
        ws->mark(2, st);
        return rc;
    }
    size_t t_sort = 0;
    PG(rocprim::radix_sort_keys<SortCfg>(nullptr, t_sort, in, ws->sorted.p, (size_t)slots, lay.sort_lo, lay.sort_hi, st));
    PG(ws->tmp.reserve(std::max(t_sort, ws->tmp.n)));
    PG(rocprim::radix_sort_keys<SortCfg>(ws->tmp.p, t_sort, in, ws->sorted.p, (size_t)slots, lay.sort_lo, lay.sort_hi, st));
    ws->mark(2, st);
    PG(ws->cnt.reserve(2 * (uint64_t)nb + 2));
    bucket_bounds_kernel<<<(nb + 1 + 255) / 256, 256, 0, st>>>(ws->sorted.p, slots, lay.sort_lo, nb, ws->cnt.p);
    PG(hipGetLastError());
    return KMP_OK;
}

// Flat front end (keys already in ws->keys): stable code sort, count pass, offsets, write pass.
// Marks 2 (sort), 3 (count + offsets), 4 (write).  On return ws->inc holds *n_inc pair keys.
int front_flat(kmp_postings* ws, uint64_t slots, const Layout& lay, const uint16_t* d_class, uint32_t n,
               uint32_t heavy_df, int require_class_diff, unsigned long long* n_inc, kmp_postings_stats* stats,
               hipStream_t st) {
    size_t t_sort = 0;
    PG(rocprim::radix_sort_keys<SortCfg>(nullptr, t_sort, ws->keys.p, ws->sorted.p, (size_t)slots, lay.sort_lo, lay.sort_hi,
                                st));
    PG(ws->tmp.reserve(std::max(t_sort, ws->tmp.n)));
    PG(rocprim::radix_sort_keys<SortCfg>(ws->tmp.p, t_sort, ws->keys.p, ws->sorted.p, (size_t)slots, lay.sort_lo,
                                lay.sort_hi, st));
    ws->mark(2, st);

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
    fill_stats(stats, acc);
    *n_inc = acc[kStInc];
    if (*n_inc && *n_inc <= 0xFFFFFFFFull) {
        PG(ws->inc.reserve(*n_inc));
        if (lay.cls_in_key)
            expand_kernel<true, true><<<nb, kExpThreads, 0, st>>>(ws->sorted.p, slots, lay, d_class, n,
                                                                  require_class_diff, heavy_df, ws->cnt.p, nullptr,
                                                                  nullptr, ws->boff.p, ws->inc.p);
        else
            expand_kernel<true, false><<<nb, kExpThreads, 0, st>>>(ws->sorted.p, slots, lay, d_class, n,
                                                                   require_class_diff, heavy_df, ws->cnt.p, nullptr,
                                                                   nullptr, ws->boff.p, ws->inc.p);
    }
    ws->mark(4, st);
    return KMP_OK;
}

// ------------------------------------------------------------- row-block tail -------------
// combine_edges (mod.rs:322-546) without a global pair-key sort.  Pair keys are p << pbits | q
// (p < q); row block r = rows [row0 + (r << rbits), row0 + ((r + 1) << rbits)).
//   pt_hist     per 16,384-key tile of each shard region: row-block histogram added to the
//               totals T[r]
//   pt_tscan    one workgroup: block starts bst[r] and the scatter's cursors from T
//   pt_scatter  per tile: keys ranked by row block in LDS and written as u32
//               (p_local << pbits | q), one run per row block reserved on the block's cursor
//               (the former per-tile column scan, three kernels, gone: pair partition 0.043 -> 0.026 ms at config 3)
//   pt_reduce   one workgroup per row block: LDS radix sort of its keys (rocprim
//               block_radix_sort), run-length encode (run = one (p, q) pair, length = w), runs
//               with w >= min_shared staged at the block's input offset, kept-run count per block
//   pt_offsets  one workgroup: exclusive scan of the run counts -> edge offsets and the total
//   pt_emit     one workgroup per row block: staged runs -> (d_p, d_q, d_w) at its offset
// A row block above kPtCap keys (a protein pairing with thousands of later proteins: real data
// at k = 5) is listed instead; the host sorts the listed blocks with one segmented radix sort
// and pt_ovf_rle encodes them (pt_finish_overflow), then offsets and emit run again.
#ifndef KMP_PT_PER
#define KMP_PT_PER 16
#endif
#ifndef KMP_PT_RADIX_BITS
#define KMP_PT_RADIX_BITS 0  // rocprim's choice (8 bits, match ranking, at 512 threads)
#endif
constexpr uint32_t kPtThreads = 1024, kPtPer = KMP_PT_PER, kPtTile = kPtThreads * kPtPer;  // partition tiles: 16,384 keys
constexpr uint32_t kPtRThreads = 512, kPtCap = 8192;  // pt_reduce: up to 16 keys per thread
constexpr uint32_t kPtMaxBlocks = 8192;  // row blocks (LDS histogram of pt_hist / pt_scatter)


// The blocks a reduce runs over: row blocks (size == nullptr: block r is keys [start[r], start[r+1])
// of row block r) or sub-blocks (block d is keys [start[d], start[d] + size[d]) of row block row[d]:
// a row block above kPtCap cut by pt_split).
// A sub-block whose size has bit 31 set is a whole row block that fitted: its keys are read in place
// from whole (the row-block keys), not from the cut keys.
struct BlkSrc {
    const uint32_t* start;
    const uint32_t* size;
    const uint32_t* row;
    const uint32_t* whole;
};
constexpr uint32_t kBlkWhole = 0x80000000u;
__device__ __forceinline__ void blk_of(const BlkSrc& b, uint32_t i, uint32_t& s0, uint32_t& n, uint32_t& r) {
    s0 = b.start[i];
    if (b.size) {
        n = b.size[i] & ~kBlkWhole;
        r = b.row[i];
    } else {
        n = b.start[i + 1] - s0;
        r = i;
    }
}
// the keys block i reads (keys: the cut keys)
__device__ __forceinline__ const uint32_t* blk_keys(const BlkSrc& b, uint32_t i, const uint32_t* keys) {
    return b.size && (b.size[i] & kBlkWhole) ? b.whole : keys;
}

__device__ __forceinline__ uint32_t pt_tile_keys(const unsigned long long* __restrict__ cursor, const PtGeom& g,
                                                 uint32_t s, uint32_t j, uint32_t& t0) {
    const uint64_t ns = g.flat_n ? g.flat_n : min<unsigned long long>(cursor[s], g.sc);
    t0 = j * kPtTile;
    return t0 < ns ? (uint32_t)min<uint64_t>(kPtTile, ns - t0) : 0u;
}

// per 16,384-key tile of each shard region: its keys counted per row block in LDS and added to
// the row-block totals T (one global atomic per nonzero count)
__global__ __launch_bounds__(kPtThreads) void pt_hist_kernel(const unsigned long long* __restrict__ in,
                                                             const unsigned long long* __restrict__ cursor, PtGeom g,
                                                             uint32_t* __restrict__ T) {
    __shared__ uint32_t lh[kPtMaxBlocks];
    const uint32_t j = blockIdx.x, s = blockIdx.y;
    for (uint32_t r = threadIdx.x; r < g.nrb; r += kPtThreads) lh[r] = 0;
    __syncthreads();
    uint32_t t0;
    const uint32_t m = pt_tile_keys(cursor, g, s, j, t0);
    const unsigned long long* src = in + s * g.sc + t0;
    const unsigned sh = g.pbits + g.sbits + g.rbits;
    const unsigned long long base = (unsigned long long)g.row0 << (g.pbits + g.sbits);
    for (uint32_t i = threadIdx.x; i < m; i += kPtThreads) {
        const unsigned long long x = src[i];
        if (x != kNoKey) atomicAdd(&lh[(uint32_t)((x - base) >> sh)], 1u);
    }
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < g.nrb; r += kPtThreads)
        if (lh[r]) atomicAdd(&T[r], lh[r]);
}

constexpr int kPtScanThreads = 1024;
// row-block starts from the totals (one workgroup): bst[r] (bst[nrb] = total), the scatter's
// cursors cur[r] = bst[r], *colmax = the largest block; T is zeroed for the next step (it is
// zero when allocated, so pt_hist's atomics always start from zero)
__global__ __launch_bounds__(kPtScanThreads) void pt_tscan_kernel(uint32_t* __restrict__ T, uint32_t nrb,
                                                                  uint32_t* __restrict__ bst,
                                                                  uint32_t* __restrict__ cur,
                                                                  uint32_t* __restrict__ colmax) {
    __shared__ uint32_t wave_tot[kPtScanThreads / 64];
    __shared__ uint32_t s_max;
    if (threadIdx.x == 0) s_max = 0;
    const uint32_t q = (nrb + kPtScanThreads - 1) / kPtScanThreads, c0 = threadIdx.x * q;
    uint32_t v[8], sum = 0, mx = 0;
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) {
        v[i] = i < q && c0 + i < nrb ? T[c0 + i] : 0u;
        sum += v[i];
        mx = max(mx, v[i]);
    }
    __syncthreads();
    if (mx) atomicMax(&s_max, mx);
    uint32_t excl, total;
    block_scan_n<kPtScanThreads>(sum, excl, total, wave_tot);  // barriers: s_max complete
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i)
        if (i < q && c0 + i < nrb) {
            bst[c0 + i] = excl;
            cur[c0 + i] = excl;
            T[c0 + i] = 0;
            excl += v[i];
        }
    if (threadIdx.x == 0) {
        bst[nrb] = total;
        *colmax = s_max;
    }
}

// the tile's keys ranked by row block in LDS, each block's run reserved with one returning
// atomic on the block's cursor (order inside a block is free: pt_reduce sorts it), written as u32
// (p - r * 2^rbits) << pbits | q
__global__ __launch_bounds__(kPtThreads) void pt_scatter_kernel(const unsigned long long* __restrict__ in,
                                                                const unsigned long long* __restrict__ cursor,
                                                                PtGeom g, uint32_t* __restrict__ cur,
                                                                uint32_t* __restrict__ out) {
    __shared__ uint32_t lh[kPtMaxBlocks];
    __shared__ uint32_t S[kPtTile];
    __shared__ uint16_t SR[kPtTile];
    __shared__ uint32_t wave_tot[kPtThreads / 64];
    __shared__ uint32_t s_n;
    const uint32_t j = blockIdx.x, s = blockIdx.y;
    uint32_t t0;
    const uint32_t m = pt_tile_keys(cursor, g, s, j, t0);
    if (m == 0) return;
    for (uint32_t r = threadIdx.x; r < g.nrb; r += kPtThreads) lh[r] = 0;
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    const unsigned long long* src = in + s * g.sc + t0;
    const unsigned sh = g.pbits + g.sbits + g.rbits;
    const unsigned long long lowm = (1ull << sh) - 1;
    const unsigned long long base = (unsigned long long)g.row0 << (g.pbits + g.sbits);
    unsigned long long x[kPtPer];
    uint32_t rk[kPtPer];
#pragma unroll
    for (uint32_t e = 0; e < kPtPer; ++e) {
        const uint32_t i = threadIdx.x + e * kPtThreads;
        x[e] = i < m ? src[i] : kNoKey;
        if (x[e] != kNoKey) x[e] -= base;  // rows from row0
    }
    uint32_t nk = 0;
#pragma unroll
    for (uint32_t e = 0; e < kPtPer; ++e) {
        rk[e] = x[e] != kNoKey ? atomicAdd(&lh[(uint32_t)(x[e] >> sh)], 1u) : 0u;
        nk += x[e] != kNoKey;
    }
    if (nk) atomicAdd(&s_n, nk);
    __syncthreads();
    constexpr uint32_t kQ = kPtMaxBlocks / kPtThreads;
    uint32_t cnt[kQ];
#pragma unroll
    for (uint32_t t = 0; t < kQ; ++t) {
        const uint32_t r = threadIdx.x + t * kPtThreads;
        cnt[t] = r < g.nrb ? lh[r] : 0u;
    }
    lds_bins_scan<kPtThreads>(lh, g.nrb, wave_tot);
    uint32_t rbase[kQ];
#pragma unroll
    for (uint32_t t = 0; t < kQ; ++t)  // reserved while the tile is placed
        rbase[t] = cnt[t] ? atomicAdd(&cur[threadIdx.x + t * kPtThreads], cnt[t]) : 0u;
#pragma unroll
    for (uint32_t e = 0; e < kPtPer; ++e)
        if (x[e] != kNoKey) {
            const uint32_t r = (uint32_t)(x[e] >> sh), pos = lh[r] + rk[e];
            S[pos] = (uint32_t)(x[e] & lowm);
            SR[pos] = (uint16_t)r;
        }
    __syncthreads();
#pragma unroll
    for (uint32_t t = 0; t < kQ; ++t) {
        const uint32_t r = threadIdx.x + t * kPtThreads;
        if (r < g.nrb) lh[r] = rbase[t] - lh[r];
    }
    __syncthreads();
    const uint32_t placed = s_n;  // m counts the kNoKey padding of a flat array too
    for (uint32_t i = threadIdx.x; i < placed; i += kPtThreads) out[lh[SR[i]] + i] = S[i];
}

// The fast tail's scatter (pt_reduce_fast): a tile of kThr * 16 keys ranked by row block in LDS;
// cur[r] counts from zero and block r's keys go to the fixed region [r * ftcap, (r + 1) * ftcap)
// of out, written as u32 (p - r * 2^rbits) << pbits | q (keys past the region are dropped; the
// reduce sees the count and flags the overflow) — no histogram pass, no scan.  Workgroup (0, 0)
// also clears the reduce's look-back words lb[0, nrb).  Tiles of 8,192 keys: twice the workgroups
// of the counting tail's 16,384-key tiles (which ran one per CU), at LDS for two per CU.
constexpr uint32_t kFtCap = 8192;  // fast tail, hash reduce: keys per row-block region
constexpr uint32_t kFdBitsMax = 15;  // dense reduce: bins 2^(pbits + rbits)
constexpr uint32_t kFtScThreads = 512, kFtScTile = kFtScThreads * 16;
__global__ __launch_bounds__(kFtScThreads) void pt_scatter_capped_kernel(const unsigned long long* __restrict__ in,
                                                                         const unsigned long long* __restrict__ cursor,
                                                                         PtGeom g, uint32_t* __restrict__ cur,
                                                                         uint32_t* __restrict__ out,
                                                                         unsigned long long* __restrict__ lb) {
    constexpr uint32_t kThr = kFtScThreads, kPer = 16;
    __shared__ uint32_t lh[kPtMaxBlocks];
    __shared__ uint32_t S[kFtScTile];
    __shared__ uint16_t SR[kFtScTile];
    __shared__ uint32_t wave_tot[kThr / 64];
    __shared__ uint32_t s_n;
    const uint32_t j = blockIdx.x, s = blockIdx.y;
    if (j == 0 && s == 0)
        for (uint32_t r = threadIdx.x; r < g.nrb; r += kThr) lb[r] = 0;
    const uint64_t ns = g.flat_n ? g.flat_n : min<unsigned long long>(cursor[s], g.sc);
    const uint64_t t0 = (uint64_t)j * kFtScTile;
    if (t0 >= ns) return;
    const uint32_t m = (uint32_t)min<uint64_t>(kFtScTile, ns - t0);
    for (uint32_t r = threadIdx.x; r < g.nrb; r += kThr) lh[r] = 0;
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    const unsigned long long* src = in + s * g.sc + t0;
    const unsigned sh = g.pbits + g.rbits;
    const unsigned long long lowm = (1ull << sh) - 1;
    const unsigned long long base = (unsigned long long)g.row0 << g.pbits;
    unsigned long long x[kPer];
    uint32_t rk[kPer];
#pragma unroll
    for (uint32_t e = 0; e < kPer; ++e) {
        const uint32_t i = threadIdx.x + e * kThr;
        x[e] = i < m ? src[i] : kNoKey;
        if (x[e] != kNoKey) x[e] -= base;  // rows from row0
    }
    uint32_t nk = 0;
#pragma unroll
    for (uint32_t e = 0; e < kPer; ++e) {
        rk[e] = x[e] != kNoKey ? atomicAdd(&lh[(uint32_t)(x[e] >> sh)], 1u) : 0u;
        nk += x[e] != kNoKey;
    }
    if (nk) atomicAdd(&s_n, nk);
    __syncthreads();
    constexpr uint32_t kQ = kPtMaxBlocks / kThr;
    uint32_t cnt[kQ];
#pragma unroll
    for (uint32_t t = 0; t < kQ; ++t) {
        const uint32_t r = threadIdx.x + t * kThr;
        cnt[t] = r < g.nrb ? lh[r] : 0u;
    }
    lds_bins_scan<kThr>(lh, g.nrb, wave_tot);
    uint32_t rbase[kQ];
#pragma unroll
    for (uint32_t t = 0; t < kQ; ++t)  // reserved while the tile is placed
        rbase[t] = cnt[t] ? atomicAdd(&cur[threadIdx.x + t * kThr], cnt[t]) : 0u;
#pragma unroll
    for (uint32_t e = 0; e < kPer; ++e)
        if (x[e] != kNoKey) {
            const uint32_t r = (uint32_t)(x[e] >> sh), pos = lh[r] + rk[e];
            S[pos] = (uint32_t)(x[e] & lowm);
            SR[pos] = (uint16_t)r;
        }
    __syncthreads();
#pragma unroll
    for (uint32_t t = 0; t < kQ; ++t) {
        const uint32_t r = threadIdx.x + t * kThr;
        if (r < g.nrb) lh[r] = rbase[t] - lh[r];  // in-region offset of the tile's run, minus its staging start
    }
    __syncthreads();
    const uint32_t placed = s_n;
    for (uint32_t i = threadIdx.x; i < placed; i += kThr) {
        const uint32_t r = SR[i], pos = lh[r] + i;
        if (pos < g.ftcap) out[(uint64_t)r * g.ftcap + pos] = S[i];
    }
}

template <uint32_t kE>
using PtSort = rocprim::block_radix_sort<uint32_t, kPtRThreads, kE, rocprim::empty_type, 1, 1, KMP_PT_RADIX_BITS,
                                         KMP_PT_RADIX_BITS == 4
                                             ? rocprim::block_radix_rank_algorithm::basic_memoize
                                             : rocprim::block_radix_rank_algorithm::default_for_radix_sort>;

// Binned sort of a block's n keys (the row-block reduce; replaces a block radix sort over all
// pbits + rbits (+ sbits) key bits, 6-8 passes of rank + scatter).  A run only needs its pair's
// keys adjacent and the pairs in (row, q) order, so the keys are counted into nb >= 2n bins over
// the block's own pair range — the monotone position rl * span + (q - qlo), q in (rowbase, nprot),
// between its min and max (a sub-block covers a slice of it) — scattered to their bin's slice of
// S, and each bin (half a key on average) insertion-sorted by its thread on the pair (key >> sbits;
// the score field below it stays in arrival order).  A range of at most nb positions makes every
// bin one pair: no sort at all.  A bin above kBinMax keys (a skewed block) makes the caller fall
// back to the radix sort (k is untouched then).  On success k holds the sorted keys blocked
// (thread t: ranks t * kE + e), the padding (all ones) last.
constexpr uint32_t kBinMax = 64, kBinCap = 8192;
struct PtBinLds {
    uint32_t H[kBinCap];  // per bin: count, then first rank
    uint32_t S[kPtCap];   // the keys by bin
};
template <uint32_t kE>
__device__ __forceinline__ bool pt_bin_sort(uint32_t (&k)[kE], uint32_t n, const PtGeom& g, uint32_t rowbase,
                                            PtBinLds& b, uint32_t* red, uint32_t* s_flag, uint32_t* wave_tot) {
    constexpr uint32_t kT = kPtRThreads, kW = kT / 64;
    const unsigned sb = g.sbits, rs = g.pbits + g.sbits;
    const uint32_t qm = (1u << g.pbits) - 1, qlo = rowbase + 1;
    const uint32_t span = g.nprot > qlo ? g.nprot - qlo : 1u;
    auto pos = [&](uint32_t x) {
        const uint32_t q = (x >> sb) & qm;
        return (x >> rs) * span + (q > qlo ? q - qlo : 0u);
    };
    uint32_t lo = 0xFFFFFFFFu, hi = 0;
#pragma unroll
    for (uint32_t e = 0; e < kE; ++e)
        if (threadIdx.x + e * kT < n) {
            const uint32_t v = pos(k[e]);
            lo = min(lo, v);
            hi = max(hi, v);
        }
    for (int off = 32; off > 0; off >>= 1) {
        lo = min(lo, (uint32_t)__shfl_xor(lo, off));
        hi = max(hi, (uint32_t)__shfl_xor(hi, off));
    }
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6] = lo;
        red[kW + (threadIdx.x >> 6)] = hi;
    }
    uint32_t nb = 2;
    while (nb < 2 * n && nb < kBinCap) nb <<= 1;
    for (uint32_t i = threadIdx.x; i < nb; i += kT) b.H[i] = 0;
    if (threadIdx.x == 0) *s_flag = 0;
    __syncthreads();
#pragma unroll
    for (uint32_t w = 0; w < kW; ++w) {
        lo = min(lo, red[w]);
        hi = max(hi, red[kW + w]);
    }
    const uint64_t range = (uint64_t)hi - lo + 1;
    const bool exact = range <= nb;  // one pair per bin
    uint32_t br[kE];                 // bin | rank in it << 16 (bins, ranks < 2^14)
#pragma unroll
    for (uint32_t e = 0; e < kE; ++e) {
        br[e] = 0;
        if (threadIdx.x + e * kT < n) {
            const uint32_t v = pos(k[e]) - lo;
            const uint32_t bin = exact ? v : (uint32_t)((uint64_t)v * nb / range);
            br[e] = bin | atomicAdd(&b.H[bin], 1u) << 16;
        }
    }
    __syncthreads();
    lds_bins_scan<kT>(b.H, nb, wave_tot);  // H[bin] = its first rank
#pragma unroll
    for (uint32_t e = 0; e < kE; ++e)
        if (threadIdx.x + e * kT < n) b.S[b.H[br[e] & 0xFFFFu] + (br[e] >> 16)] = k[e];
    __syncthreads();
    if (!exact)
        for (uint32_t i = threadIdx.x; i < nb; i += kT) {
            const uint32_t a = b.H[i], e = i + 1 < nb ? b.H[i + 1] : n;
            if (e - a < 2) continue;
            if (e - a > kBinMax) {
                *s_flag = 1;
                continue;
            }
            for (uint32_t j = a + 1; j < e; ++j) {
                const uint32_t x = b.S[j], xp = x >> sb;
                uint32_t t = j;
                while (t > a && (b.S[t - 1] >> sb) > xp) {
                    b.S[t] = b.S[t - 1];
                    --t;
                }
                b.S[t] = x;
            }
        }
    __syncthreads();
    if (*s_flag) return false;  // (uniform) the radix sort on the untouched k
#pragma unroll
    for (uint32_t e = 0; e < kE; ++e) {
        const uint32_t rank = threadIdx.x * kE + e;
        k[e] = rank < n ? b.S[rank] : 0xFFFFFFFFu;
    }
    __syncthreads();  // S read before the caller reuses the LDS
    return true;
}

union PtReduceLds {
    typename PtSort<2>::storage_type s2;
    typename PtSort<4>::storage_type s4;
    typename PtSort<8>::storage_type s8;
    typename PtSort<16>::storage_type s16;
    PtBinLds b;
    uint32_t hs[kPtCap + 1];  // rank of each run's first key
};

// row block r's n keys (n <= kE * kPtRThreads): sort, run-length encode, stage the runs with
// w >= min_shared
template <uint32_t kE>
__device__ __forceinline__ void pt_reduce_block(PtReduceLds& u, typename PtSort<kE>::storage_type& st,
                                                uint32_t* last, uint32_t* wave_tot, const uint32_t* __restrict__ keys,
                                                uint32_t r, uint32_t s0, uint32_t n, const PtGeom& g,
                                                uint32_t* __restrict__ stage_p, uint32_t* __restrict__ stage_q,
                                                uint32_t* __restrict__ stage_w, uint32_t* __restrict__ counts) {
    uint32_t k[kE];
#pragma unroll
    for (uint32_t e = 0; e < kE; ++e) {
        const uint32_t i = threadIdx.x + e * kPtRThreads;
        k[e] = i < n ? keys[s0 + i] : 0xFFFFFFFFu;
    }
    // bits [0, pbits + rbits] (one above the key): the padding (all ones) sorts after every key
    if (!g.binsort || !pt_bin_sort<kE>(k, n, g, g.row0 + (r << g.rbits), u.b, last, last + 2 * kPtRThreads / 64, wave_tot))
        PtSort<kE>().sort(k, st, 0, g.pbits + g.rbits + 1);  // blocked: thread t holds ranks t*kE + e
    last[threadIdx.x] = k[kE - 1];
    __syncthreads();
    const uint32_t rank0 = threadIdx.x * kE;
    uint32_t prev = threadIdx.x ? last[threadIdx.x - 1] : 0u, nh = 0;
    bool head[kE];
#pragma unroll
    for (uint32_t e = 0; e < kE; ++e) {
        const uint32_t rank = rank0 + e;
        head[e] = rank < n && (rank == 0 || k[e] != prev);
        prev = k[e];
        nh += head[e];
    }
    uint32_t base, nruns;
    block_scan_n<kPtRThreads>(nh, base, nruns, wave_tot);  // barriers: the sort storage is dead
    const uint32_t qm = (1u << g.pbits) - 1;
    const uint32_t rowbase = g.row0 + (r << g.rbits);
    if (g.min_shared <= 1) {
        // heads write (p, q) from registers; w = the distance to the next run's first rank
#pragma unroll
        for (uint32_t e = 0; e < kE; ++e)
            if (head[e]) {
                u.hs[base] = rank0 + e;
                stage_p[s0 + base] = rowbase + (k[e] >> g.pbits);
                stage_q[s0 + base] = k[e] & qm;
                ++base;
            }
        if (threadIdx.x == 0) {
            u.hs[nruns] = n;
            counts[r] = nruns;
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < nruns; i += kPtRThreads) stage_w[s0 + i] = u.hs[i + 1] - u.hs[i];
        return;
    }
    // min_shared > 1: run keys staged in stage_p, then thread t keeps runs [t*kE, t*kE + kE) with
    // w >= min_shared, in order (every read lands before the scan's barriers, every write after)
#pragma unroll
    for (uint32_t e = 0; e < kE; ++e)
        if (head[e]) {
            u.hs[base] = rank0 + e;
            stage_p[s0 + base] = k[e];
            ++base;
        }
    if (threadIdx.x == 0) u.hs[nruns] = n;
    __syncthreads();
    uint32_t kv[kE], wv[kE], kept = 0;
#pragma unroll
    for (uint32_t e = 0; e < kE; ++e) {
        const uint32_t rr = rank0 + e;
        wv[e] = rr < nruns ? u.hs[rr + 1] - u.hs[rr] : 0u;
        kv[e] = rr < nruns ? stage_p[s0 + rr] : 0u;
        kept += wv[e] >= g.min_shared;
    }
    uint32_t o, total;
    block_scan_n<kPtRThreads>(kept, o, total, wave_tot);
#pragma unroll
    for (uint32_t e = 0; e < kE; ++e)
        if (wv[e] >= g.min_shared) {
            stage_p[s0 + o] = rowbase + (kv[e] >> g.pbits);
            stage_q[s0 + o] = kv[e] & qm;
            stage_w[s0 + o] = wv[e];
            ++o;
        }
    if (threadIdx.x == 0) counts[r] = total;
}

// one workgroup per row block; the sort width follows the block's size.  A block above kPtCap
// is listed in ovf (count in flags[3]) for pt_finish_overflow.
__global__ __launch_bounds__(kPtRThreads) void pt_reduce_kernel(const uint32_t* __restrict__ keys,
                                                                const uint32_t* __restrict__ bst, PtGeom g,
                                                                uint32_t* __restrict__ flags,
                                                                uint32_t* __restrict__ ovf,
                                                                uint32_t* __restrict__ stage_p,
                                                                uint32_t* __restrict__ stage_q,
                                                                uint32_t* __restrict__ stage_w,
                                                                uint32_t* __restrict__ counts) {
    __shared__ PtReduceLds u;
    __shared__ uint32_t last[kPtRThreads];
    __shared__ uint32_t wave_tot[kPtRThreads / 64];
    const uint32_t r = blockIdx.x, s0 = bst[r], n = bst[r + 1] - s0;
    if (n == 0 || n > kPtCap) {
        if (threadIdx.x == 0) {
            counts[r] = 0;
            if (n) ovf[atomicAdd(&flags[3], 1u)] = r;
        }
        return;
    }
    if (n <= 2 * kPtRThreads)
        pt_reduce_block<2>(u, u.s2, last, wave_tot, keys, r, s0, n, g, stage_p, stage_q, stage_w, counts);
    else if (n <= 4 * kPtRThreads)
        pt_reduce_block<4>(u, u.s4, last, wave_tot, keys, r, s0, n, g, stage_p, stage_q, stage_w, counts);
    else if (n <= 8 * kPtRThreads)
        pt_reduce_block<8>(u, u.s8, last, wave_tot, keys, r, s0, n, g, stage_p, stage_q, stage_w, counts);
    else
        pt_reduce_block<16>(u, u.s16, last, wave_tot, keys, r, s0, n, g, stage_p, stage_q, stage_w, counts);
}

// Scored row blocks (g.sbits > 0): the keys are (p_local << pbits | q) << sbits | field, field =
// s(x) (low kScoreBits bits) | k bit; a run is one (p, q) pair (equal key >> sbits), w = its length,
// score = Σ s over it (an exclusive block scan of the fields: run score = the scan at the next
// run's head minus the scan at its own), w1 = the run's marked entries (kbit: the second k of
// kmp_pairs_multi_k's fused union).  min_shared keeps a run when its w (single k) or either k's
// count (multi-k: w - w1, w1) reaches it.
template <bool kKbit>
struct PtScoredLds {
    union {
        typename PtSort<2>::storage_type s2;
        typename PtSort<4>::storage_type s4;
        typename PtSort<8>::storage_type s8;
        typename PtSort<16>::storage_type s16;
        PtBinLds b;
        struct {
            uint32_t hs[kPtCap + 1];  // rank of each run's first key | k-bit scan at it << 16 (kKbit)
            uint32_t ps[kPtCap + 1];  // score scan at each run's head
        } r;
    };
};

template <uint32_t kE, bool kKbit>
__device__ __forceinline__ void pt_reduce_scored_block(PtScoredLds<kKbit>& u, typename PtSort<kE>::storage_type& st,
                                                       uint32_t* last, uint32_t* wave_tot,
                                                       const uint32_t* __restrict__ keys, uint32_t r, uint32_t d,
                                                       uint32_t s0, uint32_t n, const PtGeom& g,
                                                       uint32_t* __restrict__ stage_p,
                                                       uint32_t* __restrict__ stage_q, uint32_t* __restrict__ stage_w,
                                                       uint32_t* __restrict__ stage_s, uint32_t* __restrict__ stage_w1,
                                                       uint32_t* __restrict__ counts) {
    uint32_t k[kE];
#pragma unroll
    for (uint32_t e = 0; e < kE; ++e) {
        const uint32_t i = threadIdx.x + e * kPtRThreads;
        k[e] = i < n ? keys[s0 + i] : 0xFFFFFFFFu;
    }
    const unsigned sb = g.sbits;
    if (!g.binsort || !pt_bin_sort<kE>(k, n, g, g.row0 + (r << g.rbits), u.b, last, last + 2 * kPtRThreads / 64, wave_tot))
        PtSort<kE>().sort(k, st, 0, g.pbits + sb + g.rbits + 1);  // blocked: thread t holds ranks t*kE + e
    last[threadIdx.x] = k[kE - 1] >> sb;
    __syncthreads();
    const uint32_t rank0 = threadIdx.x * kE;
    const uint32_t smask = (1u << kScoreBits) - 1;
    uint32_t prev = threadIdx.x ? last[threadIdx.x - 1] : 0u, nh = 0, ssum = 0, ksum = 0;
    bool head[kE];
#pragma unroll
    for (uint32_t e = 0; e < kE; ++e) {
        const uint32_t rank = rank0 + e, pk = k[e] >> sb;
        head[e] = rank < n && (rank == 0 || pk != prev);
        prev = pk;
        nh += head[e];
        if (rank < n) {
            ssum += k[e] & smask;
            if (kKbit) ksum += (k[e] >> kScoreBits) & 1u;
        }
    }
    uint32_t base, nruns, sx, stot, kx = 0, ktot = 0;
    block_scan_n<kPtRThreads>(nh, base, nruns, wave_tot);  // barriers: the sort storage is dead
    block_scan_n<kPtRThreads>(ssum, sx, stot, wave_tot);
    if (kKbit) block_scan_n<kPtRThreads>(ksum, kx, ktot, wave_tot);
    const uint32_t qm = (1u << g.pbits) - 1;
    const uint32_t rowbase = g.row0 + (r << g.rbits);
    const bool filter = g.min_shared > 1;
#pragma unroll
    for (uint32_t e = 0; e < kE; ++e) {
        if (head[e]) {
            const uint32_t pk = k[e] >> sb;
            u.r.hs[base] = (rank0 + e) | (kKbit ? kx << 16 : 0u);
            u.r.ps[base] = sx;
            stage_p[s0 + base] = filter ? pk : rowbase + (pk >> g.pbits);
            if (!filter) stage_q[s0 + base] = pk & qm;
            ++base;
        }
        if (rank0 + e < n) {
            sx += k[e] & smask;
            if (kKbit) kx += (k[e] >> kScoreBits) & 1u;
        }
    }
    if (threadIdx.x == 0) {
        u.r.hs[nruns] = n | (kKbit ? ktot << 16 : 0u);
        u.r.ps[nruns] = stot;
        if (!filter) counts[d] = nruns;
    }
    __syncthreads();
    if (!filter) {
        for (uint32_t i = threadIdx.x; i < nruns; i += kPtRThreads) {
            const uint32_t h0 = u.r.hs[i], h1 = u.r.hs[i + 1];
            stage_w[s0 + i] = (h1 & 0xFFFFu) - (h0 & 0xFFFFu);
            stage_s[s0 + i] = u.r.ps[i + 1] - u.r.ps[i];
            if (kKbit) stage_w1[s0 + i] = (h1 >> 16) - (h0 >> 16);
        }
        return;
    }
    // min_shared > 1: thread t keeps runs [t*kE, t*kE + kE) in order (reads before the scan's
    // barriers, writes after)
    uint32_t kv[kE], wv[kE], sv[kE], w1v[kE], kept = 0;
#pragma unroll
    for (uint32_t e = 0; e < kE; ++e) {
        const uint32_t rr = rank0 + e;
        const bool in = rr < nruns;
        const uint32_t h0 = in ? u.r.hs[rr] : 0u, h1 = in ? u.r.hs[rr + 1] : 0u;
        wv[e] = in ? (h1 & 0xFFFFu) - (h0 & 0xFFFFu) : 0u;
        sv[e] = in ? u.r.ps[rr + 1] - u.r.ps[rr] : 0u;
        w1v[e] = in && kKbit ? (h1 >> 16) - (h0 >> 16) : 0u;
        kv[e] = in ? stage_p[s0 + rr] : 0u;
        const bool keep = in && (kKbit ? (wv[e] - w1v[e] >= g.min_shared || w1v[e] >= g.min_shared)
                                       : wv[e] >= g.min_shared);
        if (!keep) wv[e] = 0;
        kept += keep;
    }
    uint32_t o, total;
    block_scan_n<kPtRThreads>(kept, o, total, wave_tot);
#pragma unroll
    for (uint32_t e = 0; e < kE; ++e)
        if (wv[e]) {
            stage_p[s0 + o] = rowbase + (kv[e] >> g.pbits);
            stage_q[s0 + o] = kv[e] & qm;
            stage_w[s0 + o] = wv[e];
            stage_s[s0 + o] = sv[e];
            if (kKbit) stage_w1[s0 + o] = w1v[e];
            ++o;
        }
    if (threadIdx.x == 0) counts[d] = total;
}

template <bool kKbit>
__global__ __launch_bounds__(kPtRThreads) void pt_reduce_scored_kernel(const uint32_t* __restrict__ keys,
                                                                       BlkSrc bs, PtGeom g,
                                                                       uint32_t* __restrict__ flags,
                                                                       uint32_t* __restrict__ ovf,
                                                                       uint32_t* __restrict__ stage_p,
                                                                       uint32_t* __restrict__ stage_q,
                                                                       uint32_t* __restrict__ stage_w,
                                                                       uint32_t* __restrict__ stage_s,
                                                                       uint32_t* __restrict__ stage_w1,
                                                                       uint32_t* __restrict__ counts) {
    __shared__ PtScoredLds<kKbit> u;
    __shared__ uint32_t last[kPtRThreads];
    __shared__ uint32_t wave_tot[kPtRThreads / 64];
    const uint32_t d = blockIdx.x;
    uint32_t s0, n, r;
    blk_of(bs, d, s0, n, r);
    if (n == 0 || n > kPtCap) {
        if (threadIdx.x == 0) {
            counts[d] = 0;
            if (n) ovf[atomicAdd(&flags[3], 1u)] = d;
        }
        return;
    }
    const uint32_t* kp = blk_keys(bs, d, keys);
#define PT_SCORED(E, S) \
    pt_reduce_scored_block<E, kKbit>(u, u.S, last, wave_tot, kp, r, d, s0, n, g, stage_p, stage_q, stage_w, stage_s, \
                                     stage_w1, counts)
    if (n <= 2 * kPtRThreads) PT_SCORED(2, s2);
    else if (n <= 4 * kPtRThreads) PT_SCORED(4, s4);
    else if (n <= 8 * kPtRThreads) PT_SCORED(8, s8);
    else PT_SCORED(16, s16);
#undef PT_SCORED
}

// Row blocks above kPtCap (listed by pt_reduce): their keys, tagged with the list index j as
// j << kb | key (kb = pbits + rbits key bits), are sorted together by one device-wide radix
// sort and run-length encoded; each run (one (p, q) pair of block ovf[j], length w) is staged at
// its block's offset.  Every step is multi-workgroup, so one very long row (real data at k = 5:
// a protein sharing 5-mers with thousands of later ones) costs a sort of its keys, not one
// workgroup walking them.
__global__ void pt_ovf_sizes_kernel(const uint32_t* __restrict__ ovf, uint32_t m, BlkSrc bs,
                                    unsigned long long* __restrict__ sz) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) {
        uint32_t s0, n, r;
        blk_of(bs, ovf[j], s0, n, r);
        sz[j] = n;
    }
    if (j == m) sz[m] = 0;
}

// one workgroup per listed block: its keys, tagged, at xoff[j]
__global__ __launch_bounds__(256) void pt_ovf_gather_kernel(const uint32_t* __restrict__ ovf, BlkSrc bs,
                                                            const unsigned long long* __restrict__ xoff,
                                                            const uint32_t* __restrict__ keys, unsigned kb,
                                                            unsigned long long* __restrict__ x) {
    const uint32_t j = blockIdx.y;
    uint32_t s0, n, r;
    blk_of(bs, ovf[j], s0, n, r);
    const unsigned long long tag = (unsigned long long)j << kb, o = xoff[j];
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) x[o + i] = tag | keys[s0 + i];
}

// per run: kept (w >= min_shared) -> keep[u]; a run of a new block records the block's first run
__global__ void pt_ovf_keep_kernel(const unsigned long long* __restrict__ uniq, const uint32_t* __restrict__ w,
                                   const uint32_t* __restrict__ nruns, unsigned kb, uint32_t min_shared,
                                   uint32_t* __restrict__ keep, uint32_t* __restrict__ first) {
    const uint32_t U = *nruns;
    for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u <= U; u += gridDim.x * blockDim.x) {
        if (u == U) {
            keep[u] = 0;
            continue;
        }
        keep[u] = w[u] >= min_shared;
        const uint32_t j = (uint32_t)(uniq[u] >> kb);
        if (u == 0 || (uint32_t)(uniq[u - 1] >> kb) != j) first[j] = u;
    }
}

// kept runs -> stage at the block's offset; counts[ovf[j]] = the block's kept runs
__global__ void pt_ovf_stage_kernel(const uint32_t* __restrict__ ovf, uint32_t m, const uint32_t* __restrict__ bst,
                                    PtGeom g, const unsigned long long* __restrict__ uniq,
                                    const uint32_t* __restrict__ w, const uint32_t* __restrict__ nruns,
                                    const uint32_t* __restrict__ kpos, const uint32_t* __restrict__ first,
                                    uint32_t* __restrict__ stage_p, uint32_t* __restrict__ stage_q,
                                    uint32_t* __restrict__ stage_w, uint32_t* __restrict__ counts) {
    const uint32_t U = *nruns;
    const unsigned kb = g.pbits + g.rbits;
    const uint32_t qm = (1u << g.pbits) - 1;
    for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < U; u += gridDim.x * blockDim.x) {
        const unsigned long long x = uniq[u];
        const uint32_t j = (uint32_t)(x >> kb), r = ovf[j];
        const uint32_t f = first[j];
        const uint32_t nxt = j + 1 < m ? first[j + 1] : U;  // every listed block holds a run
        if (u == f) counts[r] = kpos[nxt] - kpos[f];
        if (w[u] < g.min_shared) continue;
        const uint32_t key = (uint32_t)x & ((1u << kb) - 1), o = bst[r] + kpos[u] - kpos[f];
        stage_p[o] = g.row0 + (r << g.rbits) + (key >> g.pbits);
        stage_q[o] = key & qm;
        stage_w[o] = w[u];
    }
}

// scored listed blocks: runs of equal pair (tagged key >> sbits), reduced to (w, w1, score)
struct RunAgg {
    uint32_t w, w1, s;
};
struct RunAggPlus {
    __host__ __device__ RunAgg operator()(const RunAgg& a, const RunAgg& b) const {
        return RunAgg{a.w + b.w, a.w1 + b.w1, a.s + b.s};
    }
};
struct PairOfKey {  // tagged scored key -> tagged pair
    unsigned sb;
    __host__ __device__ unsigned long long operator()(unsigned long long x) const { return x >> sb; }
};
struct AggOfKey {  // tagged scored key -> one entry's (1, k bit, s)
    __host__ __device__ RunAgg operator()(unsigned long long x) const {
        return RunAgg{1u, (uint32_t)(x >> kScoreBits) & 1u, (uint32_t)x & ((1u << kScoreBits) - 1)};
    }
};

__global__ void pt_ovf_keep_scored_kernel(const unsigned long long* __restrict__ uniq, const RunAgg* __restrict__ agg,
                                          const uint32_t* __restrict__ nruns, unsigned kb, uint32_t min_shared,
                                          int kbit, uint32_t* __restrict__ keep, uint32_t* __restrict__ first) {
    const uint32_t U = *nruns;
    for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u <= U; u += gridDim.x * blockDim.x) {
        if (u == U) {
            keep[u] = 0;
            continue;
        }
        const RunAgg a = agg[u];
        keep[u] = kbit ? (a.w - a.w1 >= min_shared || a.w1 >= min_shared) : a.w >= min_shared;
        const uint32_t j = (uint32_t)(uniq[u] >> kb);
        if (u == 0 || (uint32_t)(uniq[u - 1] >> kb) != j) first[j] = u;
    }
}

__global__ void pt_ovf_stage_scored_kernel(const uint32_t* __restrict__ ovf, uint32_t m, BlkSrc bs, PtGeom g,
                                           const unsigned long long* __restrict__ uniq,
                                           const RunAgg* __restrict__ agg, const uint32_t* __restrict__ nruns,
                                           const uint32_t* __restrict__ keep, const uint32_t* __restrict__ kpos,
                                           const uint32_t* __restrict__ first, uint32_t* __restrict__ stage_p,
                                           uint32_t* __restrict__ stage_q, uint32_t* __restrict__ stage_w,
                                           uint32_t* __restrict__ stage_s, uint32_t* __restrict__ stage_w1,
                                           uint32_t* __restrict__ counts) {
    const uint32_t U = *nruns;
    const unsigned kb = g.pbits + g.rbits;  // the tag above the (unscored) pair key
    const uint32_t qm = (1u << g.pbits) - 1;
    for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < U; u += gridDim.x * blockDim.x) {
        const unsigned long long x = uniq[u];
        const uint32_t j = (uint32_t)(x >> kb), d = ovf[j];
        uint32_t s0, n, r;
        blk_of(bs, d, s0, n, r);
        const uint32_t f = first[j];
        const uint32_t nxt = j + 1 < m ? first[j + 1] : U;
        if (u == f) counts[d] = kpos[nxt] - kpos[f];
        if (!keep[u]) continue;
        const RunAgg a = agg[u];
        const uint32_t key = (uint32_t)x & ((1u << kb) - 1), o = s0 + kpos[u] - kpos[f];
        stage_p[o] = g.row0 + (r << g.rbits) + (key >> g.pbits);
        stage_q[o] = key & qm;
        stage_w[o] = a.w;
        stage_s[o] = a.s;
        if (g.kbit) stage_w1[o] = a.w1;
    }
}

// Sub-blocks (the fused multi-k tail): a row block above kPtCap keys — config 5 at k = 5, where one
// protein pairs with ~10^5 later ones — is cut into sub-blocks of at most about kPtCap keys, each
// reduced in LDS like a row block, so no device-wide sort of the pass's keys is needed.  One
// 1,024-thread workgroup per row block: the keys are counted into nf fine bins over the block's
// pair range in (row in block, q) order — the linear position rl * span + (q - qlo), q in
// (rowbase, n) — the bins scanned, and sub-block j takes the bins whose first key lies in
// [j * kSbChunk, (j + 1) * kSbChunk): a monotone cut (canonical order kept) whose pieces are
// balanced whatever the q distribution (cutting by the key's top bits left late passes, whose q
// all share their top bits, in one piece).  Descriptors: nf per block (the unused ones empty);
// the keys scattered to keys2 at their bin's cursor.  A block that fits is one sub-block (copied);
// a sub-block still above kPtCap (one bin above kPtCap - kSbChunk keys) takes the overflow sort.
constexpr uint32_t kSbThreads = 1024, kSbMaxLog = 13, kSbChunk = kPtCap * 3 / 4;  // 64 KB of LDS: 2 workgroups per CU
__host__ __device__ inline unsigned pt_sub_log(uint32_t n) {
    if (n <= kPtCap) return 0;
    unsigned j = 1;  // nf * kSbChunk >= 4n: a bin holds a quarter of a sub-block on average
    while (j < kSbMaxLog && ((uint64_t)kSbChunk << j) < 4ull * n) ++j;
    return j;
}
// descriptor slots of a row block of n keys: sub-block j holds the bins whose first key lies in
// [j kSbChunk, (j + 1) kSbChunk), so at most ceil(n / kSbChunk) (not one per fine bin: at config 5
// that left ~80 % of the sub-blocks empty, 1.9M a pass)
__host__ __device__ inline uint32_t pt_sub_slots(uint32_t n) {
    return pt_sub_log(n) ? (n + kSbChunk - 1) / kSbChunk : 1u;
}

__global__ __launch_bounds__(kSbThreads) void pt_split_kernel(const uint32_t* __restrict__ keys,
                                                              const uint32_t* __restrict__ bst,
                                                              const uint32_t* __restrict__ dbase, PtGeom g,
                                                              uint32_t n_prot, uint32_t row_end,
                                                              uint32_t* __restrict__ keys2,
                                                              uint32_t* __restrict__ dstart,
                                                              uint32_t* __restrict__ dsize,
                                                              uint32_t* __restrict__ drow,
                                                              uint32_t* __restrict__ ovl) {
    __shared__ uint32_t cnt[1u << kSbMaxLog];  // per bin: count, then first key (local), then cursor
    __shared__ uint32_t lst[1u << kSbMaxLog];  // per sub-block: first key (local)
    __shared__ uint32_t wave_tot[kSbThreads / 64];
    const uint32_t r = blockIdx.x, s0 = bst[r], n = bst[r + 1] - s0;
    const unsigned lj = pt_sub_log(n);
    const uint32_t nf = 1u << lj, d0 = dbase[r], ns = pt_sub_slots(n);
    if (lj == 0) {  // fits: one sub-block, read in place (kBlkWhole)
        if (threadIdx.x == 0) {
            dstart[d0] = s0;
            dsize[d0] = n | kBlkWhole;
            drow[d0] = r;
        }
        return;
    }
    const uint32_t rowbase = g.row0 + (r << g.rbits);
    const uint32_t rows = min(1u << g.rbits, row_end > rowbase ? row_end - rowbase : 1u);
    const uint32_t qlo = rowbase + 1;  // q > p >= rowbase
    const uint64_t span = n_prot > qlo ? n_prot - qlo : 1u, range = (uint64_t)rows * span;
    const unsigned rs = g.pbits + g.sbits;
    const uint32_t qm = (1u << g.pbits) - 1;
    auto bin = [&](uint32_t k) -> uint32_t {
        const uint32_t q = (k >> g.sbits) & qm;
        const uint64_t pos = (uint64_t)(k >> rs) * span + (q > qlo ? q - qlo : 0u);
        return (uint32_t)min<uint64_t>(pos * nf / range, nf - 1);
    };
    for (uint32_t i = threadIdx.x; i < nf; i += kSbThreads) cnt[i] = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += kSbThreads) atomicAdd(&cnt[bin(keys[s0 + i])], 1u);
    __syncthreads();
    lds_bins_scan<kSbThreads>(cnt, nf, wave_tot);  // cnt[i] = first key of bin i
    // sub-block of bin i: cnt[i] / kSbChunk (monotone); sub-block j starts at the first bin whose
    // sub-block is >= j (a skipped j — one bin above kSbChunk — is empty)
    const uint32_t used = cnt[nf - 1] / kSbChunk + 1;
    for (uint32_t i = threadIdx.x; i < nf; i += kSbThreads) {
        const uint32_t sj = cnt[i] / kSbChunk;
        for (uint32_t j = i ? cnt[i - 1] / kSbChunk + 1 : 0u; j <= sj; ++j) lst[j] = cnt[i];
    }
    for (uint32_t j = used + threadIdx.x; j < nf; j += kSbThreads) lst[j] = n;
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < ns; j += kSbThreads) {
        const uint32_t a = lst[j], e = j + 1 < ns ? lst[j + 1] : n;
        dstart[d0 + j] = s0 + a;
        dsize[d0 + j] = e - a;
        drow[d0 + j] = r;
        if (e - a > kPtCap) ovl[1 + atomicAdd(&ovl[0], 1u)] = d0 + j;  // above the LDS sort: listed
    }
    for (uint32_t i = threadIdx.x; i < n; i += kSbThreads) {  // a bin's keys stay inside its sub-block
        const uint32_t k = keys[s0 + i];
        keys2[s0 + atomicAdd(&cnt[bin(k)], 1u)] = k;
    }
}

// Listed blocks whose key space is small (rbits + pbits <= 15: the next call's geometry after a
// first overflow — one or two rows per block, e.g. a protein sharing 5-mers with thousands of
// later ones): a histogram over the key (row in block, q) in LDS is the run-length encoding,
// already in canonical order.  One workgroup per listed block (grid-stride over the device
// count); no sort, no host round trip.
constexpr uint32_t kRowHistBits = 15, kRowHistBins = 1u << kRowHistBits, kRowHistThreads = 1024, kRowHistGrid = 64;
__host__ __device__ inline bool pt_rowhist_ok(const PtGeom& g) { return !g.sbits && g.rbits + g.pbits <= kRowHistBits; }

__global__ __launch_bounds__(kRowHistThreads) void pt_rowhist_kernel(const uint32_t* __restrict__ keys,
                                                                     const uint32_t* __restrict__ bst, PtGeom g,
                                                                     const uint32_t* __restrict__ flags,
                                                                     const uint32_t* __restrict__ ovf,
                                                                     uint32_t* __restrict__ stage_p,
                                                                     uint32_t* __restrict__ stage_q,
                                                                     uint32_t* __restrict__ stage_w,
                                                                     uint32_t* __restrict__ counts) {
    __shared__ uint32_t hist[kRowHistBins];  // 128 KB: one workgroup per CU
    __shared__ uint32_t wave_tot[kRowHistThreads / 64];
    const uint32_t m = flags[kFlOvf], nk = 1u << (g.rbits + g.pbits), km = nk - 1, qm = (1u << g.pbits) - 1;
    constexpr uint32_t kQ = kRowHistBins / kRowHistThreads;
    for (uint32_t j = blockIdx.x; j < m; j += gridDim.x) {
        const uint32_t r = ovf[j], s0 = bst[r], n = bst[r + 1] - s0;
        __syncthreads();  // the previous block's compaction has read hist
        for (uint32_t x = threadIdx.x; x < nk; x += kRowHistThreads) hist[x] = 0;
        __syncthreads();
        // loads in batches of 8 ahead of their atomics (one workgroup walks the whole block)
        for (uint32_t i0 = 0; i0 < n; i0 += 8 * kRowHistThreads) {
            uint32_t v[8];
#pragma unroll
            for (uint32_t e = 0; e < 8; ++e) {
                const uint32_t i = i0 + e * kRowHistThreads + threadIdx.x;
                v[e] = i < n ? keys[s0 + i] : ~0u;
            }
#pragma unroll
            for (uint32_t e = 0; e < 8; ++e)
                if (v[e] != ~0u) atomicAdd(&hist[v[e] & km], 1u);
        }
        __syncthreads();
        // thread t: keys [t * kQ, t * kQ + kQ), kept runs (w >= min_shared) in key order
        const uint32_t x0 = threadIdx.x * kQ;
        uint32_t kept = 0;
#pragma unroll
        for (uint32_t e = 0; e < kQ; ++e) {
            const uint32_t w = x0 + e < nk ? hist[x0 + e] : 0u;
            kept += w != 0 && w >= g.min_shared;
        }
        uint32_t o, total;
        block_scan_n<kRowHistThreads>(kept, o, total, wave_tot);
        const uint32_t rowbase = g.row0 + (r << g.rbits);
#pragma unroll
        for (uint32_t e = 0; e < kQ; ++e) {
            const uint32_t x = x0 + e, w = x < nk ? hist[x] : 0u;
            if (w != 0 && w >= g.min_shared) {
                stage_p[s0 + o] = rowbase + (x >> g.pbits);
                stage_q[s0 + o] = x & qm;
                stage_w[s0 + o] = w;
                ++o;
            }
        }
        if (threadIdx.x == 0) counts[r] = total;
    }
}

// exclusive scan of the nrb run counts (nrb <= 8 * 1024) -> eoff; eoff[nrb] and *total = edges
__global__ __launch_bounds__(kPtScanThreads) void pt_offsets_kernel(const uint32_t* __restrict__ counts, uint32_t nrb,
                                                                    uint32_t* __restrict__ eoff,
                                                                    uint32_t* __restrict__ total,
                                                                    unsigned long long* __restrict__ total64 = nullptr) {
    __shared__ uint32_t wave_tot[kPtScanThreads / 64];
    const uint32_t q = (nrb + kPtScanThreads - 1) / kPtScanThreads, c0 = threadIdx.x * q;
    uint32_t v[8], sum = 0;
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) {
        v[i] = i < q && c0 + i < nrb ? counts[c0 + i] : 0u;
        sum += v[i];
    }
    uint32_t excl, tot;
    block_scan_n<kPtScanThreads>(sum, excl, tot, wave_tot);
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i)
        if (i < q && c0 + i < nrb) {
            eoff[c0 + i] = excl;
            excl += v[i];
        }
    if (threadIdx.x == 0) {
        eoff[nrb] = tot;
        *total = tot;
        if (total64) *total64 = tot;
    }
}

__device__ void step_pack_body(const unsigned long long* __restrict__ gstats, const uint32_t* __restrict__ flags,
                               const uint32_t* __restrict__ runs, unsigned long long* __restrict__ rb,
                               unsigned long long fast_ovf = 0);

// pack: nonzero -> workgroup 0 also writes the step's read-back (step_pack_kernel's work: every
// input of it is final once pt_offsets has run)
struct PtPack {
    const unsigned long long* gstats;
    const uint32_t* flags;
    const uint32_t* runs;
    unsigned long long* rb;
};

// scored calls: the staged scores / second-k weights and where they go (d_w1 nullptr: single k)
struct PtScoreOut {
    const uint32_t* stage_s;
    const uint32_t* stage_w1;
    uint32_t* d_s;
    uint32_t* d_w1;
    uint32_t* d_w0;  // multi-k: w of the first k (w - w1)
};

__global__ __launch_bounds__(256) void pt_emit_kernel(const uint32_t* __restrict__ stage_p,
                                                      const uint32_t* __restrict__ stage_q,
                                                      const uint32_t* __restrict__ stage_w,
                                                      const uint32_t* __restrict__ bst,
                                                      const uint32_t* __restrict__ counts,
                                                      const uint32_t* __restrict__ eoff, uint32_t* __restrict__ d_p,
                                                      uint32_t* __restrict__ d_q, uint32_t* __restrict__ d_w,
                                                      uint64_t cap, uint32_t stride = 1, PtPack pack = {},
                                                      uint32_t* __restrict__ total_out = nullptr,
                                                      PtScoreOut so = {}) {
    const uint32_t r = blockIdx.x, s0 = bst[r], m = counts[r];
    uint64_t o;
    if (eoff) {
        o = eoff[r];
    } else {
        // no pt_offsets: this block's offset = the runs of the blocks before it (block 0: the
        // total, for the read-back)
        __shared__ uint32_t wave_tot[256 / 64];
        const uint32_t lim = r ? r : gridDim.x;
        uint32_t v = 0;
        for (uint32_t i = threadIdx.x; i < lim; i += 256) v += counts[i];
        uint32_t excl, tot;
        block_scan_n<256>(v, excl, tot, wave_tot);
        o = r ? tot : 0u;
        if (r == 0 && threadIdx.x == 0) *total_out = tot;
        if (r == 0) __syncthreads();  // the total is in memory before the pack reads it
    }
    if (pack.rb && blockIdx.x == 0) step_pack_body(pack.gstats, pack.flags, pack.runs, pack.rb);
    for (uint32_t i = threadIdx.x; i < m; i += 256) {
        if (o + i >= cap) break;
        d_p[(o + i) * stride] = stage_p[s0 + i];
        d_q[(o + i) * stride] = stage_q[s0 + i];
        d_w[(o + i) * stride] = stage_w[s0 + i];
        if (so.d_s) so.d_s[(o + i) * stride] = so.stage_s[s0 + i];
        if (so.d_w1) {
            const uint32_t w1 = so.stage_w1[s0 + i];
            so.d_w1[(o + i) * stride] = w1;
            so.d_w0[(o + i) * stride] = stage_w[s0 + i] - w1;
        }
    }
}

// ------------------------------------------------------------- the step --------------------
// One call of the bucketed residue path (or of the set path: make_keys differs):
//   front   keys (make_keys: the counting partition's level 1 for residues), level 2 / bucket
//           sort, bucket kernels (group + expand, heavy groups spilled)
//   heavy   the spilled frequent k-mers (heavy_phase; only when something spilled)
//   tail    row-block tail into (d_p, d_q, d_w), canonical order
// Fused step (nothing spilled, the usual case): all of it enqueued with no host wait and read
// back once (one D2H of statistics, cursors, flags and the run count), captured as a HIP graph
// from the second call of an unchanged shape and replayed after that.  Split step (the batch
// spills, or the fused step found a spill): front, one read-back, heavy path, exact tail
// geometry from the cursors, tail, read-back.  Overflowing buffers (shard regions, spill
// regions, level-2 bins) grow to the measured need and the step reruns; row blocks above the
// LDS capacity are finished by one segmented sort (pt_finish_overflow) without a rerun.
// Marks 0 (start), 1 (keys / level 1), 2 (level 2), 3 (bucket kernels [+ heavy]), 4 (pair
// partition), 5 (row-block sort + encode), 6 (emit + read-back).
// read-back: gstats (8 per shard) | pair cursors | spill cursors | the words below
enum : uint32_t {
    kRbCursor = kShards * 8, kRbSpill = kShards * 9, kRbFlagBin = kShards * 10, kRbFlagClass, kRbRuns, kRbOvf,
    kRbMaxBlock, kRbBinTiles, kRbFlagCur, kRbSegs, kRbSegMax, kRbFast, kRbList, kRbWords
};
constexpr uint32_t kGsWords = kShards * 10;  // gstats | cursors | spill cursors (u64)

// clears a step's flags and statistics (and extra[0, n_extra): the k-mer split's send cursors)
__global__ void step_clear_kernel(uint32_t* __restrict__ flags, unsigned long long* __restrict__ gstats,
                                  unsigned long long* __restrict__ extra = nullptr, uint32_t n_extra = 0) {
    for (uint32_t i = threadIdx.x; i < kGsWords; i += blockDim.x) gstats[i] = 0;
    if (threadIdx.x < kFlN) flags[threadIdx.x] = 0;
    for (uint32_t i = threadIdx.x; i < n_extra; i += blockDim.x) extra[i] = 0;
}

__global__ void step_pack_kernel(const unsigned long long* __restrict__ gstats, const uint32_t* __restrict__ flags,
                                 const uint32_t* __restrict__ runs, unsigned long long* __restrict__ rb) {
    step_pack_body(gstats, flags, runs, rb);
}

__device__ void step_pack_body(const unsigned long long* __restrict__ gstats, const uint32_t* __restrict__ flags,
                               const uint32_t* __restrict__ runs, unsigned long long* __restrict__ rb,
                               unsigned long long fast_ovf) {
    for (uint32_t i = threadIdx.x; i < kGsWords; i += blockDim.x) rb[i] = gstats[i];
    if (threadIdx.x == 0) {
        rb[kRbFast] = fast_ovf;
        rb[kRbList] = flags[kFlList];
        rb[kRbFlagBin] = flags[kFlBin];
        rb[kRbFlagClass] = flags[kFlClass];
        rb[kRbRuns] = runs ? runs[0] : 0;
        rb[kRbOvf] = flags[kFlOvf];
        rb[kRbMaxBlock] = runs ? runs[1] : 0;
        rb[kRbBinTiles] = flags[kFlBinTiles];
        rb[kRbFlagCur] = flags[kFlCur];
        rb[kRbSegs] = flags[kFlSegs];
        rb[kRbSegMax] = flags[kFlSegMax];
    }
    __threadfence_system();  // rb is host memory, read after the stream synchronises
}

// ------------------------------------------------------------- fast row-block tail --------
// The default tail of an unscored single-k call (combine_edges, mod.rs:322-546; KmerEdgeGroup::new,
// edge.rs:56-85): no histogram pass, no scan, no staging, no emit kernel.
//   pt_scatter<true>  row block r's keys (u32 p_local << pbits | q) into the fixed region
//                     [r * kFtCap, (r + 1) * kFtCap), reserved on fcur[r] (from zero);
//   pt_reduce_fast    one workgroup per row block: its keys aggregated in an LDS hash table on the
//                     pair (count = w, i.e. one KmerEdge::Group per pair with len(kmers) = w), the
//                     distinct pairs grouped by row (a counting sort on the row), each ranked within
//                     its row by q (its rank = the row's pairs with a smaller q), and written in
//                     canonical order straight to (d_p, d_q, d_w) at the block's edge offset, which a
//                     decoupled look-back over the blocks before it supplies (wave 0, while nothing
//                     else of the block waits on it until the copy-out).  It re-zeroes fcur[r] for the
//                     next call.  A block above kFtHashMax keys, one with a row of more than
//                     kFtRankMax pairs, or one whose pair count would pass 16 bits sorts its keys
//                     instead (block radix sort + run-length encoding).  A block above kFtCap keys
//                     (its region overflowed) raises the read-back's kRbFast word: the caller reruns
//                     the call on the counting tail and keeps it for the shape.
// The last block writes the edge count and the step's read-back.
constexpr uint32_t kFtThreads = 512, kFtHashMax = 6144, kFtSlots = 8192, kFtRowsMax = 1024, kFtRankMax = 256;
constexpr uint32_t kFtEmpty = 0xFFFFFFFFu;
constexpr unsigned long long kLbAgg = 1ull << 62, kLbInc = 2ull << 62, kLbOvf = 1ull << 61;
static_assert(kFtCap == 16 * kFtThreads && kFtHashMax <= 12 * kFtThreads && kFtSlots == 16 * kFtThreads,
              "per-thread register arrays of pt_reduce_fast");

// look-back words: one 8-B word per block, written and polled with agent-scope relaxed atomics
// (sc1): the word itself is the only datum handed over
__device__ __forceinline__ unsigned long long lb_load(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wave 0 of block r: publishes the block's aggregate (count | overflow bit), sums the aggregates of
// the blocks before it (64 per round, one per lane) back to the nearest inclusive prefix, publishes
// its own inclusive prefix; returns the exclusive one (count | overflow bit of any earlier block).
// Blocks are dispatched in index order, so every predecessor is resident or done: the polls end.
// ft_publish: the aggregate alone, as soon as it is known (a block that still has work before its
// writes publishes early, so the blocks after it find it there); ft_lookback(..., published) then
// skips the store.
__device__ __forceinline__ void ft_publish(unsigned long long* lb, uint32_t r, unsigned long long agg) {
    if ((threadIdx.x & 63) == 0) lb_store(lb + r, (r ? kLbAgg : kLbInc) | agg);
}
__device__ unsigned long long ft_lookback(unsigned long long* lb, uint32_t r, unsigned long long agg,
                                          bool published = false) {
    const uint32_t lane = threadIdx.x & 63;
    if (r == 0) {
        if (lane == 0 && !published) lb_store(lb, kLbInc | agg);
        return 0;
    }
    if (lane == 0 && !published) lb_store(lb + r, kLbAgg | agg);
    uint32_t cnt = 0;
    bool ovf = false;
    int64_t top = (int64_t)r - 1;
    while (true) {
        const int64_t j = top - (int64_t)lane;
        const unsigned long long v = j >= 0 ? lb_load(lb + j) : kLbInc;
        const uint32_t st = (uint32_t)(v >> 62);
        const unsigned long long inc = __ballot(st == 2), none = __ballot(st == 0);
        const uint32_t first = inc ? (uint32_t)__builtin_ctzll(inc) : 64u;
        const unsigned long long upto = first >= 63 ? ~0ull : (2ull << first) - 1;
        if (none & upto) {  // a predecessor has not published yet
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        const bool in = lane <= first;
        cnt += wave_sum(in ? (uint32_t)v : 0u);
        ovf |= __ballot(in && (v & kLbOvf)) != 0;
        if (first < 64) break;
        top -= 64;
    }
    const unsigned long long excl = (unsigned long long)cnt | (ovf ? kLbOvf : 0ull);
    if (lane == 0) lb_store(lb + r, kLbInc | ((unsigned long long)(cnt + (uint32_t)agg) | ((agg | excl) & kLbOvf)));
    return excl;
}

struct FtLds {
    union {
        struct {
            uint32_t K[kFtSlots];  // hash slots (pair key), then the block's pairs in row / canonical order
            uint16_t C[kFtSlots + 2];  // counts (w), two per 32-bit word for the LDS atomics; the
                                       // sort path's run heads use C[0, nruns] (nruns <= kFtCap)
        } h;
        typename PtSort<16>::storage_type s16;
    };
    uint32_t RC[kFtRowsMax + 1];  // pairs per row -> row starts
    uint32_t last[kFtThreads];
    uint32_t wave_tot[kFtThreads / 64];
    uint32_t s_max, s_flag;
    unsigned long long s_excl;
};

__global__ __launch_bounds__(kFtThreads) void pt_reduce_fast_kernel(const uint32_t* __restrict__ keys,
                                                                    uint32_t* __restrict__ fcur, PtGeom g,
                                                                    unsigned long long* __restrict__ lb,
                                                                    uint32_t* __restrict__ d_p,
                                                                    uint32_t* __restrict__ d_q,
                                                                    uint32_t* __restrict__ d_w, uint64_t cap,
                                                                    uint32_t stride, PtPack pack,
                                                                    uint32_t* __restrict__ runs) {
    __shared__ FtLds u;
    const uint32_t r = blockIdx.x, tid = threadIdx.x;
    const uint32_t nraw = fcur[r];
    __syncthreads();  // every thread has its count before the cursor is cleared for the next call
    if (tid == 0) fcur[r] = 0;
    const bool ovf = nraw > kFtCap;
    const uint32_t n = ovf ? 0u : nraw;
    const uint32_t* src = keys + (uint64_t)r * kFtCap;  // g.ftcap == kFtCap in this mode
    const unsigned pb = g.pbits;
    const uint32_t R = 1u << g.rbits;
    uint32_t D = 0;  // the block's kept pairs
    bool sort = n > kFtHashMax, published = false;
    if (!sort) {
        // ---- hash aggregation: pair -> slot, count per slot ----
        for (uint32_t i = tid; i < kFtSlots; i += kFtThreads) u.h.K[i] = kFtEmpty;
        for (uint32_t i = tid; i < kFtSlots / 2; i += kFtThreads) reinterpret_cast<uint32_t*>(u.h.C)[i] = 0;
        for (uint32_t i = tid; i <= R; i += kFtThreads) u.RC[i] = 0;
        if (tid == 0) u.s_max = u.s_flag = 0;
        uint32_t x[12];
#pragma unroll
        for (uint32_t e = 0; e < 12; ++e) {
            const uint32_t i = tid + e * kFtThreads;
            x[e] = i < n ? src[i] : kFtEmpty;
        }
        __syncthreads();
#pragma unroll
        for (uint32_t e = 0; e < 12; ++e) {
            if (x[e] == kFtEmpty) continue;
            uint32_t sl = (x[e] * 0x9E3779B1u) >> 19;  // 13 bits: kFtSlots
            while (true) {
                const uint32_t old = atomicCAS(&u.h.K[sl], kFtEmpty, x[e]);
                if (old == kFtEmpty || old == x[e]) break;
                sl = (sl + 1) & (kFtSlots - 1);
            }
            const uint32_t sh = 16 * (sl & 1);
            const uint32_t old = atomicAdd(reinterpret_cast<uint32_t*>(u.h.C) + (sl >> 1), 1u << sh);
            if (((old >> sh) & 0xFFFFu) >= 0xFFFEu) u.s_flag = 1;  // w would reach 16 bits: sort instead
        }
        __syncthreads();
        // ---- kept pairs (w >= min_shared) counted per row, ranked in arrival order ----
        uint32_t ek[16], er[16];  // pair key | rank in its row << 16 | w
#pragma unroll
        for (uint32_t j = 0; j < 16; ++j) {
            const uint32_t sl = tid + j * kFtThreads;
            const uint32_t k = u.h.K[sl], w = u.h.C[sl];
            ek[j] = kFtEmpty;
            if (k != kFtEmpty && w >= g.min_shared) {
                ek[j] = k;
                er[j] = atomicAdd(&u.RC[k >> pb], 1u) << 16 | w;
            }
        }
        __syncthreads();
        // row starts (R <= kFtRowsMax = 2 * kFtThreads rows) and the largest row
        const uint32_t a0 = 2 * tid < R ? u.RC[2 * tid] : 0u, a1 = 2 * tid + 1 < R ? u.RC[2 * tid + 1] : 0u;
        const uint32_t mx = wave_max(max(a0, a1));
        if ((tid & 63) == 0) atomicMax(&u.s_max, mx);
        uint32_t excl, total;
        block_scan_n<kFtThreads>(a0 + a1, excl, total, u.wave_tot);
        if (2 * tid < R) u.RC[2 * tid] = excl;
        if (2 * tid + 1 < R) u.RC[2 * tid + 1] = excl + a0;
        if (tid == 0) u.RC[R] = total;
        __syncthreads();
        D = total;
        sort = u.s_flag || u.s_max > kFtRankMax;  // uniform
        if (!sort) {
            // the count is final: published before the ranking, the blocks after this one wait less
            if (tid < 64) ft_publish(lb, r, (unsigned long long)D | (ovf ? kLbOvf : 0ull));
            published = true;
            // grouped by row (the slots were read above the barriers)
#pragma unroll
            for (uint32_t j = 0; j < 16; ++j)
                if (ek[j] != kFtEmpty) {
                    const uint32_t pos = u.RC[ek[j] >> pb] + (er[j] >> 16);
                    u.h.K[pos] = ek[j];
                    u.h.C[pos] = (uint16_t)er[j];
                }
            __syncthreads();
            // rank within the row by q: canonical position
            uint32_t fk[12], fp[12];  // key | position << 16 | w
#pragma unroll
            for (uint32_t e = 0; e < 12; ++e) {
                const uint32_t i = tid + e * kFtThreads;
                fk[e] = kFtEmpty;
                if (i < D) {
                    const uint32_t key = u.h.K[i], row = key >> pb, a = u.RC[row], b = u.RC[row + 1];
                    uint32_t rk = 0;
                    for (uint32_t t = a; t < b; ++t) rk += u.h.K[t] < key;
                    fk[e] = key;
                    fp[e] = (a + rk) << 16 | u.h.C[i];
                }
            }
            __syncthreads();
#pragma unroll
            for (uint32_t e = 0; e < 12; ++e)
                if (fk[e] != kFtEmpty) {
                    u.h.K[fp[e] >> 16] = fk[e];
                    u.h.C[fp[e] >> 16] = (uint16_t)fp[e];
                }
        }
        __syncthreads();
    }
    if (sort) {
        // ---- a block too large or too skewed for the hash: block radix sort + run-length encode ----
        uint32_t k[16];
#pragma unroll
        for (uint32_t e = 0; e < 16; ++e) {
            const uint32_t i = tid + e * kFtThreads;
            k[e] = i < n ? src[i] : kFtEmpty;
        }
        PtSort<16>().sort(k, u.s16, 0, pb + g.rbits + 1);  // blocked: thread t holds ranks t * 16 + e
        u.last[tid] = k[15];
        __syncthreads();
        uint32_t prev = tid ? u.last[tid - 1] : 0u, nh = 0;
        bool head[16];
#pragma unroll
        for (uint32_t e = 0; e < 16; ++e) {
            const uint32_t rank = tid * 16 + e;
            head[e] = rank < n && (rank == 0 || k[e] != prev);
            prev = k[e];
            nh += head[e];
        }
        uint32_t base, nruns;
        block_scan_n<kFtThreads>(nh, base, nruns, u.wave_tot);  // barriers: the sort storage is dead
        // run keys in K, head ranks in C (ranks < kFtCap fit 16 bits; C[nruns] = n needs n < 2^16)
#pragma unroll
        for (uint32_t e = 0; e < 16; ++e)
            if (head[e]) {
                u.h.K[base] = k[e];
                u.h.C[base] = (uint16_t)(tid * 16 + e);
                ++base;
            }
        if (tid == 0) u.h.C[nruns] = (uint16_t)n;
        __syncthreads();
        // runs with w >= min_shared, compacted in order (thread t: runs [t q, t q + q))
        const uint32_t q = (nruns + kFtThreads - 1) / kFtThreads;
        uint32_t kv[16], wv[16], kept = 0;
#pragma unroll
        for (uint32_t e = 0; e < 16; ++e) {
            const uint32_t jr = tid * q + e;
            wv[e] = 0;
            if (e < q && jr < nruns) {
                kv[e] = u.h.K[jr];
                wv[e] = (uint32_t)u.h.C[jr + 1] - u.h.C[jr];
                kept += wv[e] >= g.min_shared;
            }
        }
        uint32_t o;
        block_scan_n<kFtThreads>(kept, o, D, u.wave_tot);
#pragma unroll
        for (uint32_t e = 0; e < 16; ++e)
            if (wv[e] && wv[e] >= g.min_shared) {
                u.h.K[o] = kv[e];
                u.h.C[o] = (uint16_t)wv[e];
                ++o;
            }
        __syncthreads();
    }
    // ---- the block's edge offset, then the pairs straight to the edge arrays ----
    if (tid < 64) {
        const unsigned long long ex = ft_lookback(lb, r, (unsigned long long)D | (ovf ? kLbOvf : 0ull), published);
        if (tid == 0) u.s_excl = ex;
    }
    __syncthreads();
    const unsigned long long ex = u.s_excl;
    const uint64_t o = (uint32_t)ex;
    const uint32_t rowbase = g.row0 + (r << g.rbits), qm = (1u << pb) - 1;
    for (uint32_t i = tid; i < D; i += kFtThreads) {
        if (o + i >= cap) break;
        const uint32_t key = u.h.K[i];
        d_p[(o + i) * stride] = rowbase + (key >> pb);
        d_q[(o + i) * stride] = key & qm;
        d_w[(o + i) * stride] = u.h.C[i];
    }
    if (r + 1 == gridDim.x) {  // the last block: the edge count and the read-back
        const bool any_ovf = ovf || (ex & kLbOvf);
        if (tid == 0) {
            runs[0] = (uint32_t)(o + D);
            runs[1] = 0;
        }
        __syncthreads();
        if (pack.rb) step_pack_body(pack.gstats, pack.flags, runs, pack.rb, any_ovf ? 1ull : 0ull);
    }
}


// The dense variant (small batches: pbits + rbits <= kFdBitsMax, the reference's uniprot_arg.fasta at
// k = 5 among them, whose rows pair with thousands of later proteins — up to ~10^5 keys in one row:
// near-identical AMR families): block r's keys counted in 2^(pbits + rbits) LDS bins over (row, q) —
// u16 counts, two per word — so the bins ARE the canonical order: no hash, no rank, no sort.  Its
// keys come from the counting partition (bst: block r is [bst[r], bst[r + 1]), any size; a fixed
// region would overflow on such rows).  Thread t owns the contiguous words [t q, t q + q) (q = words
// / kFtThreads); stored XOR-swizzled (word w at w ^ ((w / q) mod min(q, 32))) so the owners' reads of
// their words hit distinct banks.  A count that would reach 16 bits raises the fast tail's overflow
// (the caller reruns on the counting tail).
__device__ __forceinline__ uint32_t fd_phys(uint32_t w, unsigned qs) {
    return w ^ ((w >> qs) & ((1u << min(qs, 5u)) - 1));
}
__global__ __launch_bounds__(kFtThreads) void pt_reduce_dense_kernel(const uint32_t* __restrict__ keys,
                                                                     const uint32_t* __restrict__ bst, PtGeom g,
                                                                     unsigned long long* __restrict__ lb,
                                                                     uint32_t* __restrict__ d_p,
                                                                     uint32_t* __restrict__ d_q,
                                                                     uint32_t* __restrict__ d_w, uint64_t cap,
                                                                     uint32_t stride, PtPack pack,
                                                                     uint32_t* __restrict__ runs) {
    __shared__ uint32_t W[1u << (kFdBitsMax - 1)];  // 64 KB
    __shared__ uint32_t wave_tot[kFtThreads / 64];
    __shared__ uint32_t s_flag;
    __shared__ unsigned long long s_excl;
    const uint32_t r = blockIdx.x, tid = threadIdx.x;
    if (tid == 0) s_flag = 0;
    bool ovf = false;
    const uint32_t s0 = bst[r], n = bst[r + 1] - s0;
    const uint32_t* src = keys + s0;
    const unsigned pb = g.pbits, bits = g.pbits + g.rbits;
    const uint32_t words = 1u << (bits - 1);
    unsigned qs = 0;  // q = words / kFtThreads = 2^qs words per thread (at least one)
    while ((kFtThreads << qs) < words) ++qs;
    for (uint32_t i = tid; i < words; i += kFtThreads) W[i] = 0;
    __syncthreads();
    for (uint32_t i0 = 0; i0 < n; i0 += 8 * kFtThreads) {  // loads in batches ahead of their atomics
        uint32_t x[8];
#pragma unroll
        for (uint32_t e = 0; e < 8; ++e) {
            const uint32_t i = i0 + e * kFtThreads + tid;
            x[e] = i < n ? src[i] : kFtEmpty;
        }
#pragma unroll
        for (uint32_t e = 0; e < 8; ++e)
            if (x[e] != kFtEmpty) {
                const uint32_t sh = 16 * (x[e] & 1u);
                const uint32_t old = atomicAdd(&W[fd_phys(x[e] >> 1, qs)], 1u << sh);
                if (((old >> sh) & 0xFFFFu) >= 0xFFFEu) s_flag = 1;
            }
    }
    __syncthreads();
    ovf = ovf || s_flag;  // uniform
    // kept bins (w >= min_shared) of the thread's words, in bin order
    const uint32_t q = 1u << qs, w0 = tid << qs;
    uint32_t kept = 0;
    if (!ovf)
        for (uint32_t j = 0; j < q && w0 + j < words; ++j) {
            const uint32_t v = W[fd_phys(w0 + j, qs)];
            kept += ((v & 0xFFFFu) >= g.min_shared) + ((v >> 16) >= g.min_shared);
        }
    uint32_t excl, D;
    block_scan_n<kFtThreads>(kept, excl, D, wave_tot);
    if (tid < 64) {
        const unsigned long long ex = ft_lookback(lb, r, (unsigned long long)D | (ovf ? kLbOvf : 0ull));
        if (tid == 0) s_excl = ex;
    }
    __syncthreads();
    const unsigned long long ex = s_excl;
    uint64_t o = (uint32_t)ex + (uint64_t)excl;
    const uint32_t rowbase = g.row0 + (r << g.rbits), qm = (1u << pb) - 1;
    if (kept)
        for (uint32_t j = 0; j < q && w0 + j < words; ++j) {
            const uint32_t v = W[fd_phys(w0 + j, qs)];
#pragma unroll
            for (uint32_t h = 0; h < 2; ++h) {
                const uint32_t c = h ? v >> 16 : v & 0xFFFFu;
                if (c < g.min_shared || c == 0) continue;
                const uint32_t bin = 2 * (w0 + j) + h;
                if (o < cap) {
                    d_p[o * stride] = rowbase + (bin >> pb);
                    d_q[o * stride] = bin & qm;
                    d_w[o * stride] = c;
                }
                ++o;
            }
        }
    if (r + 1 == gridDim.x) {  // the last block: the edge count and the read-back
        const bool any_ovf = ovf || (ex & kLbOvf);
        if (tid == 0) {
            runs[0] = (uint32_t)ex + D;
            runs[1] = 0;
        }
        __syncthreads();
        if (pack.rb) step_pack_body(pack.gstats, pack.flags, runs, pack.rb, any_ovf ? 1ull : 0ull);
    }
}

// The fused multi-k tail with its edges written in place (no staging and no emit kernel): the
// sub-blocks of a pass are sorted in place and their kept runs counted (pt_reduce_count_kernel),
// the counts scanned on the device, and each sub-block's runs written at its offset
// (pt_reduce_write_kernel) as (p, q, w, score, w0, w1) columns.  A sub-block above kPtCap (a fine
// bin of pt_split above kPtCap - kSbChunk keys: a row pairing many times with a few partners) is
// reduced in windows of kDwWin pair positions — per position a count (| w1 << 16) and a score sum
// in LDS, the windows visiting only occupied positions — counted by pt_window_count_kernel and
// written by the write launch: no device sort anywhere.
constexpr uint32_t kDwWin = 8192;
struct PtDirectOut {
    uint32_t *d_p, *d_q, *d_w, *d_s, *d_w0, *d_w1;
    uint64_t cap;
    uint32_t stride;
};
struct PtDirectLds {
    union {
        typename PtSort<2>::storage_type s2;
        typename PtSort<4>::storage_type s4;
        typename PtSort<8>::storage_type s8;
        typename PtSort<16>::storage_type s16;
        PtBinLds b;
        struct {
            uint32_t H[kPtCap + 1];  // each run's first rank | k-bit scan at it << 16
            uint32_t P[kPtCap + 1];  // each run's pair key, then the score scan at its head
        } r;
        struct {
            uint32_t A[kDwWin];  // count | w1 << 16 per pair position of the window
            uint32_t S[kDwWin];  // score sum
        } w;
    };
    uint32_t last[kPtRThreads];
    uint32_t wave_tot[kPtRThreads / 64];
    unsigned long long s_excl, s_next;
};

__device__ __forceinline__ bool pt_keep(uint32_t w, uint32_t w1, bool kbit, uint32_t ms) {
    return w != 0 && (kbit ? (w - w1 >= ms || w1 >= ms) : w >= ms);
}

__device__ __forceinline__ void pt_direct_write(const PtDirectOut& o, uint64_t at, uint32_t p, uint32_t q, uint32_t w,
                                                uint32_t s, uint32_t w1, bool kbit) {
    if (at >= o.cap) return;
    const uint64_t x = at * o.stride;
    o.d_p[x] = p;
    o.d_q[x] = q;
    o.d_w[x] = w;
    o.d_s[x] = s;
    if (kbit) {
        o.d_w1[x] = w1;
        o.d_w0[x] = w - w1;
    }
}

// One sub-block of at most kPtCap keys, in two launches with a device scan between them (no
// look-back: waiting on the predecessors' counts cost as much as the sort at config 5, where the
// ~4e5 sub-blocks of a pass finish in no particular order).  kWrite false: load, sort (bins, or the
// block radix sort), store the sorted keys back in place, count the kept runs into *wc.  kWrite
// true: load the sorted keys (thread t: ranks t kE + e), encode, and write the runs from edge
// offset ex: the runs' first ranks (| k-bit scan << 16) and pair keys sit in LDS (H, P), then P
// takes the score scan at the heads for the score column; one run per thread per round, coalesced.
template <uint32_t kE, bool kKbit, bool kWrite>
__device__ __forceinline__ void pt_direct_block(PtDirectLds& L, typename PtSort<kE>::storage_type& st,
                                                uint32_t* __restrict__ src, uint32_t s0, uint32_t n, uint32_t r,
                                                const PtGeom& g, const PtDirectOut& out, uint32_t* __restrict__ wc,
                                                uint64_t ex) {
    uint32_t k[kE];
    const unsigned sb = g.sbits;
    const uint32_t rowbase = g.row0 + (r << g.rbits);
    const uint32_t rank0 = threadIdx.x * kE, smask = (1u << kScoreBits) - 1;
    if (!kWrite) {
#pragma unroll
        for (uint32_t e = 0; e < kE; ++e) {
            const uint32_t i = threadIdx.x + e * kPtRThreads;
            k[e] = i < n ? src[s0 + i] : 0xFFFFFFFFu;
        }
        if (!g.binsort || !pt_bin_sort<kE>(k, n, g, rowbase, L.b, L.last, L.last + 2 * kPtRThreads / 64, L.wave_tot))
            PtSort<kE>().sort(k, st, 0, g.pbits + sb + g.rbits + 1);  // blocked: thread t holds ranks t*kE + e
#pragma unroll
        for (uint32_t e = 0; e < kE; ++e)
            if (rank0 + e < n) src[s0 + rank0 + e] = k[e];
    } else {
#pragma unroll
        for (uint32_t e = 0; e < kE; ++e) k[e] = rank0 + e < n ? src[s0 + rank0 + e] : 0xFFFFFFFFu;
    }
    __syncthreads();  // the sort's LDS is dead before last (aliased) is written
    L.last[threadIdx.x] = k[kE - 1] >> sb;
    __syncthreads();
    uint32_t prev = threadIdx.x ? L.last[threadIdx.x - 1] : 0u, nh = 0, ssum = 0, ksum = 0;
    uint32_t hm = 0;  // head bits
#pragma unroll
    for (uint32_t e = 0; e < kE; ++e) {
        const uint32_t rank = rank0 + e, pk = k[e] >> sb;
        const bool h = rank < n && (rank == 0 || pk != prev);
        hm |= (uint32_t)h << e;
        prev = pk;
        nh += h;
        if (rank < n) {
            ssum += k[e] & smask;
            if (kKbit) ksum += (k[e] >> kScoreBits) & 1u;
        }
    }
    const bool filter = g.min_shared > 1;
    uint32_t base0, nruns, sx0 = 0, stot = 0, kx = 0, ktot = 0;
    block_scan_n<kPtRThreads>(nh, base0, nruns, L.wave_tot);
    if (!kWrite && !filter) {  // every run kept: the count is the run count
        if (threadIdx.x == 0) *wc = nruns;
        return;
    }
    if (kWrite) block_scan_n<kPtRThreads>(ssum, sx0, stot, L.wave_tot);
    if (kKbit) block_scan_n<kPtRThreads>(ksum, kx, ktot, L.wave_tot);
    {
        uint32_t base = base0;
#pragma unroll
        for (uint32_t e = 0; e < kE; ++e) {
            if (hm >> e & 1u) {
                L.r.H[base] = (rank0 + e) | (kKbit ? kx << 16 : 0u);
                L.r.P[base] = k[e] >> sb;
                ++base;
            }
            if (kKbit && rank0 + e < n) kx += (k[e] >> kScoreBits) & 1u;
        }
    }
    if (threadIdx.x == 0) L.r.H[nruns] = n | (kKbit ? ktot << 16 : 0u);
    __syncthreads();
    auto run_w = [&](uint32_t i, uint32_t& w, uint32_t& w1) {
        const uint32_t h0 = L.r.H[i], h1 = L.r.H[i + 1];
        w = (h1 & 0xFFFFu) - (h0 & 0xFFFFu);
        w1 = kKbit ? (h1 >> 16) - (h0 >> 16) : 0u;
    };
    if (!kWrite) {  // min_shared > 1: the kept runs
        uint32_t kept = 0;
        for (uint32_t i = threadIdx.x; i < nruns; i += kPtRThreads) {
            uint32_t w, w1;
            run_w(i, w, w1);
            kept += pt_keep(w, w1, kKbit, g.min_shared);
        }
        uint32_t e, total;
        block_scan_n<kPtRThreads>(kept, e, total, L.wave_tot);
        if (threadIdx.x == 0) *wc = total;
        return;
    }
    const uint32_t qm = (1u << g.pbits) - 1;
    // rounds of kPtRThreads runs, thread t the round's run t; filter: the kept runs compacted
    // (a block scan per round — uniform trip count)
    auto rounds = [&](auto&& body) {
        uint32_t o = 0;
        for (uint32_t i0 = 0; i0 < nruns; i0 += kPtRThreads) {
            const uint32_t i = i0 + threadIdx.x;
            uint32_t w = 0, w1 = 0;
            if (i < nruns) run_w(i, w, w1);
            const bool keep = i < nruns && pt_keep(w, w1, kKbit, g.min_shared);
            uint32_t at = i, rt = 0;
            if (filter) {
                uint32_t e;
                block_scan_n<kPtRThreads>(keep ? 1u : 0u, e, rt, L.wave_tot);
                at = o + e;
                o += rt;
            }
            if (keep) body(i, ex + at, w, w1);
        }
    };
    rounds([&](uint32_t i, uint64_t at, uint32_t w, uint32_t w1) {
        const uint32_t pk = L.r.P[i];
        if (at >= out.cap) return;
        const uint64_t x = at * out.stride;
        out.d_p[x] = rowbase + (pk >> g.pbits);
        out.d_q[x] = pk & qm;
        out.d_w[x] = w;
        if (kKbit) {
            out.d_w1[x] = w1;
            out.d_w0[x] = w - w1;
        }
    });
    __syncthreads();  // P read: it takes the score scan
    {
        uint32_t base = base0, sx = sx0;
#pragma unroll
        for (uint32_t e = 0; e < kE; ++e) {
            if (hm >> e & 1u) L.r.P[base++] = sx;
            if (rank0 + e < n) sx += k[e] & smask;
        }
    }
    if (threadIdx.x == 0) L.r.P[nruns] = stot;
    __syncthreads();
    rounds([&](uint32_t i, uint64_t at, uint32_t, uint32_t) {
        if (at < out.cap) out.d_s[at * out.stride] = L.r.P[i + 1] - L.r.P[i];
    });
}

// a sub-block above kPtCap: windows of kDwWin pair positions (the monotone position of pt_bin_sort),
// visiting only occupied positions; one pass: the kept count (write false), or the writes from
// output offset ex.  Returns the kept count.
template <bool kKbit>
__device__ uint32_t pt_windows(PtDirectLds& L, const uint32_t* __restrict__ src, uint32_t s0, uint32_t n, uint32_t r,
                               const PtGeom& g, bool write, uint64_t ex, const PtDirectOut& out) {
    constexpr uint32_t kPer = kDwWin / kPtRThreads;
    const unsigned sb = g.sbits, rs = g.pbits + g.sbits;
    const uint32_t rowbase = g.row0 + (r << g.rbits), qm = (1u << g.pbits) - 1, qlo = rowbase + 1;
    const uint64_t span = g.nprot > qlo ? g.nprot - qlo : 1u;
    const uint32_t smask = (1u << kScoreBits) - 1;
    auto pos = [&](uint32_t x) -> uint64_t {
        const uint32_t q = (x >> sb) & qm;
        return (uint64_t)(x >> rs) * span + (q > qlo ? q - qlo : 0u);
    };
    auto wave_min64 = [](unsigned long long v) {
        for (int off = 32; off > 0; off >>= 1) v = min(v, (unsigned long long)__shfl_xor(v, off));
        return v;
    };
    // the first occupied position
    unsigned long long mn = ~0ull;
    for (uint32_t i = threadIdx.x; i < n; i += kPtRThreads) mn = min(mn, (unsigned long long)pos(src[s0 + i]));
    __syncthreads();  // the caller's LDS reads are done
    if (threadIdx.x == 0) L.s_next = ~0ull;
    __syncthreads();
    mn = wave_min64(mn);
    if ((threadIdx.x & 63) == 0) atomicMin(&L.s_next, mn);
    __syncthreads();
    unsigned long long wlo = L.s_next;
    uint64_t o = 0;
    while (wlo != ~0ull) {  // uniform
        __syncthreads();  // the previous window's reads are done
        for (uint32_t i = threadIdx.x; i < kDwWin; i += kPtRThreads) {
            L.w.A[i] = 0;
            L.w.S[i] = 0;
        }
        if (threadIdx.x == 0) L.s_next = ~0ull;
        __syncthreads();
        unsigned long long nx = ~0ull;
        for (uint32_t i0 = 0; i0 < n; i0 += 8 * kPtRThreads) {  // loads in batches ahead of the atomics
            uint32_t v[8];
#pragma unroll
            for (uint32_t e = 0; e < 8; ++e) {
                const uint32_t i = i0 + e * kPtRThreads + threadIdx.x;
                v[e] = i < n ? src[s0 + i] : 0xFFFFFFFFu;
            }
#pragma unroll
            for (uint32_t e = 0; e < 8; ++e) {
                if (i0 + e * kPtRThreads + threadIdx.x >= n) continue;
                const uint64_t ps = pos(v[e]);
                if (ps < wlo) continue;
                if (ps >= wlo + kDwWin) {
                    nx = min(nx, (unsigned long long)ps);
                    continue;
                }
                const uint32_t a = (uint32_t)(ps - wlo);
                atomicAdd(&L.w.A[a], 1u | (kKbit ? ((v[e] >> kScoreBits) & 1u) << 16 : 0u));
                if (write) atomicAdd(&L.w.S[a], v[e] & smask);
            }
        }
        nx = wave_min64(nx);
        if ((threadIdx.x & 63) == 0) atomicMin(&L.s_next, nx);
        __syncthreads();
        // thread t: positions [t kPer, t kPer + kPer)
        uint32_t kept = 0;
#pragma unroll
        for (uint32_t j = 0; j < kPer; ++j) {
            const uint32_t a = L.w.A[threadIdx.x * kPer + j];
            kept += pt_keep(a & 0xFFFFu, a >> 16, kKbit, g.min_shared);
        }
        uint32_t e0, wt;
        block_scan_n<kPtRThreads>(kept, e0, wt, L.wave_tot);
        if (write) {
            uint64_t at = ex + o + e0;
            for (uint32_t j = 0; j < kPer; ++j) {
                const uint32_t x = threadIdx.x * kPer + j, a = L.w.A[x];
                const uint32_t w = a & 0xFFFFu, w1 = a >> 16;
                if (!pt_keep(w, w1, kKbit, g.min_shared)) continue;
                const uint64_t ps = wlo + x, rl = ps / span;
                pt_direct_write(out, at, rowbase + (uint32_t)rl, qlo + (uint32_t)(ps - rl * span), w, L.w.S[x], w1,
                                kKbit);
                ++at;
            }
        }
        o += wt;
        wlo = L.s_next;
    }
    return (uint32_t)o;
}

// the kept counts of the sub-blocks above kPtCap (listed by pt_split: ovl[0] of them at ovl + 1),
// before the in-place reduce: there each publishes its count at once, so the look-back of the
// blocks after it never waits on its windows
template <bool kKbit>
__global__ __launch_bounds__(kPtRThreads) void pt_window_count_kernel(const uint32_t* __restrict__ keys, BlkSrc bs,
                                                                      PtGeom g, const uint32_t* __restrict__ ovl,
                                                                      uint32_t* __restrict__ wc) {
    __shared__ PtDirectLds L;
    const uint32_t m = ovl[0];
    for (uint32_t i = blockIdx.x; i < m; i += gridDim.x) {
        const uint32_t d = ovl[1 + i];
        uint32_t s0, n, r;
        blk_of(bs, d, s0, n, r);
        const uint32_t t = pt_windows<kKbit>(L, blk_keys(bs, d, keys), s0, n, r, g, false, 0, PtDirectOut{});
        if (threadIdx.x == 0) wc[d] = t;
    }
}

// count launch: every sub-block of at most kPtCap keys sorted in place and its kept runs counted
// into wc (the larger ones: pt_window_count_kernel; stat[0] counts them)
template <bool kKbit>
__global__ __launch_bounds__(kPtRThreads) void pt_reduce_count_kernel(uint32_t* __restrict__ keys, BlkSrc bs, PtGeom g,
                                                                      uint32_t* __restrict__ wc,
                                                                      unsigned long long* __restrict__ stat) {
    __shared__ PtDirectLds L;
    const uint32_t d = blockIdx.x;
    uint32_t s0, n, r;
    blk_of(bs, d, s0, n, r);
    uint32_t* src = const_cast<uint32_t*>(blk_keys(bs, d, keys));
    const PtDirectOut none{};
    if (n == 0) {
        if (threadIdx.x == 0) wc[d] = 0;
    } else if (n <= 2 * kPtRThreads) {
        pt_direct_block<2, kKbit, false>(L, L.s2, src, s0, n, r, g, none, wc + d, 0);
    } else if (n <= 4 * kPtRThreads) {
        pt_direct_block<4, kKbit, false>(L, L.s4, src, s0, n, r, g, none, wc + d, 0);
    } else if (n <= 8 * kPtRThreads) {
        pt_direct_block<8, kKbit, false>(L, L.s8, src, s0, n, r, g, none, wc + d, 0);
    } else if (n <= kPtCap) {
        pt_direct_block<16, kKbit, false>(L, L.s16, src, s0, n, r, g, none, wc + d, 0);
    } else if (threadIdx.x == 0) {
        atomicAdd(&stat[0], 1ull);
    }
}

// write launch: each sub-block's runs at its offset off[d] (the exclusive scan of the counts)
template <bool kKbit>
__global__ __launch_bounds__(kPtRThreads) void pt_reduce_write_kernel(uint32_t* __restrict__ keys, BlkSrc bs, PtGeom g,
                                                                      PtDirectOut out,
                                                                      const uint32_t* __restrict__ off) {
    __shared__ PtDirectLds L;
    const uint32_t d = blockIdx.x;
    uint32_t s0, n, r;
    blk_of(bs, d, s0, n, r);
    uint32_t* src = const_cast<uint32_t*>(blk_keys(bs, d, keys));
    const uint64_t ex = off[d];
    if (n == 0) return;
    if (n <= 2 * kPtRThreads)
        pt_direct_block<2, kKbit, true>(L, L.s2, src, s0, n, r, g, out, nullptr, ex);
    else if (n <= 4 * kPtRThreads)
        pt_direct_block<4, kKbit, true>(L, L.s4, src, s0, n, r, g, out, nullptr, ex);
    else if (n <= 8 * kPtRThreads)
        pt_direct_block<8, kKbit, true>(L, L.s8, src, s0, n, r, g, out, nullptr, ex);
    else if (n <= kPtCap)
        pt_direct_block<16, kKbit, true>(L, L.s16, src, s0, n, r, g, out, nullptr, ex);
    else
        pt_windows<kKbit>(L, src, s0, n, r, g, true, ex, out);
}

// one call's parameters
struct StepCfg {
    uint64_t slots;
    Layout lay;
    uint32_t n, heavy_df, min_shared;
    int require_diff;
    bool ranged;              // pairs of rows [row_lo, row_hi) only
    uint32_t row_lo, row_hi;
    uint32_t *d_p, *d_q, *d_w;
    uint64_t cap;
    uint32_t stride;          // edge arrays' element stride (3: interleaved triples)
    const std::vector<unsigned long long>* front_key;  // the batch: pointers and shape
    // scored calls (sb > 0): pair keys carry the k-mer self-score (and sor: the k bit), the tail
    // sums it into d_s (and counts the k bit into d_w1: the second k's w of a fused union)
    int k;
    unsigned sb;
    uint32_t sor;
    uint32_t *d_s, *d_w1, *d_w0;
    // expand only (kmp_dev_pairs_rows_multi): front, buckets and heavy path into this workspace's
    // shard regions, no tail; *n_inc_out = the pair keys written (the fused multi-k tail reads them)
    bool expand_only;
    uint64_t* n_inc_out;
};

// row-block tail geometry: rows per block so that an average block holds about a quarter of
// kPtCap keys (from the expected incidence count)
#ifndef KMP_FT_TARGET
#define KMP_FT_TARGET 2275
#endif
#ifndef KMP_BINSORT_MODE
#define KMP_BINSORT_MODE 1
#endif
bool pt_geometry(const kmp_postings* ws, const StepCfg& c, uint64_t inc, PtGeom* g) {
    g->pbits = bits_for(c.n);
    g->sbits = c.sb;
    g->kbit = c.d_w1 != nullptr;
    const uint32_t rows = c.ranged ? c.row_hi - c.row_lo : c.n;
    const uint64_t est = std::max<uint64_t>(1, inc);
    // rows per block ~ (kPtCap / 2.4) * rows / est, to the nearest power of two: an average block
    // of 2.4-4.8K keys; the first rows (p is the smaller index) hold about twice the average.  A
    // small call (a rank's rows of the k-mer split) takes smaller blocks, down to ~1K keys, so
    // that ~1,000 workgroups still fill the GPU
    // the fast tail (unscored) keeps its blocks well inside its fixed regions and hash table: an
    // average of ~1.1-2.3K keys (KMP_FT_TARGET), twice that in the first rows
    const double target = (!c.sb && ws->fast_tail) ? (double)KMP_FT_TARGET : (double)kPtCap / 2.4;
    const double per_block = std::min(target, std::max(1024.0, (double)est / 1024));
    const double want = per_block * std::max<uint32_t>(rows, 1) / est;
    unsigned rb = 0;
    while (rb < 16 && (double)(1u << rb) * 1.41421356 < want) ++rb;
    rb = std::min(rb, ws->pt_rb_max);  // learned from overflowing blocks
    // the key and one padding bit in a u32 (sparse rows would otherwise ask for wider blocks)
    if (g->pbits + g->sbits > 31) return false;
    rb = std::min(rb, 31 - g->pbits - g->sbits);
    while (rb < 31 && ((rows + (1ull << rb) - 1) >> rb) > kPtMaxBlocks) ++rb;
    if (g->pbits + g->sbits + rb > 31) return false;  // too many rows for one call (kmp_dev_rows_max)
    g->rbits = rb;
    g->nrb = std::max(1u, (uint32_t)((rows + (1ull << rb) - 1) >> rb));
    g->sc = ws->shard_cap;
    g->jt = (uint32_t)((g->sc + kPtTile - 1) / kPtTile);
    g->nshards = kShards;
    g->row0 = c.ranged ? c.row_lo : 0;
    g->flat_n = 0;
    g->min_shared = std::max(1u, c.min_shared);
    g->nprot = c.n;
    g->rowend = c.ranged ? c.row_hi : c.n;
    g->ftcap = kFtCap;
    g->dense = 0;
    if (!c.sb && ws->fast_tail && ws->dense_on && g->pbits < kFdBitsMax) {
        // dense fast tail: the fewest rows per block that the block count allows, when the blocks
        // still average a few hundred keys (a sparse call keeps the hash reduce: clearing 2^15 bins
        // for a handful of keys would dominate)
        unsigned rd = 0;
        while (((rows + (1ull << rd) - 1) >> rd) > kPtMaxBlocks) ++rd;
        const uint64_t nrd = (rows + (1ull << rd) - 1) >> rd;
        if (g->pbits + rd <= kFdBitsMax && est / std::max<uint64_t>(1, nrd) >= 256) {
            g->rbits = rd;
            g->nrb = (uint32_t)std::max<uint64_t>(1, nrd);
            g->dense = 1;  // on the counting partition (blocks of any size)
        }
    }
    // the bin sort for scored blocks only (unscored at config 3: 0.130 -> 0.387 ms);
    // KMP_BINSORT_MODE (A/B builds): 0 the radix sort everywhere, 2 the bin sort everywhere
    g->binsort = KMP_BINSORT_MODE == 2 ? 1 : KMP_BINSORT_MODE == 0 ? 0 : (g->sbits != 0);
    return true;
}

// ws->pt: T (totals) | fcur (fast-tail cursors) | cur | lb (fast-tail look-back, u64) | block starts
// (nrb + 1) | run counts (nrb) | edge offsets (nrb + 1)
struct PtBufs {
    uint32_t *T, *fcur, *cur, *bst, *counts, *eoff;  // row-block totals | fast cursors | scatter cursors | starts | runs | edge offsets
    unsigned long long* lb;
};
PtBufs pt_bufs(kmp_postings* ws, const PtGeom& g, bool reserve, hipError_t* e, hipStream_t st = nullptr) {
    PtBufs b{};
    if (reserve) {
        *e = ws->pt.reserve(5 * (uint64_t)kPtMaxBlocks + 3 * (uint64_t)g.nrb + 2);
        // T (row-block totals) and fcur must be zero: pt_tscan / pt_reduce_fast re-zero what they
        // used, a new allocation (a new pointer or capacity: reserve only reallocates to grow) is
        // cleared once, on the step's stream (a null-stream memset does not order with the
        // non-blocking streams: the first pt_hist of a grown buffer could run before it)
        if (*e == hipSuccess && (ws->pt_zero_p != ws->pt.p || ws->pt_zero_n != ws->pt.n)) {
            *e = hipMemsetAsync(ws->pt.p, 0, 2 * kPtMaxBlocks * sizeof(uint32_t), st);
            ws->pt_zero_p = ws->pt.p;
            ws->pt_zero_n = ws->pt.n;
        }
    }
    b.T = ws->pt.p;
    b.fcur = b.T + kPtMaxBlocks;
    b.cur = b.fcur + kPtMaxBlocks;
    b.lb = reinterpret_cast<unsigned long long*>(b.cur + kPtMaxBlocks);
    b.bst = b.cur + 3 * kPtMaxBlocks;
    b.counts = b.bst + g.nrb + 1;
    b.eoff = b.counts + g.nrb;
    return b;
}

// the fast row-block tail applies: unscored keys, at most kFtRowsMax rows per block, not turned off
// for the shape
bool pt_fast(const kmp_postings* ws, const PtGeom& g) {
    return ws->fast_tail && !g.sbits && g.rbits <= 10 && (1u << g.rbits) <= kFtRowsMax;
}

// spill segments: every one holds more than kHeavySub keys (a heavy group, or a whole bucket)
uint32_t seg_capacity(const kmp_postings* ws) {
    return (uint32_t)std::min<uint64_t>(ws->spill_cap * kShards / kHeavySub + 64, 1u << 30);
}

BucketArgs bucket_args(kmp_postings* ws, const StepCfg& c, bool spill) {
    BucketArgs a{};
    const uint32_t nb = 1u << c.lay.bbits;
    a.sorted = ws->sorted.p;
    a.bstart = ws->cnt.p;
    if (ws->cur_used) {
        a.bstart = ws->cur.p;  // bucket counts
        a.capb = ws->cg.capb;
        a.vreg = ws->cg.vreg;
    }
    a.lay = c.lay;
    a.mul = 1u << bits_for(c.n);  // pair key p << pbits | q (the row-block tail's key)
    a.require_diff = c.require_diff;
    a.heavy_df = c.heavy_df;
    a.row_lo = c.ranged ? c.row_lo : 0;
    a.row_hi = c.ranged ? c.row_hi : c.n;
    a.out = ws->inc_sorted.p;
    a.shard_cap = ws->shard_cap;
    a.gstats = ws->bstats.p;
    a.cursor = ws->bstats.p + kRbCursor;
    a.flags = ws->flags.p;
    a.list = ws->cnt.p + nb + 1;
    a.list_count = ws->flags.p + kFlList;
    a.spill = spill ? ws->spill.p : nullptr;
    a.spill_cap = ws->spill_cap;
    a.spill_cursor = ws->bstats.p + kRbSpill;
    a.seg = ws->hseg.p;
    a.seg_cap = seg_capacity(ws);
    a.k = c.k;
    a.sb = c.sb;
    a.sor = c.sor;
    a.spill_all = c.ranged && ws->reuse && ws->flat_heavy && ws->spill_all_on;
    if (ws->route_send && !c.sb) {
        a.send = ws->route_send;
        a.send_cap = ws->route_cap;
        a.send_sub = ws->route_cap / kShards;
        a.dcur = ws->split_cur.p;
        a.rows = ws->route_rows;
    }
    return a;
}

// buffers of one step (reserved before any launch, so a capture allocates nothing)
int step_reserve(kmp_postings* ws, const StepCfg& c, const PtGeom& g, hipStream_t st) {
    if (ws->shard_cap < ws->shard_floor) ws->shard_cap = ws->shard_floor;
    const uint64_t total = ws->shard_cap * kShards;
    PG(ws->keys.reserve(c.slots));
    PG(ws->sorted.reserve(c.slots));
    PG(ws->flags.reserve(kFlN));
    PG(ws->cnt.reserve(2 * ((uint64_t)1 << c.lay.bbits) + 2));
    PG(ws->bstats.reserve(kGsWords));
    PG(ws->small.reserve(16));  // [1] run count, [2] largest row block
    PG(ws->inc_sorted.reserve(total));
    if (!c.expand_only) {  // an expand-only call leaves the tail (and its staging) to tail_multi
        // u32 row-block keys (pt_scatter; the fast tail's fixed regions) ...
        PG(ws->inc.reserve(pt_fast(ws, g) && !g.dense ? std::max<uint64_t>(total, (uint64_t)g.nrb * g.ftcap / 2)
                                                         : total));
        PG(ws->uniq.reserve(total));  // ... staged p | q (u32 each)
        PG(ws->w.reserve(total));     // ... staged w
        if (c.sb) PG(ws->stg2.reserve(2 * total));  // ... staged scores | second-k weights
    }
    PG(ws->spill.reserve(ws->spill_cap * kShards));
    PG(ws->hseg.reserve(seg_capacity(ws)));
    PG(ws->ovf.reserve((uint64_t)g.nrb + 1));
    if (!ws->hrb) PG(hipHostMalloc((void**)&ws->hrb, kRbWords * sizeof(unsigned long long), hipHostMallocCoherent));
    hipError_t e = hipSuccess;
    pt_bufs(ws, g, true, &e, st);
    PG(e);
    return KMP_OK;
}

// front: clear, keys, level 2 (or the bucket sort), bucket kernels
template <class MakeKeys>
int enqueue_front(kmp_postings* ws, MakeKeys& make_keys, const StepCfg& c, bool spill, hipStream_t st,
                  bool keys = true) {
    // the residue front folds the clear into its first kernel (chunk_desc); any other: a kernel here
    ws->defer_clear = keys && ws->clear_in_keys;
    if (!ws->defer_clear)
        step_clear_kernel<<<1, 256, 0, st>>>(ws->flags.p, ws->bstats.p, ws->clear_extra, ws->clear_n);
    ws->mark(0, st);
    if (keys) {  // else: the keys grouped by bucket of the last call (front reuse)
        PG(make_keys(c.lay, st));
        if (ws->defer_clear) {  // (a key path that did not take it)
            ws->defer_clear = false;
            return KMP_EINVAL;
        }
        ws->mark(1, st);
        int rc = bucket_group(ws, ws->keys.p, c.slots, c.lay, st);  // marks 2
        if (rc != KMP_OK) return rc;
    } else {
        ws->mark(1, st);
        ws->mark(2, st);
    }
    const BucketArgs a = bucket_args(ws, c, spill);
    const BpDigits dg = bp_digits(c.lay);
    uint32_t c0, c1;
    own_bins(ws, dg, &c0, &c1);
    const uint32_t b0 = c0 * dg.nb2, nbk = (c1 - c0) * dg.nb2;  // the call's buckets
    // the large-bucket kernel loops over its list: a grid sized from the last call's list (a
    // thousand idle 1,024-thread workgroups cost ~5 us); a bucket-range share of the k-mer split
    // lists about 1/parts of them
    const uint32_t lg = ws->bin_hi ? std::max<uint32_t>(64, kBucketLargeGrid * (c1 - c0) / dg.nb1) : ws->large_grid;
    ws->large_used = lg;
    if (spill) ws->front_all = a.spill_all != 0;  // what the spill of this front will hold
    if (a.spill_all && !a.spill) return KMP_OK;  // every bucket already in the heavy path (a later pass)
    if (c.sb) {
        if (c.ranged) launch_buckets<true, true>(a, b0, nbk, lg, st);
        else launch_buckets<false, true>(a, b0, nbk, lg, st);
    } else {
        if (c.ranged) launch_buckets<true, false>(a, b0, nbk, lg, st);
        else launch_buckets<false, false>(a, b0, nbk, lg, st);
    }
    PG(hipGetLastError());
    return KMP_OK;
}

// the scored call's staging (ws->stg2: scores | second-k weights, total each) and outputs
PtScoreOut pt_score_out(kmp_postings* ws, const StepCfg& c, uint64_t total) {
    if (!c.sb) return PtScoreOut{};
    return PtScoreOut{ws->stg2.p, ws->stg2.p + total, c.d_s, c.d_w1, c.d_w0};
}

// tail over the shard regions, then the read-back; marks 4, 5, 6
// in: the pair keys (g.nshards regions of g.sc keys, counts in cursor; or, g.flat_n, one array
// padded with kNoKey); total: capacity of the staging arrays (>= every key)
int enqueue_tail_in(kmp_postings* ws, const StepCfg& c, const PtGeom& g, const unsigned long long* in,
                    const unsigned long long* cursor, uint64_t total, hipStream_t st) {
    hipError_t e = hipSuccess;
    const PtBufs b = pt_bufs(ws, g, false, &e);
    uint32_t* keys32 = reinterpret_cast<uint32_t*>(ws->inc.p);
    if (pt_fast(ws, g)) {  // one reduce that writes the edges (marks 4, 5, 6)
        if (g.dense) {  // the counting partition (blocks of any size), the dense reduce
            pt_hist_kernel<<<dim3(g.jt, g.nshards), kPtThreads, 0, st>>>(in, cursor, g, b.T);
            pt_tscan_kernel<<<1, kPtScanThreads, 0, st>>>(b.T, g.nrb, b.bst, b.cur, ws->small.p + 2);
            pt_scatter_kernel<<<dim3(g.jt, g.nshards), kPtThreads, 0, st>>>(in, cursor, g, b.cur, keys32);
            ws->mark(4, st);
            if (g.nrb) {  // the look-back words (the capped scatter clears them otherwise)
                PG(hipMemsetAsync(b.lb, 0, (size_t)g.nrb * sizeof(unsigned long long), st));
            }
            pt_reduce_dense_kernel<<<g.nrb, kFtThreads, 0, st>>>(keys32, b.bst, g, b.lb, c.d_p, c.d_q, c.d_w, c.cap,
                                                                  c.stride,
                                                                  PtPack{ws->bstats.p, ws->flags.p, nullptr, ws->hrb},
                                                                  ws->small.p + 1);
            ws->mark(5, st);
            ws->mark(6, st);
            PG(hipGetLastError());
            return KMP_OK;
        }
        const uint32_t jt = (uint32_t)(((g.flat_n ? g.flat_n : g.sc) + kFtScTile - 1) / kFtScTile);
        pt_scatter_capped_kernel<<<dim3(jt, g.nshards), kFtScThreads, 0, st>>>(in, cursor, g, b.fcur, keys32, b.lb);
        ws->mark(4, st);
        {
            pt_reduce_fast_kernel<<<g.nrb, kFtThreads, 0, st>>>(keys32, b.fcur, g, b.lb, c.d_p, c.d_q, c.d_w, c.cap,
                                                                 c.stride,
                                                                 PtPack{ws->bstats.p, ws->flags.p, nullptr, ws->hrb},
                                                                 ws->small.p + 1);
        }
        ws->mark(5, st);
        ws->mark(6, st);
        PG(hipGetLastError());
        return KMP_OK;
    }
    uint32_t* stage_p = reinterpret_cast<uint32_t*>(ws->uniq.p);
    uint32_t* stage_q = stage_p + total;
    pt_hist_kernel<<<dim3(g.jt, g.nshards), kPtThreads, 0, st>>>(in, cursor, g, b.T);
    pt_tscan_kernel<<<1, kPtScanThreads, 0, st>>>(b.T, g.nrb, b.bst, b.cur, ws->small.p + 2);
    ws->mark(4, st);
    pt_scatter_kernel<<<dim3(g.jt, g.nshards), kPtThreads, 0, st>>>(in, cursor, g, b.cur, keys32);
    const PtScoreOut so = pt_score_out(ws, c, total);
    if (g.sbits && g.kbit)
        pt_reduce_scored_kernel<true><<<g.nrb, kPtRThreads, 0, st>>>(keys32, BlkSrc{b.bst, nullptr, nullptr}, g, ws->flags.p, ws->ovf.p, stage_p,
                                                                     stage_q, ws->w.p, ws->stg2.p, ws->stg2.p + total,
                                                                     b.counts);
    else if (g.sbits)
        pt_reduce_scored_kernel<false><<<g.nrb, kPtRThreads, 0, st>>>(keys32, BlkSrc{b.bst, nullptr, nullptr}, g, ws->flags.p, ws->ovf.p, stage_p,
                                                                      stage_q, ws->w.p, ws->stg2.p, nullptr, b.counts);
    else
        pt_reduce_kernel<<<g.nrb, kPtRThreads, 0, st>>>(keys32, b.bst, g, ws->flags.p, ws->ovf.p, stage_p, stage_q,
                                                        ws->w.p, b.counts);
    if (pt_rowhist_ok(g))  // one-row blocks above kPtCap: finished here (none listed: every workgroup exits)
        pt_rowhist_kernel<<<kRowHistGrid, kRowHistThreads, 0, st>>>(keys32, b.bst, g, ws->flags.p, ws->ovf.p,
                                                                    stage_p, stage_q, ws->w.p, b.counts);
    ws->mark(5, st);
    // edge offsets computed by the emit blocks themselves (no pt_offsets launch); + read-back
    pt_emit_kernel<<<g.nrb, 256, 0, st>>>(stage_p, stage_q, ws->w.p, b.bst, b.counts, nullptr, c.d_p, c.d_q, c.d_w,
                                          c.cap, c.stride, PtPack{ws->bstats.p, ws->flags.p, ws->small.p + 1, ws->hrb},
                                          ws->small.p + 1, so);
    ws->mark(6, st);
    PG(hipGetLastError());
    return KMP_OK;
}

// the step's tail: the shard regions the bucket kernels filled
int enqueue_tail(kmp_postings* ws, const StepCfg& c, const PtGeom& g, hipStream_t st) {
    return enqueue_tail_in(ws, c, g, ws->inc_sorted.p, ws->bstats.p + kRbCursor, ws->shard_cap * kShards, st);
}

// the listed row blocks (above kPtCap keys): the composite sort + encode above, then offsets
// and emit again; host-synchronous, returns the edge count in *edges

// bsrc (sub-blocks; nullptr: the row blocks) / nblk, counts, eoff: the blocks the reduce ran over
// and their run counts and edge offsets (sub-block mode: ws->dsc)
int pt_finish_overflow(kmp_postings* ws, const StepCfg& c, const PtGeom& g, uint32_t m, uint64_t* edges,
                       hipStream_t st, uint64_t total = 0, const BlkSrc* bsrc = nullptr, uint32_t nblk = 0,
                       uint32_t* bcounts = nullptr, uint32_t* beoff = nullptr, const uint32_t* bkeys = nullptr) {
    hipError_t e = hipSuccess;
    PtBufs b = pt_bufs(ws, g, false, &e);
    const BlkSrc bs = bsrc ? *bsrc : BlkSrc{b.bst, nullptr, nullptr};
    const uint32_t nb = bsrc ? nblk : g.nrb;
    if (bsrc) {
        b.counts = bcounts;
        b.eoff = beoff;
    }
    if (!total) total = ws->shard_cap * kShards;
    const uint32_t* keys32 = bkeys ? bkeys : reinterpret_cast<uint32_t*>(ws->inc.p);
    uint32_t* stage_p = reinterpret_cast<uint32_t*>(ws->uniq.p);
    uint32_t* stage_q = stage_p + total;
    const unsigned kb = g.pbits + g.sbits + g.rbits, mb = bits_for((uint64_t)m + 1);
    if (kb + mb > 63) return KMP_EINVAL;
    PG(ws->ovx.reserve(m + 1));
    unsigned long long* xoff = ws->ovx.p;
    pt_ovf_sizes_kernel<<<(m + 256) / 256, 256, 0, st>>>(ws->ovf.p, m, bs, xoff);
    size_t t0 = 0;
    PG(rocprim::exclusive_scan(nullptr, t0, xoff, xoff, 0ull, (size_t)m + 1, rocprim::plus<unsigned long long>(), st));
    PG(ws->tmp.reserve(std::max(t0, ws->tmp.n)));
    PG(rocprim::exclusive_scan(ws->tmp.p, t0, xoff, xoff, 0ull, (size_t)m + 1, rocprim::plus<unsigned long long>(),
                               st));
    unsigned long long nx = 0;
    PG(hipMemcpyAsync(&nx, xoff + m, 8, hipMemcpyDeviceToHost, st));
    PG(hipStreamSynchronize(st));
    if (nx > 0xFFFFFFFFull) return KMP_ENOMEM;
    PG(ws->ovk.reserve(3 * nx + 1));  // tagged keys | sorted | runs
    PG(ws->ovr.reserve(3 * (nx + 1) + m + 1));  // w | keep | kept positions | first run per block
    unsigned long long *x = ws->ovk.p, *xs = x + nx, *uq = xs + nx;
    uint32_t *rw = ws->ovr.p, *keep = rw + nx + 1, *kpos = keep + nx + 1, *first = kpos + nx + 1;
    uint32_t* nruns = ws->small.p + 4;
    const uint32_t gx = (uint32_t)std::min<unsigned long long>((nx / m + 255) / 256 + 1, 64);
    pt_ovf_gather_kernel<<<dim3(gx, m), 256, 0, st>>>(ws->ovf.p, bs, xoff, keys32, kb, x);
    size_t t1 = 0, t2 = 0, t3 = 0;
    PG(rocprim::radix_sort_keys<SortCfg>(nullptr, t1, x, xs, (size_t)nx, 0u, kb + mb, st));
    PG(rocprim::run_length_encode(nullptr, t2, xs, (unsigned)nx, uq, rw, nruns, st));
    PG(rocprim::exclusive_scan(nullptr, t3, keep, kpos, 0u, (size_t)nx + 1, rocprim::plus<uint32_t>(), st));
    PG(ws->tmp.reserve(std::max({t1, t2, t3, ws->tmp.n})));
    PG(rocprim::radix_sort_keys<SortCfg>(ws->tmp.p, t1, x, xs, (size_t)nx, 0u, kb + mb, st));
    const uint32_t gr = (uint32_t)std::min<unsigned long long>((nx + 256) / 256, 4096);
    if (g.sbits) {
        // scored: runs of equal (tag, pair) = sorted key >> sbits, reduced to (w, w1, score)
        PG(ws->ova.reserve(3 * (nx + 1)));
        RunAgg* agg = reinterpret_cast<RunAgg*>(ws->ova.p);
        auto kin = rocprim::make_transform_iterator(xs, PairOfKey{g.sbits});
        auto vin = rocprim::make_transform_iterator(xs, AggOfKey{});
        size_t t4 = 0;
        PG(rocprim::reduce_by_key(nullptr, t4, kin, vin, (size_t)nx, uq, agg, nruns, RunAggPlus{},
                                  rocprim::equal_to<unsigned long long>(), st));
        PG(ws->tmp.reserve(std::max({t4, t3, ws->tmp.n})));
        PG(rocprim::reduce_by_key(ws->tmp.p, t4, kin, vin, (size_t)nx, uq, agg, nruns, RunAggPlus{},
                                  rocprim::equal_to<unsigned long long>(), st));
        pt_ovf_keep_scored_kernel<<<gr, 256, 0, st>>>(uq, agg, nruns, kb - g.sbits, g.min_shared, g.kbit, keep, first);
        PG(rocprim::exclusive_scan(ws->tmp.p, t3, keep, kpos, 0u, (size_t)nx + 1, rocprim::plus<uint32_t>(), st));
        const PtScoreOut so = pt_score_out(ws, c, total);
        pt_ovf_stage_scored_kernel<<<gr, 256, 0, st>>>(ws->ovf.p, m, bs, g, uq, agg, nruns, keep, kpos, first,
                                                       stage_p, stage_q, ws->w.p, ws->stg2.p, ws->stg2.p + total,
                                                       b.counts);
        if (bsrc) {  // the caller scans the sub-blocks' counts and emits
            PG(hipStreamSynchronize(st));
            return KMP_OK;
        }
        pt_offsets_kernel<<<1, kPtScanThreads, 0, st>>>(b.counts, nb, b.eoff, ws->small.p + 1);
        pt_emit_kernel<<<nb, 256, 0, st>>>(stage_p, stage_q, ws->w.p, b.bst, b.counts, b.eoff, c.d_p, c.d_q, c.d_w,
                                           c.cap, c.stride, PtPack{}, nullptr, so);
        uint32_t ne = 0;
        PG(hipMemcpyAsync(&ne, ws->small.p + 1, 4, hipMemcpyDeviceToHost, st));
        PG(hipStreamSynchronize(st));
        *edges = ne;
        return KMP_OK;
    }
    PG(rocprim::run_length_encode(ws->tmp.p, t2, xs, (unsigned)nx, uq, rw, nruns, st));
    pt_ovf_keep_kernel<<<gr, 256, 0, st>>>(uq, rw, nruns, kb, g.min_shared, keep, first);
    PG(rocprim::exclusive_scan(ws->tmp.p, t3, keep, kpos, 0u, (size_t)nx + 1, rocprim::plus<uint32_t>(), st));
    pt_ovf_stage_kernel<<<gr, 256, 0, st>>>(ws->ovf.p, m, b.bst, g, uq, rw, nruns, kpos, first, stage_p, stage_q,
                                            ws->w.p, b.counts);
    pt_offsets_kernel<<<1, kPtScanThreads, 0, st>>>(b.counts, g.nrb, b.eoff, ws->small.p + 1);
    pt_emit_kernel<<<g.nrb, 256, 0, st>>>(stage_p, stage_q, ws->w.p, b.bst, b.counts, b.eoff, c.d_p, c.d_q, c.d_w,
                                          c.cap, c.stride);
    uint32_t ne = 0;
    PG(hipMemcpyAsync(&ne, ws->small.p + 1, 4, hipMemcpyDeviceToHost, st));
    PG(hipStreamSynchronize(st));
    *edges = ne;
    return KMP_OK;
}

// Heavy path (after the front): gather, sort and compact the spill once per front; plan and
// expand the rows of this call into the shard regions.  stats: post the heavy k-mers' statistics
// (once per batch).  No host round trip: the element, k-mer and run counts stay on the device
// (hoff tail), the arrays are sized by the spill count m, and the plan and expansion grids cover
// that bound.
__global__ void heavy_totals_kernel(const uint32_t* __restrict__ cnt, const unsigned long long* __restrict__ off,
                                    uint64_t nt, unsigned long long* __restrict__ tot) {
    const uint32_t a = threadIdx.x;  // elements, k-mers, runs
    if (a < 3) tot[a] = nt ? off[a * (nt + 1) + nt - 1] + cnt[a * nt + nt - 1] : 0ull;
}
__global__ void heavy_sentinel_kernel(const unsigned long long* __restrict__ tot, uint64_t* __restrict__ GS,
                                      uint64_t* __restrict__ RH) {
    if (threadIdx.x == 0) GS[tot[1]] = tot[0];
    if (threadIdx.x == 1 && RH) RH[tot[2]] = tot[0];
}

// one workgroup: exclusive scans of the per-tile counts (elements | k-mers | runs, na arrays of nt
// <= kHvScanMax), their totals in tot, and the sentinels GS[ng] = RH[nr] = ne (compact writes
// the entries before them); in place of na device-wide scans + heavy_totals + heavy_sentinel
constexpr uint32_t kHvScanThreads = 1024, kHvScanMax = 8 * kHvScanThreads;
__global__ __launch_bounds__(kHvScanThreads) void heavy_tscan_kernel(const uint32_t* __restrict__ cnt, uint32_t nt,
                                                                     uint32_t na, unsigned long long* __restrict__ off,
                                                                     unsigned long long* __restrict__ tot,
                                                                     uint64_t* __restrict__ GS,
                                                                     uint64_t* __restrict__ RH) {
    __shared__ uint32_t wave_tot[kHvScanThreads / 64];
    __shared__ unsigned long long s_tot[3];
    const uint32_t q = (nt + kHvScanThreads - 1) / kHvScanThreads, c0 = threadIdx.x * q;
    for (uint32_t a = 0; a < na; ++a) {
        uint32_t v[8], sum = 0;
#pragma unroll
        for (uint32_t i = 0; i < 8; ++i) {
            v[i] = i < q && c0 + i < nt ? cnt[a * nt + c0 + i] : 0u;
            sum += v[i];
        }
        uint32_t excl, total;  // per-tile counts are <= 4,096 and nt <= 8,192: u32 totals
        block_scan_n<kHvScanThreads>(sum, excl, total, wave_tot);
#pragma unroll
        for (uint32_t i = 0; i < 8; ++i)
            if (i < q && c0 + i < nt) {
                off[a * (nt + 1) + c0 + i] = excl;
                excl += v[i];
            }
        if (threadIdx.x == 0) {
            tot[a] = total;
            s_tot[a] = total;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (na < 3) tot[2] = 0;
        GS[s_tot[1]] = s_tot[0];
        if (RH && na == 3) RH[s_tot[2]] = s_tot[0];
    }
}

int heavy_phase(kmp_postings* ws, const StepCfg& c, uint64_t m, bool stats, hipStream_t st) {
    const Layout& lay = c.lay;
    HeavyOrder ho{};
    ho.cb = lay.clsbits;
    ho.hshift = lay.hshift;
    ho.pbits = lay.hshift - lay.clsbits;
    // class order skips same-class pairs without testing them, but puts the rows of a range
    // anywhere in a k-mer's elements: a ranged call (a pass or a rank's rows) would walk every
    // pair of every frequent k-mer on every pass.  Plain order keeps a range's rows contiguous, so
    // a pass enumerates only its own rows' pairs (testing the class per pair).
    ho.cls = c.require_diff && lay.clsbits > 0 && !c.ranged;
    if (ws->heavy_ready && ws->h_cls != ho.cls) {  // the kept spill, compacted again in this order
        ws->heavy_ready = false;
        m = ws->h_m;
    }
    // 256 x 256 tiles: one workgroup's write stream bounds a tile (a 256 x 2,048 block of pairs
    // left one CU writing 4 MB), and a filtered tile (the class test per pair) takes its kept
    // partners through a per-row bit mask of the chunk (8 words a row)
    ho.hj = kHvJ;
    // the passes of one batch (front reuse), plain order: the rows drive the expansion
    const bool flat = c.ranged && !ho.cls && ws->flat_heavy && ws->reuse;
    if (flat && ws->heavy_ready && !ws->h_kg) {  // compacted without each element's k-mer: again
        ws->heavy_ready = false;
        m = ws->h_m;
    }
    if (!ws->heavy_ready) {
        ws->h_flat_ready = false;
        if (flat) PG(ws->hKG.reserve(m + 1));
        const uint64_t nt = (m + kHvTile - 1) / kHvTile;
        PG(ws->hkeys.reserve(m));
        PG(ws->hsorted.reserve(m));
        PG(ws->hcnt.reserve(3 * nt + 1));
        PG(ws->hoff.reserve(3 * (nt + 1) + 4));
        PG(ws->hE.reserve(m + 1));
        PG(ws->hGS.reserve(m + 1));
        PG(ws->hGH.reserve(m + 1));
        if (ho.cls) {
            PG(ws->hrun.reserve(m + 1));
            PG(ws->hRH.reserve(m + 1));
        }
        // the spill's region fill levels: this front's cursors, kept aside so that a reused front
        // (its cursors cleared by the next call) can be compacted again in the other order
        PG(ws->hcur.reserve(kShards));
        if (!ws->hcur_valid) {
            PG(hipMemcpyAsync(ws->hcur.p, ws->bstats.p + kRbSpill, kShards * sizeof(unsigned long long),
                              hipMemcpyDeviceToDevice, st));
            ws->hcur_valid = true;
        }
        const unsigned long long* spill_cursor = ws->hcur.p;
        if (ws->h_segs && ws->h_segs <= seg_capacity(ws) && ws->h_segmax <= kSegLarge) {
            const uint32_t ns = (uint32_t)ws->h_segs;
            if (ho.cls)
                heavy_segclass_kernel<<<ns, kScThreads, 0, st>>>(ws->spill.p, ws->spill_cap, spill_cursor, ws->hseg.p,
                                                                 ho, ws->hsorted.p);
            heavy_segsort_bitonic_kernel<kSegSmall, 256><<<ns, 256, 0, st>>>(
                ws->spill.p, ws->spill_cap, spill_cursor, ws->hseg.p, ho, ws->hsorted.p);
            if (ws->h_segmax > kSegSmall)
                heavy_segsort_kernel<kSegSmall, kSegLarge><<<ns, kSegLarge / kSegItems, 0, st>>>(
                    ws->spill.p, ws->spill_cap, spill_cursor, ws->hseg.p, ho, ws->hsorted.p);
        } else {  // a segment above the LDS sort: gather and one radix sort
            gather_shards_kernel<<<dim3((uint32_t)std::min<uint64_t>((ws->spill_cap + 255) / 256, 1024), kShards),
                                   256, 0, st>>>(ws->spill.p, ws->spill_cap, spill_cursor, ho, ws->hkeys.p);
            const unsigned lo_bit = ho.eshift();
            size_t tb = 0;
            PG(rocprim::radix_sort_keys<SortCfg>(nullptr, tb, ws->hkeys.p, ws->hsorted.p, (size_t)m, lo_bit, 63u, st));
            PG(ws->tmp.reserve(std::max(tb, ws->tmp.n)));
            PG(rocprim::radix_sort_keys<SortCfg>(ws->tmp.p, tb, ws->hkeys.p, ws->hsorted.p, (size_t)m, lo_bit, 63u,
                                                 st));
        }
        uint32_t* cnt = ws->hcnt.p;             // elements | k-mers | runs, nt each
        unsigned long long* off = ws->hoff.p;   // their exclusive scans, nt + 1 apart
        unsigned long long* tot = off + 3 * (nt + 1);
        heavy_scan_kernel<<<(uint32_t)nt, kHvThreads, 0, st>>>(ws->hsorted.p, m, ho, cnt, cnt + nt, cnt + 2 * nt);
        uint64_t* GS = reinterpret_cast<uint64_t*>(ws->hGS.p);
        uint64_t* RH = ho.cls ? reinterpret_cast<uint64_t*>(ws->hRH.p) : nullptr;
        const uint32_t na = ho.cls ? 3 : 2;
        const bool one_wg = nt <= kHvScanMax;
        if (one_wg) {
            heavy_tscan_kernel<<<1, kHvScanThreads, 0, st>>>(cnt, (uint32_t)nt, na, off, tot, GS, RH);
        } else {
            size_t t1 = 0;
            PG(rocprim::exclusive_scan(nullptr, t1, cnt, off, 0ull, (size_t)nt, rocprim::plus<unsigned long long>(),
                                       st));
            PG(ws->tmp.reserve(std::max(t1, ws->tmp.n)));
            for (uint32_t a = 0; a < na; ++a)
                PG(rocprim::exclusive_scan(ws->tmp.p, t1, cnt + a * nt, off + a * (nt + 1), 0ull, (size_t)nt,
                                           rocprim::plus<unsigned long long>(), st));
            heavy_totals_kernel<<<1, 64, 0, st>>>(cnt, off, nt, tot);
        }
        heavy_compact_kernel<<<(uint32_t)nt, kHvThreads, 0, st>>>(
            ws->hsorted.p, m, ho, reinterpret_cast<const uint64_t*>(off),
            reinterpret_cast<const uint64_t*>(off + nt + 1), reinterpret_cast<const uint64_t*>(off + 2 * (nt + 1)),
            ws->hE.p, GS, ho.cls ? ws->hrun.p : nullptr, RH, ws->hGH.p, flat ? ws->hKG.p : nullptr);
        ws->h_kg = flat;
        if (!one_wg) heavy_sentinel_kernel<<<1, 64, 0, st>>>(tot, GS, RH);
        PG(hipGetLastError());
        ws->heavy_ready = true;
        ws->h_m = m;
        ws->h_cls = ho.cls;
        ws->h_tot = tot;
    }
    if (ws->h_cls != ho.cls) return KMP_EINVAL;  // (compacted above in this call's order)
    bool index_built = false;
    if (flat && !ws->h_flat_ready) {
        index_built = true;
        // once per compaction: the per-protein index (one read-back: the element and k-mer counts)
        unsigned long long ht[2] = {0, 0};
        PG(hipMemcpyAsync(ht, ws->h_tot, sizeof(ht), hipMemcpyDeviceToHost, st));
        PG(hipStreamSynchronize(st));
        if (ht[0] >= (1ull << 32)) return KMP_EINVAL;
        const uint32_t np = c.n;
        PG(ws->hPE.reserve(ht[0] + 1));
        PG(ws->hPO.reserve((uint64_t)np + 1));
        PG(ws->hPC.reserve((uint64_t)np + 1));
        PG(hipMemsetAsync(ws->hPC.p, 0, ((size_t)np + 1) * sizeof(uint32_t), st));
        const uint32_t grid = (uint32_t)std::min<uint64_t>((ht[0] + 255) / 256 + 1, 16384);
        heavy_pcount_kernel<<<grid, 256, 0, st>>>(ws->hE.p, ws->h_tot, ho.cb, ws->hPC.p);
        size_t tb = 0;
        PG(rocprim::exclusive_scan(nullptr, tb, ws->hPC.p, ws->hPO.p, 0u, (size_t)np + 1, rocprim::plus<uint32_t>(), st));
        PG(ws->tmp.reserve(std::max(tb, ws->tmp.n)));
        PG(rocprim::exclusive_scan(ws->tmp.p, tb, ws->hPC.p, ws->hPO.p, 0u, (size_t)np + 1, rocprim::plus<uint32_t>(),
                                   st));
        PG(hipMemsetAsync(ws->hPC.p, 0, ((size_t)np + 1) * sizeof(uint32_t), st));
        heavy_pscatter_kernel<<<grid, 256, 0, st>>>(ws->hE.p, ws->h_tot, ho.cb, ws->hPO.p, ws->hPC.p, ws->hPE.p);
        PG(hipGetLastError());
        ws->hPOh.resize((size_t)np + 1);
        PG(hipMemcpyAsync(ws->hPOh.data(), ws->hPO.p, ((size_t)np + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        PG(hipStreamSynchronize(st));
        ws->h_ng = ht[1];
        ws->h_flat_ready = true;
    }
    // bound on the k-mer count (device: h_tot[1]); exact once the flat index read it back
    const uint64_t ngb = flat ? ws->h_ng : ws->h_m;
    if (ngb == 0) return KMP_OK;
    const uint32_t row_lo = c.ranged ? c.row_lo : 0, row_hi = c.ranged ? c.row_hi : c.n;
    const uint64_t* GS = reinterpret_cast<const uint64_t*>(ws->hGS.p);
    const uint64_t* RH = ho.cls ? reinterpret_cast<const uint64_t*>(ws->hRH.p) : nullptr;
    const uint32_t* RUN = ho.cls ? ws->hrun.p : nullptr;
    if (flat) {
        // the plan only for the k-mers' statistics, on the pass that built the index (they do not
        // change between the passes; a spill-all batch holds every k-mer, ~10^8 at k = 7)
        if (stats && index_built)
            heavy_plan_kernel<<<(uint32_t)((ngb + 1 + 255) / 256), 256, 0, st>>>(
                ws->hE.p, GS, ngb + 1, ws->h_tot + 1, ho, RUN, RH, 0, row_lo, row_hi, c.heavy_df, 1, 0, ws->bstats.p,
                nullptr, nullptr, nullptr, nullptr);
        const uint32_t a0 = ws->hPOh[row_lo], a1 = ws->hPOh[row_hi];
        if (a1 > a0)
            heavy_flat_kernel<<<(a1 - a0 + kHfThreads - 1) / kHfThreads, kHfThreads, 0, st>>>(
                ws->hE.p, GS, ws->hKG.p, ws->hGH.p, ws->hPE.p, a0, a1, ho.cb, 1u << bits_for(c.n), c.require_diff,
                c.heavy_df, c.k, c.sb, c.sor, ws->inc_sorted.p, ws->shard_cap, ws->bstats.p + kRbCursor,
                ws->bstats.p);
        PG(hipGetLastError());
        return KMP_OK;
    }
    PG(ws->hgi.reserve(2 * (ngb + 1)));
    PG(ws->htc.reserve(ngb + 1));
    PG(ws->htoff.reserve(ngb + 1));
    PG(ws->hblk.reserve(2 * (ngb + ngb / kHvI + 2)));
    uint32_t* BT = ws->hblk.p;
    uint32_t* BP = BT + ngb + ngb / kHvI + 2;
    heavy_plan_kernel<<<(uint32_t)((ngb + 1 + 255) / 256), 256, 0, st>>>(
        ws->hE.p, GS, ngb + 1, ws->h_tot + 1, ho, RUN, RH, ho.cls && !c.ranged ? 1 : 0, row_lo, row_hi, c.heavy_df,
        stats ? 1 : 0, 1, ws->bstats.p, ws->hgi.p, BT, BP, ws->htc.p);
    size_t t2 = 0;
    PG(rocprim::exclusive_scan(nullptr, t2, ws->htc.p, ws->htoff.p, 0ull, (size_t)ngb + 1,
                               rocprim::plus<unsigned long long>(), st));
    PG(ws->tmp.reserve(std::max(t2, ws->tmp.n)));
    PG(rocprim::exclusive_scan(ws->tmp.p, t2, ws->htc.p, ws->htoff.p, 0ull, (size_t)ngb + 1,
                               rocprim::plus<unsigned long long>(), st));
    // tiles = htoff[ng] (device); the grid strides them
    const uint32_t grid = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(ngb / 4, 256), 8192);
    heavy_expand_kernel<<<grid, kHvI, 0, st>>>(ws->hE.p, GS, ws->hgi.p, BT, BP, RUN, RH, ws->htoff.p, ws->h_tot + 1,
                                               ho, 1u << bits_for(c.n), c.require_diff, c.ranged ? 1 : 0, row_lo,
                                               row_hi, ws->inc_sorted.p, ws->shard_cap, ws->bstats.p + kRbCursor,
                                               ws->bstats.p, ws->hGH.p, c.k, c.sb, c.sor);
    PG(hipGetLastError());
    return KMP_OK;
}

// enqueue the fused step: replay the captured graph when the shape matches the capture, capture
// it when the shape repeats a plain run (buffers sized), else run plain
// enqueue(s) on `st` as a HIP graph of `slot`: replayed when key matches its capture, captured when
// key repeats the last plain run (every buffer sized by then), else run plain.  key must hold
// every input of the sequence (shape, pointers, learned capacities, g_grow_gen).
template <class Enqueue>
int slot_launch(kmp_postings* ws, kmp_postings::GraphSlot& slot, std::vector<unsigned long long> key,
                Enqueue enqueue, hipStream_t st) {
    key.push_back(g_grow_gen.load());
    if (!ws->graph_on) return enqueue(st);
    if (slot.gexec && slot.key == key) {
        PG(hipGraphLaunch(slot.gexec, st));
        ++ws->graph_replays;
        return KMP_OK;
    }
    if (slot.seen != key) {
        slot.seen = key;
        return enqueue(st);
    }
    if (slot.gexec) (void)hipGraphExecDestroy(slot.gexec);
    slot.gexec = nullptr;
    slot.key.clear();
    if (!ws->cst && hipStreamCreateWithFlags(&ws->cst, hipStreamNonBlocking) != hipSuccess) ws->cst = nullptr;
    hipGraph_t gr = nullptr;
    if (!ws->cst || hipStreamBeginCapture(ws->cst, hipStreamCaptureModeRelaxed) != hipSuccess) {
        (void)hipGetLastError();
        return enqueue(st);
    }
    const unsigned long long gen = g_grow_gen.load();
    int rc = enqueue(ws->cst);
    hipError_t e = hipStreamEndCapture(ws->cst, &gr);
    hipGraphExec_t ex = nullptr;
    if (rc == KMP_OK && e == hipSuccess && gr && gen == g_grow_gen.load()) e = hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0);
    else if (e == hipSuccess) e = hipErrorUnknown;
    if (gr) (void)hipGraphDestroy(gr);
    if (e != hipSuccess || !ex) {  // not capturable this time: plain
        (void)hipGetLastError();
        return enqueue(st);
    }
    slot.gexec = ex;
    slot.key = key;
    PG(hipGraphLaunch(slot.gexec, st));
    return KMP_OK;
}

template <class MakeKeys>
int fused_launch(kmp_postings* ws, MakeKeys& make_keys, const std::vector<unsigned long long>& key, const StepCfg& c,
                 const PtGeom& g, hipStream_t st) {
    auto enqueue = [&](hipStream_t s) {
        int rc = enqueue_front(ws, make_keys, c, true, s);
        if (rc == KMP_OK) {
            ws->mark(3, s);
            rc = enqueue_tail(ws, c, g, s);
        }
        return rc;
    };
    if (!ws->graph_on) return enqueue(st);
    if (ws->gexec && ws->gkey == key) {
        PG(hipGraphLaunch(ws->gexec, st));
        ++ws->graph_replays;
        return KMP_OK;
    }
    if (ws->gkey_seen != key) {
        ws->gkey_seen = key;
        return enqueue(st);
    }
    if (ws->gexec) {
        (void)hipGraphExecDestroy(ws->gexec);
        ws->gexec = nullptr;
        ws->gkey.clear();
    }
    const unsigned long long gen = g_grow_gen.load();
    hipGraph_t gr = nullptr;
    // captured on a private stream (the caller's may be the legacy null stream, which cannot be
    // captured), launched on the caller's
    if (!ws->cst && hipStreamCreateWithFlags(&ws->cst, hipStreamNonBlocking) != hipSuccess) ws->cst = nullptr;
    if (!ws->cst || hipStreamBeginCapture(ws->cst, hipStreamCaptureModeRelaxed) != hipSuccess) {
        (void)hipGetLastError();
        ws->graph_on = false;
        return enqueue(st);
    }
    int rc = enqueue(ws->cst);
    hipError_t e = hipStreamEndCapture(ws->cst, &gr);
    hipGraphExec_t ex = nullptr;
    if (rc == KMP_OK && e == hipSuccess && gr && gen == g_grow_gen.load())
        e = hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0);
    else if (e == hipSuccess)
        e = hipErrorUnknown;
    if (gr) (void)hipGraphDestroy(gr);
    if (e != hipSuccess || !ex) {  // capture not usable: plain from now on
        (void)hipGetLastError();
        if (getenv("KMP_DEBUG"))
            fprintf(stderr, "kmp: step graph capture failed (rc %d, %s); plain launches from now on\n", rc,
                    hipGetErrorString(e));
        ws->graph_on = false;
        return enqueue(st);
    }
    ws->gexec = ex;
    ws->gkey = key;
    PG(hipGraphLaunch(ws->gexec, st));
    return KMP_OK;
}

void sum_stats(const unsigned long long* rb, unsigned long long* acc, unsigned long long* most,
               unsigned long long* n_inc, unsigned long long* spill_most, unsigned long long* spill_total) {
    for (int t = 0; t < kStN; ++t) acc[t] = 0;
    *most = *n_inc = *spill_most = *spill_total = 0;
    for (int sh = 0; sh < kShards; ++sh) {
        for (int t = 0; t < kStN; ++t)
            acc[t] = t == kStMaxDf ? std::max(acc[t], rb[sh * 8 + t]) : acc[t] + rb[sh * 8 + t];
        *most = std::max(*most, rb[kRbCursor + sh]);
        *n_inc += rb[kRbCursor + sh];
        *spill_most = std::max(*spill_most, rb[kRbSpill + sh]);
        *spill_total += rb[kRbSpill + sh];
    }
}

// One call: the fused step, or the split step when the batch spills.  *fallback: a class id
// wider than the key's class field (the caller reruns on the flat layout).
template <class MakeKeys>
int run_step(kmp_postings* ws, MakeKeys& make_keys, std::vector<unsigned long long> key, const StepCfg& c,
             uint64_t* n_edges, bool* fallback, kmp_postings_stats* stats, hipStream_t st) {
    *fallback = false;
    const std::vector<unsigned long long> shape = {c.n, c.slots, (unsigned long long)c.lay.cbits, c.lay.bbits};
    if (ws->shape != shape) {  // a new batch: forget what the last one taught the row tail and level 2
        ws->shape = shape;
        ws->pt_inc = 0;
        ws->pt_rb_max = 16;
        ws->fast_tail = ws->fast_mode;
        ws->large_grid = kBucketLargeGrid;
        ws->vreg_on = false;
        ws->vreg_tries = 0;
        ws->bp_J_min = 0;
        ws->heavy = false;
        ws->cur_on = ws->cur_mode;
    }
    if (ws->shard_cap == 0) ws->shard_cap = c.slots / 4 / kShards + 4096;
    if (ws->spill_cap == 0) ws->spill_cap = 1024;
    const bool debug = getenv("KMP_DEBUG") != nullptr;
    // a front whose spill holds every bucket (spill-all passes) and one holding the frequent k-mers
    // only are not interchangeable: a whole-batch call between passes of the same batch recomputes
    const bool want_all = c.ranged && ws->reuse && ws->flat_heavy && ws->spill_all_on;
    const bool reuse = ws->reuse && ws->front_ok && c.front_key && *c.front_key == ws->front_key &&
                       ws->front_all == want_all;
    if (!reuse) ws->front_ok = false;
    // every rerun grows a capacity to its measured need, so a handful of attempts suffices
    for (int attempt = 0; attempt < 16; ++attempt) {
        PtGeom g;
        if (!pt_geometry(ws, c, ws->pt_inc ? ws->pt_inc : c.slots / 4, &g)) return KMP_EINVAL;
        {
            int rc = step_reserve(ws, c, g, st);
            if (rc != KMP_OK) return rc;
        }
        const unsigned long long* rb = ws->hrb;
        unsigned long long acc[kStN], most, n_inc, spill_most, spill_total;
        const bool split = ws->heavy || reuse || c.expand_only;
        if (!reuse) ws->heavy_ready = ws->hcur_valid = false;  // a recomputed front: no compacted spill yet
        if (!split) {
            key.push_back(ws->shard_cap);
            key.push_back(ws->spill_cap);
            key.push_back(ws->timing);
            key.push_back(g.rbits + 1);
            key.push_back(g_grow_gen.load());
            key.push_back(ws->cur_on);
            key.push_back(ws->fast_tail);
            key.push_back(ws->large_grid);
            key.push_back(ws->vreg_on ? ws->vreg_total + 1 : 0);
            int rc = fused_launch(ws, make_keys, key, c, g, st);
            key.resize(key.size() - 9);
            if (rc != KMP_OK) return rc;
            PG(hipStreamSynchronize(st));
        } else {
            int rc = enqueue_front(ws, make_keys, c, !ws->heavy_ready, st, !reuse);
            if (rc != KMP_OK) return rc;
            step_pack_kernel<<<1, 256, 0, st>>>(ws->bstats.p, ws->flags.p, nullptr, ws->hrb);
            PG(hipStreamSynchronize(st));
        }
        if (rb[kRbFlagClass]) {
            *fallback = true;
            return KMP_OK;
        }
        sum_stats(rb, acc, &most, &n_inc, &spill_most, &spill_total);
        bool rerun = false;
        if (rb[kRbList] && ws->large_used == 0) {  // listed buckets, no large-bucket launch: again with it
            ws->large_grid = kBucketLargeGrid;
            rerun = true;
        }
        if (rb[kRbFlagCur] && ws->cur_used) {  // a region of the cursor partition overflowed
            // learn the layout from this call's exact bucket counts (own bins: all of them here);
            // the counting partition only if the learned layout keeps overflowing
            const uint32_t nb = 1u << c.lay.bbits;
            bool learned = false;
            if (ws->vreg_tries < kVregTries && ws->vreg.reserve(nb + 1) == hipSuccess) {
                vreg_kernel<<<1, 1024, 0, st>>>(ws->cur.p, nb, ws->vreg.p);
                uint32_t tot = 0;
                if (hipMemcpyAsync(&tot, ws->vreg.p + nb, 4, hipMemcpyDeviceToHost, st) == hipSuccess &&
                    hipStreamSynchronize(st) == hipSuccess && (uint64_t)tot + 2 * kBpTile < (1ull << 32)) {
                    ws->vreg_total = tot;
                    ws->vreg_on = learned = true;
                    ++ws->vreg_tries;
                }
            }
            if (!learned) {
                ws->vreg_on = false;
                ws->cur_on = false;
            }
            rerun = true;
        }
        if (rb[kRbFlagBin]) {  // a coarse bin above its level-2 tile budget
            ws->bp_J_min = (uint32_t)rb[kRbBinTiles] + 2;
            rerun = true;
        }
        if (spill_most > ws->spill_cap) {
            ws->spill_cap = spill_most + spill_most / 8 + 1024;
            rerun = true;
        }
        if (spill_total && !split) {  // frequent k-mers: the split step from now on
            ws->heavy = true;
            rerun = true;
        }
        if (!split && most > ws->shard_cap) {
            ws->shard_cap = most + most / 64 + 256;
            rerun = true;
        }
        if (rerun) {
            if (debug)
                fprintf(stderr, "kmp: rerun (bin %llu tiles %llu, spill %llu/%llu, heavy %d, shard %llu/%llu)\n",
                        rb[kRbFlagBin], rb[kRbBinTiles], spill_most, (unsigned long long)ws->spill_cap,
                        (int)ws->heavy, most, (unsigned long long)ws->shard_cap);
            continue;
        }
        if (split) {
            if (spill_total || ws->heavy_ready) {
                if (spill_total) {  // a new spill (a reused front spills nothing: keep its segments)
                    ws->h_segs = rb[kRbSegs];
                    ws->h_segmax = rb[kRbSegMax];
                }
                int rc = heavy_phase(ws, c, spill_total ? spill_total : ws->h_m, true, st);
                if (rc != KMP_OK) return rc;
            }
            ws->mark(3, st);
            step_pack_kernel<<<1, 256, 0, st>>>(ws->bstats.p, ws->flags.p, nullptr, ws->hrb);
            PG(hipStreamSynchronize(st));
            sum_stats(rb, acc, &most, &n_inc, &spill_most, &spill_total);
            if (most > ws->shard_cap) {
                if (debug)
                    fprintf(stderr, "kmp: rerun after the heavy path (shard %llu/%llu, segments %llu, largest %llu)\n",
                            most, (unsigned long long)ws->shard_cap, (unsigned long long)ws->h_segs,
                            (unsigned long long)ws->h_segmax);
                // an eighth of slack: the heavy path's region loads vary by a few percent between
                // calls, and with 1/64 uniprot k = 5 reran its front on most steps
                ws->shard_cap = most + most / 8 + 256;
                continue;
            }
            ws->pt_inc = n_inc;
            if (c.expand_only) {  // the shard regions stay for the fused tail (shard_cap unchanged)
                ws->last_most = most;
                fill_stats(stats, acc);
                if (stats) stats->incidences = n_inc;
                ws->last_heavy = ws->heavy_ready;
                ws->last_fused = false;
                if (c.front_key) {
                    ws->front_ok = true;
                    ws->front_key = *c.front_key;
                }
                *c.n_inc_out = n_inc;
                *n_edges = 0;
                return KMP_OK;
            }
            if (!pt_geometry(ws, c, n_inc, &g)) return KMP_EINVAL;
            int rc = step_reserve(ws, c, g, st);
            if (rc != KMP_OK) return rc;
            rc = enqueue_tail(ws, c, g, st);
            if (rc != KMP_OK) return rc;
            PG(hipStreamSynchronize(st));
        }
        if (rb[kRbFast]) {  // a fast-tail row-block region overflowed: the counting tail for this shape
            if (debug) fprintf(stderr, "kmp: fast tail region overflow (rows per block %u): counting tail\n", 1u << g.rbits);
            ws->fast_tail = false;
            continue;
        }
        ws->pt_inc = n_inc;  // sizes the next call's row blocks
        ws->last_fast = pt_fast(ws, g);
        ws->vreg_tries = 0;  // a call without a region overflow
        {  // the large-bucket grid of the next call: twice the listed buckets, 64 .. kBucketLargeGrid;
           // none listed: not launched (an idle 64-workgroup launch cost ~5 us of the config-3 step)
            uint32_t lg = rb[kRbList] ? 64u : 0u;
            while (lg && lg < kBucketLargeGrid && lg < 2 * rb[kRbList]) lg *= 2;
            ws->large_grid = lg;
        }
        uint64_t ne = rb[kRbRuns];
        ws->last_ovf = (uint32_t)rb[kRbOvf];
        if (rb[kRbOvf] && !pt_rowhist_ok(g)) {
            // row blocks above the LDS capacity: finished by the segmented sort; the next call
            // uses fewer rows per block when one row is not already the whole block
            if (g.rbits > 0) {
                const double over = (double)rb[kRbMaxBlock] / (0.8 * kPtCap);
                unsigned shrink = 1;
                while (shrink < 16 && (double)(1u << shrink) < over) ++shrink;
                ws->pt_rb_max = g.rbits > shrink ? g.rbits - shrink : 0u;
            }
            int rc = pt_finish_overflow(ws, c, g, (uint32_t)rb[kRbOvf], &ne, st);
            if (rc != KMP_OK) return rc;
            if (debug)
                fprintf(stderr, "kmp: %llu row blocks above %u keys (largest %llu) sorted apart; rbits bound %u\n",
                        rb[kRbOvf], kPtCap, rb[kRbMaxBlock], ws->pt_rb_max);
        }
        ws->shard_cap = most + most / 64 + 256;  // learned for the next call (after the last use of this one)
        fill_stats(stats, acc);
        if (stats) {
            stats->incidences = n_inc;
            stats->pairs = ne;
        }
        ws->last_heavy = ws->heavy_ready;
        ws->last_fused = !split;
        if (c.front_key) {
            ws->front_ok = true;
            ws->front_key = *c.front_key;
        }
        if (!reuse && ws->heavy && !spill_total) ws->heavy = false;  // nothing spilled: the fused step next
        *n_edges = ne;
        return ne > c.cap ? KMP_EOVERFLOW : KMP_OK;
    }
    return KMP_EDEVICE;
}

// The fused multi-k tail (kmp_dev_pairs_rows_multi): the pair keys that every workspace's
// expand-only call left in its shard regions (k bit and self-score in the field below the pair)
// reduced together by the row-block tail of ws[0]: one run per pair over both k, w = its length,
// w1 = its k-bit entries, score = Σ s — the union of the per-k lists without building or merging
// them.  Host-synchronous; *n_edges = the kept pairs.
// the in-place reduce of tail_multi's nd sub-blocks (keys in k2 / inc, descriptors in dsc): the
// count launches and the scan (*ne = the pass's edges; one read-back), then (tail_direct_write)
// the writes into the call's arrays — only the first c.cap edges
int tail_direct_count(kmp_postings* w0, const PtGeom& g, uint32_t nd, uint64_t* ne, hipStream_t st) {
    uint32_t *dstart = w0->dsc.p, *dsize = dstart + nd, *drow = dsize + nd;
    const BlkSrc bs{dstart, dsize, drow, reinterpret_cast<const uint32_t*>(w0->inc.p)};
    // dsc's run counts | offsets regions (the staged path's): the kept counts | the list of the
    // oversized sub-blocks (pt_split); the offsets in doff, the statistics in dlb
    uint32_t *wc = drow + nd, *ovl = wc + nd + 1;
    PG(w0->doff.reserve((uint64_t)nd + 1));
    PG(w0->dlb.reserve(2));
    PG(hipMemsetAsync(wc + nd, 0, sizeof(uint32_t), st));
    PG(hipMemsetAsync(w0->dlb.p, 0, sizeof(unsigned long long), st));
    constexpr uint32_t kWcGrid = 1024;
    if (g.kbit) {
        pt_window_count_kernel<true><<<kWcGrid, kPtRThreads, 0, st>>>(w0->k2.p, bs, g, ovl, wc);
        pt_reduce_count_kernel<true><<<nd, kPtRThreads, 0, st>>>(w0->k2.p, bs, g, wc, w0->dlb.p);
    } else {
        pt_window_count_kernel<false><<<kWcGrid, kPtRThreads, 0, st>>>(w0->k2.p, bs, g, ovl, wc);
        pt_reduce_count_kernel<false><<<nd, kPtRThreads, 0, st>>>(w0->k2.p, bs, g, wc, w0->dlb.p);
    }
    PG(hipGetLastError());
    size_t tb = 0;
    PG(rocprim::exclusive_scan(nullptr, tb, wc, w0->doff.p, 0u, (size_t)nd + 1, rocprim::plus<uint32_t>(), st));
    PG(w0->tmp.reserve(std::max(tb, w0->tmp.n)));
    PG(rocprim::exclusive_scan(w0->tmp.p, tb, wc, w0->doff.p, 0u, (size_t)nd + 1, rocprim::plus<uint32_t>(), st));
    uint32_t h_ne = 0;
    unsigned long long h_win = 0;
    PG(hipMemcpyAsync(&h_ne, w0->doff.p + nd, sizeof(h_ne), hipMemcpyDeviceToHost, st));
    PG(hipMemcpyAsync(&h_win, w0->dlb.p, sizeof(h_win), hipMemcpyDeviceToHost, st));
    PG(hipStreamSynchronize(st));
    *ne = h_ne;
    w0->last_ovf = (uint32_t)h_win;
    return KMP_OK;
}

int tail_direct_write(kmp_postings* w0, const StepCfg& c, const PtGeom& g, uint32_t nd, hipStream_t st) {
    uint32_t *dstart = w0->dsc.p, *dsize = dstart + nd, *drow = dsize + nd;
    const BlkSrc bs{dstart, dsize, drow, reinterpret_cast<const uint32_t*>(w0->inc.p)};
    const PtDirectOut out{c.d_p, c.d_q, c.d_w, c.d_s, c.d_w0, c.d_w1, c.cap, c.stride};
    if (g.kbit)
        pt_reduce_write_kernel<true><<<nd, kPtRThreads, 0, st>>>(w0->k2.p, bs, g, out, w0->doff.p);
    else
        pt_reduce_write_kernel<false><<<nd, kPtRThreads, 0, st>>>(w0->k2.p, bs, g, out, w0->doff.p);
    PG(hipGetLastError());
    return KMP_OK;
}

int tail_multi(kmp_postings* const* ws, uint32_t nk, const StepCfg& c, const uint64_t* inc, uint64_t* n_edges,
               kmp_postings_stats* stats, hipStream_t st) {
    kmp_postings* w0 = ws[0];
    uint64_t T = 0;
    for (uint32_t j = 0; j < nk; ++j) T += inc[j];
    PtGeom g;
    if (!pt_geometry(w0, c, std::max<uint64_t>(T, 1), &g)) return KMP_EINVAL;
    // staging capacity: every key of the pass (the row-block positions); a stream's planned pass
    // size at least, so the staging arrays are allocated once, not regrown as the passes vary
    uint64_t total = T + 1;
    for (uint32_t j = 0; j < nk; ++j) total = std::max<uint64_t>(total, ws[j]->stage_floor);
    PG(w0->inc.reserve(total / 2 + 1));  // u32 keys in a u64 buffer
    const bool direct = w0->direct_tail != 0;
    if (!direct) {  // staged runs (the direct reduce writes the edges in place)
        PG(w0->uniq.reserve(total));
        PG(w0->w.reserve(total));
        PG(w0->stg2.reserve(2 * total));
    }
    PG(w0->ovf.reserve((uint64_t)g.nrb + 1));
    PG(w0->small.reserve(16));
    hipError_t e = hipSuccess;
    const PtBufs b = pt_bufs(w0, g, true, &e, st);
    PG(e);
    PG(hipMemsetAsync(w0->flags.p + kFlOvf, 0, sizeof(uint32_t), st));
    uint32_t* keys32 = reinterpret_cast<uint32_t*>(w0->inc.p);
    uint32_t* stage_p = reinterpret_cast<uint32_t*>(w0->uniq.p);
    uint32_t* stage_q = stage_p + total;
    auto geo = [&](uint32_t j) {  // input j: its shard regions
        PtGeom gj = g;
        gj.sc = ws[j]->shard_cap;
        gj.jt = (uint32_t)((gj.sc + kPtTile - 1) / kPtTile);
        return gj;
    };
    for (uint32_t j = 0; j < nk; ++j)
        pt_hist_kernel<<<dim3(geo(j).jt, kShards), kPtThreads, 0, st>>>(ws[j]->inc_sorted.p, ws[j]->bstats.p + kRbCursor,
                                                                       geo(j), b.T);
    pt_tscan_kernel<<<1, kPtScanThreads, 0, st>>>(b.T, g.nrb, b.bst, b.cur, w0->small.p + 2);
    for (uint32_t j = 0; j < nk; ++j)
        pt_scatter_kernel<<<dim3(geo(j).jt, kShards), kPtThreads, 0, st>>>(ws[j]->inc_sorted.p,
                                                                          ws[j]->bstats.p + kRbCursor, geo(j), b.cur,
                                                                          keys32);
    // the row blocks' sizes -> sub-blocks (a block above kPtCap cut into pieces the LDS reduce takes)
    std::vector<uint32_t> hb(g.nrb + 1), hd(g.nrb + 1);
    PG(hipMemcpyAsync(hb.data(), b.bst, (g.nrb + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    PG(hipStreamSynchronize(st));
    uint32_t nd = 0;
    for (uint32_t r = 0; r < g.nrb; ++r) {
        hd[r] = nd;
        nd += pt_sub_slots(hb[r + 1] - hb[r]);
    }
    hd[g.nrb] = nd;
    PG(w0->k2.reserve(total));
    PG(w0->dsc.reserve(5 * (uint64_t)nd + 2 + g.nrb + 1));
    // dstart | dsize | drow (nd each) | run counts (nd + 1: the scan's last input is 0) | edge offsets
    // (nd + 1) | dbase (nrb + 1)
    uint32_t *dstart = w0->dsc.p, *dsize = dstart + nd, *drow = dsize + nd, *dcnt = drow + nd, *deoff = dcnt + nd + 1,
             *dbase = deoff + nd + 1;
    PG(w0->ovf.reserve((uint64_t)std::max(nd, g.nrb) + 1));  // the sub-blocks the reduce lists
    PG(hipMemcpyAsync(dbase, hd.data(), (g.nrb + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, st));
    PG(hipMemsetAsync(deoff, 0, sizeof(uint32_t), st));  // the oversized sub-blocks' list count
    pt_split_kernel<<<g.nrb, kSbThreads, 0, st>>>(keys32, b.bst, dbase, g, c.n, c.ranged ? c.row_hi : c.n,
                                                  w0->k2.p, dstart, dsize, drow, deoff);
    const BlkSrc bs{dstart, dsize, drow, keys32};
    if (direct) {
        w0->pend_g = g;
        w0->pend_nd = nd;
        w0->pend_direct = true;
        w0->last_ovf = 0;
        uint64_t ne = 0;
        int rc = tail_direct_count(w0, g, nd, &ne, st);
        if (rc == KMP_OK && ne <= c.cap) rc = tail_direct_write(w0, c, g, nd, st);
        if (rc != KMP_OK) return rc;
        for (uint32_t j = 0; j < nk; ++j) ws[j]->shard_cap = ws[j]->last_most + ws[j]->last_most / 4 + 256;
        w0->pt_inc = T;
        w0->pend_ne = ne;
        if (stats) {
            stats->incidences = T;
            stats->pairs = ne;
        }
        *n_edges = ne;
        return ne > c.cap ? KMP_EOVERFLOW : KMP_OK;
    }
    w0->pend_direct = false;
    if (g.kbit)
        pt_reduce_scored_kernel<true><<<nd, kPtRThreads, 0, st>>>(w0->k2.p, bs, g, w0->flags.p, w0->ovf.p, stage_p,
                                                                  stage_q, w0->w.p, w0->stg2.p, w0->stg2.p + total,
                                                                  dcnt);
    else
        pt_reduce_scored_kernel<false><<<nd, kPtRThreads, 0, st>>>(w0->k2.p, bs, g, w0->flags.p, w0->ovf.p, stage_p,
                                                                   stage_q, w0->w.p, w0->stg2.p, nullptr, dcnt);
    PG(hipGetLastError());
    uint32_t h_ovf = 0;
    PG(hipMemcpyAsync(&h_ovf, w0->flags.p + kFlOvf, 4, hipMemcpyDeviceToHost, st));
    PG(hipStreamSynchronize(st));
    w0->last_ovf = h_ovf;
    if (h_ovf) {  // sub-blocks still above kPtCap: the tagged sort (their counts land in dcnt)
        uint64_t unused = 0;
        int rc = pt_finish_overflow(w0, c, g, h_ovf, &unused, st, total, &bs, nd, dcnt, deoff, w0->k2.p);
        if (rc != KMP_OK) return rc;
    }
    // edge offsets of the sub-blocks (canonical: row blocks in order, sub-blocks by key range)
    size_t tscan = 0;
    PG(rocprim::exclusive_scan(nullptr, tscan, dcnt, deoff, 0u, (size_t)nd + 1, rocprim::plus<uint32_t>(), st));
    PG(w0->tmp.reserve(std::max(tscan, w0->tmp.n)));
    PG(hipMemsetAsync(dcnt + nd, 0, sizeof(uint32_t), st));
    PG(rocprim::exclusive_scan(w0->tmp.p, tscan, dcnt, deoff, 0u, (size_t)nd + 1, rocprim::plus<uint32_t>(), st));
    uint32_t h_ne = 0;
    PG(hipMemcpyAsync(&h_ne, deoff + nd, 4, hipMemcpyDeviceToHost, st));
    PG(hipStreamSynchronize(st));
    uint64_t ne = h_ne;
    // the staged runs stay in w0: a caller that finds its arrays too small (KMP_EOVERFLOW) grows them
    // and calls again with the same rows, and only the emit runs (tail_multi_emit)
    w0->pend_nd = nd;
    w0->pend_total = total;
    w0->pend_ne = ne;
    if (ne <= c.cap) {
        pt_emit_kernel<<<nd, 256, 0, st>>>(stage_p, stage_q, w0->w.p, dstart, dcnt, deoff, c.d_p, c.d_q, c.d_w, c.cap,
                                           c.stride, PtPack{}, nullptr, pt_score_out(w0, c, total));
        PG(hipGetLastError());
    }
    // the next call's regions, learned now that the tail has read them; a quarter of slack (the
    // passes' sizes and shard loads vary, and an overflow reruns the whole expansion)
    for (uint32_t j = 0; j < nk; ++j) ws[j]->shard_cap = ws[j]->last_most + ws[j]->last_most / 4 + 256;
    w0->pt_inc = T;
    if (stats) {
        stats->incidences = T;
        stats->pairs = ne;
    }
    *n_edges = ne;
    return ne > c.cap ? KMP_EOVERFLOW : KMP_OK;
}

// the emit of the last tail_multi of w0 again, into larger arrays (its runs are still staged)
int tail_multi_emit(kmp_postings* w0, const StepCfg& c, uint64_t* n_edges, hipStream_t st) {
    const uint32_t nd = w0->pend_nd;
    if (w0->pend_direct) {  // the in-place reduce again, into the larger arrays
        *n_edges = w0->pend_ne;
        if (w0->pend_ne > c.cap) return KMP_EOVERFLOW;
        return tail_direct_write(w0, c, w0->pend_g, nd, st);  // the keys stay sorted in place
    }
    const uint64_t total = w0->pend_total;
    uint32_t *dstart = w0->dsc.p, *dsize = dstart + nd, *drow = dsize + nd, *dcnt = drow + nd, *deoff = dcnt + nd + 1;
    (void)drow;
    uint32_t* stage_p = reinterpret_cast<uint32_t*>(w0->uniq.p);
    *n_edges = w0->pend_ne;
    if (w0->pend_ne > c.cap) return KMP_EOVERFLOW;
    pt_emit_kernel<<<nd, 256, 0, st>>>(stage_p, stage_p + total, w0->w.p, dstart, dcnt, deoff, c.d_p, c.d_q, c.d_w,
                                       c.cap, c.stride, PtPack{}, nullptr, pt_score_out(w0, c, total));
    PG(hipGetLastError());
    return KMP_OK;
}

// Shared tail: sort the pair keys, run-length encode -> (pair, w) in canonical order, keep
// w >= min_shared, unpack.  Marks 5 (pair sort) and 6 (encode + emit).
int tail(kmp_postings* ws, const unsigned long long* in, unsigned long long n_inc, uint32_t n, uint32_t min_shared,
         uint32_t* d_p, uint32_t* d_q,
         uint32_t* d_w, uint64_t cap, uint64_t* n_edges, kmp_postings_stats* stats, hipStream_t st) {
    if (stats) stats->incidences = n_inc;
    if (n_inc == 0) {
        ws->mark(5, st);
        ws->mark(6, st);
        return KMP_OK;
    }
    if (n_inc > 0xFFFFFFFFull) return KMP_ENOMEM;  // run-length counts are u32
    const unsigned pair_bits = bits_for((uint64_t)n * n);
    PG(ws->inc_sorted.reserve(n_inc));
    PG(ws->uniq.reserve(n_inc));
    PG(ws->w.reserve(n_inc));
    PG(ws->small.reserve(16));
    const bool filter_w = min_shared > 1;
    if (filter_w) {
        PG(ws->keep.reserve(n_inc));
        PG(ws->pos.reserve(n_inc));
    }
    size_t t2 = 0, t3 = 0, t4 = 0;
    PG(rocprim::radix_sort_keys<PairSortCfg>(nullptr, t2, in, ws->inc_sorted.p, (size_t)n_inc, 0u, pair_bits, st));
    PG(rocprim::run_length_encode(nullptr, t3, ws->inc_sorted.p, (unsigned int)n_inc, ws->uniq.p, ws->w.p,
                                  ws->small.p + 1, st));
    if (filter_w)
        PG(rocprim::exclusive_scan(nullptr, t4, ws->keep.p, ws->pos.p, 0u, (size_t)n_inc, rocprim::plus<uint32_t>(),
                                   st));
    PG(ws->tmp.reserve(std::max({t2, t3, t4, ws->tmp.n})));
    PG(rocprim::radix_sort_keys<PairSortCfg>(ws->tmp.p, t2, in, ws->inc_sorted.p, (size_t)n_inc, 0u, pair_bits, st));
    ws->mark(5, st);
    PG(rocprim::run_length_encode(ws->tmp.p, t3, ws->inc_sorted.p, (unsigned int)n_inc, ws->uniq.p, ws->w.p,
                                  ws->small.p + 1, st));
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
    (void)hipGetLastError();  // a stage the call did not run (never recorded) must not poison the next launch check
}

int postings_args(kmp_postings* ws, int k, uint64_t* n_edges, kmp_postings_stats* stats, uint32_t* d_p,
                  uint32_t* d_q, uint32_t* d_w, uint64_t cap) {
    if (!ws || !n_edges || k < 1 || k > kMaxK) return KMP_EINVAL;
    *n_edges = 0;
    if (stats) *stats = kmp_postings_stats{};
    if (cap && (!d_p || !d_q || !d_w)) return KMP_EINVAL;
    return KMP_OK;
}

// keys of proteins [p_lo, p_hi) into ws->keys (slots [slot_begin, slot_end) of the batch layout)
hipError_t launch_residue_keys(kmp_postings* ws, const uint8_t* d_res, const uint64_t* d_res_off,
                               const uint16_t* d_class, int k, uint32_t p_lo, uint32_t p_hi, uint64_t slot_begin,
                               uint64_t slot_end, const Layout& lay, hipStream_t st) {
    const uint32_t g = (uint32_t)((slot_end - slot_begin + kKeyChunk - 1) / kKeyChunk);
    hipError_t e = ws->chunk_first.reserve(g + 1);
    if (e != hipSuccess) return e;
    chunk_first_kernel<<<(p_hi - p_lo + 1 + 255) / 256, 256, 0, st>>>(d_res_off, p_lo, p_hi, slot_begin, slot_end, g,
                                                                      ws->chunk_first.p);
    residue_keys_chunk_kernel<<<g, kKeyThreads, 0, st>>>(d_res, d_res_off, d_class, k, p_hi, slot_begin, slot_end,
                                                          ws->chunk_first.p, lay, ws->keys.p, ws->flags.p);
    return hipGetLastError();
}

// Both entry points: keys from `make_keys(layout)`, the bucketed step (flat on fallback).
template <class MakeKeys>
int run_postings(kmp_postings* ws, MakeKeys make_keys, const std::vector<unsigned long long>& key_extra, uint32_t n,
                 int k, uint64_t slots, const uint16_t* d_class, uint32_t heavy_df, uint32_t min_shared,
                 int require_class_diff, bool ranged, uint32_t row_lo, uint32_t row_hi, uint32_t* d_p, uint32_t* d_q,
                 uint32_t* d_w, uint64_t cap, uint64_t* n_edges, kmp_postings_stats* stats, hipStream_t st,
                 unsigned sb = 0, uint32_t sor = 0, uint32_t* d_s = nullptr, uint32_t* d_w1 = nullptr,
                 uint64_t* n_inc_out = nullptr) {
    if (heavy_df < 2) heavy_df = 2;
    if (min_shared < 1) min_shared = 1;
    ws->bin_lo = ws->bin_hi = 0;  // every bucket (the k-mer split restricts its own calls)
    PG(ws->keys.reserve(slots));
    PG(ws->sorted.reserve(slots));
    PG(ws->flags.reserve(kFlN));
    ws->parted = false;
    Layout lay = make_layout(n, k, slots, ws->bucketed);
    std::vector<unsigned long long> front_key = {n, (unsigned long long)k, slots, heavy_df,
                                                 (unsigned long long)require_class_diff};
    front_key.insert(front_key.end(), key_extra.begin(), key_extra.end());
    if (lay.bucketed) {
        StepCfg c{};
        c.slots = slots;
        c.lay = lay;
        c.n = n;
        c.heavy_df = heavy_df;
        c.min_shared = min_shared;
        c.require_diff = require_class_diff;
        c.ranged = ranged;
        c.row_lo = row_lo;
        c.row_hi = row_hi;
        c.d_p = d_p;
        c.d_q = d_q;
        c.d_w = d_w;
        c.cap = cap;
        c.stride = 1;
        c.front_key = &front_key;
        c.k = k;
        c.sb = sb;
        c.sor = sor;
        c.d_s = d_s;
        c.d_w1 = d_w1;
        c.expand_only = n_inc_out != nullptr;
        c.n_inc_out = n_inc_out;
        // graph key: the call's shape and pointers (run_step adds the capacities, the timing
        // switch, the row-block geometry and the buffer generation)
        std::vector<unsigned long long> key = {n, (unsigned long long)k, slots, heavy_df, min_shared,
                                               (unsigned long long)require_class_diff, ranged, row_lo, row_hi, cap,
                                               (unsigned long long)(uintptr_t)d_p, (unsigned long long)(uintptr_t)d_q,
                                               (unsigned long long)(uintptr_t)d_w, sb, sor,
                                               (unsigned long long)(uintptr_t)d_s, (unsigned long long)(uintptr_t)d_w1};
        key.insert(key.end(), key_extra.begin(), key_extra.end());
        bool fallback = false;
        int rc = run_step(ws, make_keys, key, c, n_edges, &fallback, stats, st);
        if (!fallback) {
            ws->last_bucketed = true;
            if (rc == KMP_OK) finish_timing(ws, stats, st);
            return rc;
        }
    }
    // flat layout: class ids wider than the bucketed key's class field (or the layout forced)
    ws->front_ok = false;
    if (ranged || sb || n_inc_out) return KMP_ESTATE;  // no row filter, scores or fused tail on the flat layout
    lay = make_layout(n, k, slots, false);
    if (lay.sort_hi > 64) return KMP_EINVAL;
    ws->parted = false;
    PG(hipMemsetAsync(ws->flags.p, 0, kFlN * sizeof(uint32_t), st));
    ws->mark(0, st);
    PG(make_keys(lay, st));
    ws->mark(1, st);
    unsigned long long n_inc = 0;
    int rc = front_flat(ws, slots, lay, d_class, n, heavy_df, require_class_diff, &n_inc, stats, st);
    if (rc != KMP_OK) return rc;
    ws->last_bucketed = false;
    ws->last_fused = ws->last_heavy = false;
    ws->last_ovf = 0;
    rc = tail(ws, ws->inc.p, n_inc, n, min_shared, d_p, d_q, d_w, cap, n_edges, stats, st);
    if (rc == KMP_OK) finish_timing(ws, stats, st);
    return rc;
}

// ------------------------------------------------------------- multi-GPU k-mer split --------
// kmp_dev_split_expand / kmp_dev_split_edges (kmerpair.h): rank `part` of `parts` groups and
// expands only the k-mers of its coarse bins (a contiguous share of the bucket hash range; every
// rank computes the windows of the whole batch and keeps its share at level 1), routes the pair
// keys to the rank owning the row of their smaller protein, and that rank reduces them with the
// row-block tail.  A pair's incidences from every k-mer meet on its row owner, so w is complete
// there, and the ranks' row ranges are ordered: the rank-order concatenation is canonical.
constexpr uint32_t kRtThreads = 256, kRtPer = 16, kRtTile = kRtThreads * kRtPer;

// pair keys (p << pbits | q) of the shard regions -> region d (cap keys) of send, d = the rank
// owning row p; one reservation per destination per 4,096-key tile on dcursor[d]
__global__ __launch_bounds__(kRtThreads) void split_route_kernel(const unsigned long long* __restrict__ in,
                                                                 const unsigned long long* __restrict__ cursor,
                                                                 uint64_t sc, unsigned pbits, SplitRows rows,
                                                                 uint64_t cap, unsigned long long* __restrict__ send,
                                                                 unsigned long long* __restrict__ dcursor) {
    __shared__ uint32_t lcnt[kSplitMax];
    __shared__ unsigned long long base[kSplitMax];
    const uint32_t s = blockIdx.y;
    const uint64_t ns = min<unsigned long long>(cursor[s], sc), t0 = (uint64_t)blockIdx.x * kRtTile;
    if (t0 >= ns) return;
    const uint32_t m = (uint32_t)min<uint64_t>(kRtTile, ns - t0);
    const unsigned long long* src = in + s * sc + t0;
    if (threadIdx.x < kSplitMax) lcnt[threadIdx.x] = 0;
    __syncthreads();
    unsigned long long x[kRtPer];
    uint32_t dr[kRtPer];  // destination << 24 | rank in the tile's run
#pragma unroll
    for (uint32_t e = 0; e < kRtPer; ++e) {
        const uint32_t i = threadIdx.x + e * kRtThreads;
        x[e] = i < m ? src[i] : kNoKey;
    }
#pragma unroll
    for (uint32_t e = 0; e < kRtPer; ++e) {
        dr[e] = ~0u;
        if (x[e] == kNoKey) continue;
        const uint32_t p = (uint32_t)(x[e] >> pbits);
        uint32_t d = 0;
        while (d + 1 < rows.parts && p >= rows.start[d + 1]) ++d;
        dr[e] = d << 24 | atomicAdd(&lcnt[d], 1u);
    }
    __syncthreads();
    if (threadIdx.x < rows.parts)
        base[threadIdx.x] =
            lcnt[threadIdx.x] ? atomicAdd(&dcursor[threadIdx.x], (unsigned long long)lcnt[threadIdx.x]) : 0ull;
    __syncthreads();
#pragma unroll
    for (uint32_t e = 0; e < kRtPer; ++e) {
        if (dr[e] == ~0u) continue;
        const uint32_t d = dr[e] >> 24;
        const unsigned long long pos = base[d] + (dr[e] & 0xFFFFFFu);
        if (pos < cap) send[d * cap + pos] = x[e];
    }
}

// the unused tail of every send region -> kNoKey (the receiver's tail skips it); workgroup (0, 0)
// also writes the rank's flags (KMP_SPLIT_*) and statistics (kSt* order, summed over the shards)
// routed (the bucket kernels wrote the send regions themselves, kShards sub-regions of cap / kShards
// keys per destination, the buffer pre-filled with kNoKey): no padding; the part size reported is
// kShards x the fullest sub-region, so a grown cap gives every sub-region its need
__global__ void split_pad_finish_kernel(unsigned long long* __restrict__ send, uint64_t cap,
                                        const unsigned long long* __restrict__ dcursor,
                                        const unsigned long long* __restrict__ gstats,
                                        const uint32_t* __restrict__ wflags, uint64_t sc, uint32_t parts,
                                        uint32_t* __restrict__ out, unsigned long long* __restrict__ stats,
                                        int heavy_done, int routed) {
    const uint32_t d = blockIdx.y;
    if (!routed)
        for (uint64_t i = dcursor[d] + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap;
             i += (uint64_t)gridDim.x * blockDim.x)
            send[d * cap + i] = kNoKey;
    if (blockIdx.x || blockIdx.y) return;
    // one workgroup: the statistics and the fullest regions reduced over its threads (one thread
    // walking the parts x kShards cursors took 45 us at G = 8)
    const uint32_t t = threadIdx.x;
    __shared__ unsigned long long s_red[3][256 / 64];
    if (t < kStN) {
        unsigned long long v = 0;
        for (int sh = 0; sh < kShards; ++sh) {
            const unsigned long long x = gstats[sh * 8 + t];
            v = t == kStMaxDf ? max(v, x) : v + x;
        }
        stats[t] = v;
    }
    unsigned long long shard = 0, spill = 0, part = 0;
    for (uint32_t sh = t; sh < kShards; sh += blockDim.x) {
        shard = max(shard, gstats[kRbCursor + sh]);
        spill += gstats[kRbSpill + sh];
    }
    const uint32_t nq = routed ? parts * kShards : parts;
    for (uint32_t q = t; q < nq; q += blockDim.x) part = max(part, dcursor[q] * (routed ? kShards : 1u));
    for (int off = 32; off > 0; off >>= 1) {
        shard = max(shard, (unsigned long long)__shfl_xor(shard, off));
        spill += (unsigned long long)__shfl_xor(spill, off);
        part = max(part, (unsigned long long)__shfl_xor(part, off));
    }
    if ((t & 63) == 0) {
        s_red[0][t >> 6] = shard;
        s_red[1][t >> 6] = spill;
        s_red[2][t >> 6] = part;
    }
    __syncthreads();
    if (t == 0) {
        shard = spill = part = 0;
        for (uint32_t w = 0; w < (blockDim.x + 63) / 64; ++w) {
            shard = max(shard, s_red[0][w]);
            spill += s_red[1][w];
            part = max(part, s_red[2][w]);
        }
        const uint32_t clamp = 0xFFFFFFFFu;
        out[KMP_SPLIT_CLASS] = wflags[kFlClass];
        out[KMP_SPLIT_HEAVY] = spill != 0 && !heavy_done;  // spilled with the heavy path off: rerun with it on
        out[KMP_SPLIT_MAX_PART] = (uint32_t)min<unsigned long long>(part, clamp);
        out[KMP_SPLIT_MAX_SHARD] = (uint32_t)min<unsigned long long>(shard, clamp);
        out[KMP_SPLIT_BIN_TILES] = wflags[kFlBin] ? wflags[kFlBinTiles] : 0u;
        out[KMP_SPLIT_CURSOR] = wflags[kFlCur];
        out[KMP_SPLIT_RERUN] = (part > cap || shard > sc || wflags[kFlBin] || wflags[kFlCur]) ? 1u : 0u;
        for (uint32_t i = KMP_SPLIT_CURSOR + 1; i < KMP_SPLIT_FLAGS; ++i) out[i] = 0;
    }
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

int kmp_postings_set_layout(kmp_postings* ws, int bucketed) {
    if (!ws) return KMP_EINVAL;
    ws->bucketed = bucketed != 0;
    return KMP_OK;
}

int kmp_postings_last_layout(const kmp_postings* ws) {
    if (!ws || !ws->last_bucketed) return KMP_LAYOUT_FLAT;
    return ws->last_heavy ? KMP_LAYOUT_BUCKETED_HEAVY : KMP_LAYOUT_BUCKETED;
}

uint32_t kmp_postings_last_overflow_blocks(const kmp_postings* ws) { return ws ? ws->last_ovf : 0u; }

int kmp_postings_set_flat_heavy(kmp_postings* ws, int enable) {
    if (!ws) return KMP_EINVAL;
    ws->flat_heavy = enable ? 1 : 0;
    return KMP_OK;
}

int kmp_postings_set_direct(kmp_postings* ws, int enable) {
    if (!ws) return KMP_EINVAL;
    ws->direct_tail = enable ? 1 : 0;
    return KMP_OK;
}

int kmp_postings_set_tail(kmp_postings* ws, int mode) {
    if (!ws || (mode != KMP_TAIL_FAST && mode != KMP_TAIL_COUNT && mode != KMP_TAIL_DENSE)) return KMP_EINVAL;
    ws->fast_mode = mode != KMP_TAIL_COUNT;
    ws->dense_on = mode == KMP_TAIL_DENSE;
    ws->fast_tail = ws->fast_mode;
    return KMP_OK;
}

int kmp_postings_last_tail(const kmp_postings* ws) {
    if (!ws || !ws->last_bucketed) return -1;
    return ws->last_fast ? KMP_TAIL_FAST : KMP_TAIL_COUNT;
}

int kmp_postings_set_graph(kmp_postings* ws, int enable) {
    if (!ws) return KMP_EINVAL;
    ws->graph_on = enable != 0;
    if (!ws->graph_on && ws->gexec) {
        (void)hipGraphExecDestroy(ws->gexec);
        ws->gexec = nullptr;
        ws->gkey.clear();
    }
    if (!ws->graph_on)
        for (auto& g : ws->split_g) g.reset();
    ws->gkey_seen.clear();
    return KMP_OK;
}

uint64_t kmp_postings_graph_replays(const kmp_postings* ws) { return ws ? ws->graph_replays : 0; }

int kmp_postings_set_partition(kmp_postings* ws, int mode) {
    if (!ws || (mode != KMP_PARTITION_AUTO && mode != KMP_PARTITION_COUNT)) return KMP_EINVAL;
    ws->cur_mode = mode == KMP_PARTITION_AUTO;
    ws->cur_on = ws->cur_mode;
    ws->front_ok = false;
    return KMP_OK;
}

int kmp_postings_last_partition(const kmp_postings* ws) {
    if (!ws || !ws->last_bucketed) return -1;
    return ws->cur_used ? KMP_PARTITION_CURSOR : KMP_PARTITION_COUNT;
}

int kmp_postings_set_shard_floor(kmp_postings* ws, uint64_t keys) {
    if (!ws) return KMP_EINVAL;
    // the fullest region at up to twice the mean (measured 1.6x at config 5: frequent k-mers' tiles
    // land on few shards), a quarter of slack; the fused tail's staging for the pass + 15 %
    ws->shard_floor = keys ? 2 * keys / kShards + 2 * keys / kShards / 4 + 256 : 0;
    ws->stage_floor = keys + keys * 3 / 20;
    return KMP_OK;
}

int kmp_postings_set_reuse(kmp_postings* ws, int enable) {
    if (!ws) return KMP_EINVAL;
    ws->reuse = enable != 0;
    if (!ws->reuse) ws->front_ok = false;
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
    hipStream_t st = as_stream(stream);
    auto keys = [&](const Layout& lay, hipStream_t st) {
        ws->cur_used = false;  // keys grouped by the bucket sort
        set_keys_kernel<<<n + 1, 256, 0, st>>>(d_set, d_set_len, d_res_off, d_class, n, slots, lay, ws->keys.p,
                                               ws->flags.p);
        return hipGetLastError();
    };
    const std::vector<unsigned long long> key_extra = {0, (uintptr_t)d_set, (uintptr_t)d_set_len, (uintptr_t)d_res_off,
                                                       (uintptr_t)d_class};
    return run_postings(ws, keys, key_extra, n, k, slots, d_class, heavy_df, min_shared, require_class_diff, false, 0,
                        n, d_p, d_q, d_w, cap, n_edges, stats, st);
}

// the residue key paths take the step's clear into their first kernel, for the call that sets this
struct ClearInKeys {
    kmp_postings* ws;
    explicit ClearInKeys(kmp_postings* w) : ws(w) { ws->clear_in_keys = true; }
    ~ClearInKeys() {
        ws->clear_in_keys = false;
        ws->defer_clear = false;
    }
};

static int residues_impl(kmp_postings* ws, const uint8_t* d_res, const uint64_t* d_res_off, const uint16_t* d_class,
                         uint32_t n, int k, uint64_t slots, uint32_t heavy_df, uint32_t min_shared,
                         int require_class_diff, bool ranged, uint32_t row_lo, uint32_t row_hi, uint32_t* d_p,
                         uint32_t* d_q, uint32_t* d_w, uint64_t cap, uint64_t* n_edges, kmp_postings_stats* stats,
                         void* stream, unsigned sb = 0, uint32_t sor = 0, uint32_t* d_s = nullptr,
                         uint32_t* d_w1 = nullptr, uint64_t* n_inc_out = nullptr) {
    int rc = postings_args(ws, k, n_edges, stats, d_p, d_q, d_w, cap);
    if (rc != KMP_OK || n < 2) return rc;
    if (!d_res || !d_res_off || !d_class) return KMP_EINVAL;
    hipStream_t st = as_stream(stream);
    auto keys = [&](const Layout& lay, hipStream_t st) {
        if (lay.bucketed) {
            ws->parted = true;
            ws->cur_used = ws->cur_on && cur_geometry(lay, &ws->cg);
            ws->cg.vreg = ws->cur_used && ws->vreg_on ? ws->vreg.p : nullptr;
            return bp_level1(ws, d_res, d_res_off, d_class, k, n, slots, lay, st);
        }
        ws->cur_used = false;
        if (ws->defer_clear) {
            step_clear_kernel<<<1, 256, 0, st>>>(ws->flags.p, ws->bstats.p, ws->clear_extra, ws->clear_n);
            ws->defer_clear = false;
        }
        return launch_residue_keys(ws, d_res, d_res_off, d_class, k, 0u, n, 0ull, slots, lay, st);
    };
    const std::vector<unsigned long long> key_extra = {1, (uintptr_t)d_res, (uintptr_t)d_res_off, (uintptr_t)d_class};
    const ClearInKeys guard(ws);
    return run_postings(ws, keys, key_extra, n, k, slots, d_class, heavy_df, min_shared, require_class_diff, ranged,
                        row_lo, row_hi, d_p, d_q, d_w, cap, n_edges, stats, st, sb, sor, d_s, d_w1, n_inc_out);
}

int kmp_dev_pairs_residues(kmp_postings* ws, const uint8_t* d_res, const uint64_t* d_res_off,
                           const uint16_t* d_class, uint32_t n, int k, uint64_t slots, uint32_t heavy_df,
                           uint32_t min_shared, int require_class_diff, uint32_t* d_p, uint32_t* d_q, uint32_t* d_w,
                           uint64_t cap, uint64_t* n_edges, kmp_postings_stats* stats, void* stream) {
    return residues_impl(ws, d_res, d_res_off, d_class, n, k, slots, heavy_df, min_shared, require_class_diff, false,
                         0, n, d_p, d_q, d_w, cap, n_edges, stats, stream);
}

int kmp_dev_pairs_rows(kmp_postings* ws, const uint8_t* d_res, const uint64_t* d_res_off, const uint16_t* d_class,
                       uint32_t n, int k, uint64_t slots, uint32_t heavy_df, uint32_t min_shared,
                       int require_class_diff, uint32_t row_lo, uint32_t row_hi, uint32_t* d_p, uint32_t* d_q,
                       uint32_t* d_w, uint64_t cap, uint64_t* n_edges, kmp_postings_stats* stats, void* stream) {
    if (row_lo > row_hi || row_hi > n) return KMP_EINVAL;
    if (row_lo == row_hi) {
        int rc = postings_args(ws, k, n_edges, stats, d_p, d_q, d_w, cap);
        return rc;
    }
    return residues_impl(ws, d_res, d_res_off, d_class, n, k, slots, heavy_df, min_shared, require_class_diff, true,
                         row_lo, row_hi, d_p, d_q, d_w, cap, n_edges, stats, stream);
}

uint32_t kmp_dev_rows_max(uint32_t n, int scored) {
    // the row-block tail's u32 key (p_local << pbits | q, scored << kScoreBits more, multi-k one k
    // bit more, one padding bit) and its kPtMaxBlocks row blocks bound the rows of one call
    const unsigned used = bits_for(n) + (scored ? kScoreBits : 0u) + (scored > 1 ? 1u : 0u);
    if (used >= 31) return 0;
    const uint64_t m = (uint64_t)kPtMaxBlocks << (31 - used);
    return (uint32_t)std::min<uint64_t>(m, n);
}

int kmp_dev_pairs_rows_scored(kmp_postings* ws, const uint8_t* d_res, const uint64_t* d_res_off, const uint16_t* d_class,
                              uint32_t n, int k, uint64_t slots, uint32_t heavy_df, uint32_t min_shared,
                              int require_class_diff, uint32_t row_lo, uint32_t row_hi, uint32_t* d_p, uint32_t* d_q,
                              uint32_t* d_w, uint32_t* d_score, uint64_t cap, uint64_t* n_edges,
                              kmp_postings_stats* stats, void* stream) {
    if (row_lo > row_hi || row_hi > n) return KMP_EINVAL;
    if (cap && !d_score) return KMP_EINVAL;
    if (row_hi - row_lo > kmp_dev_rows_max(n, 1)) return KMP_EINVAL;
    if (row_lo == row_hi) return postings_args(ws, k, n_edges, stats, d_p, d_q, d_w, cap);
    const bool ranged = !(row_lo == 0 && row_hi == n);
    return residues_impl(ws, d_res, d_res_off, d_class, n, k, slots, heavy_df, min_shared, require_class_diff, ranged,
                         row_lo, row_hi, d_p, d_q, d_w, cap, n_edges, stats, stream, kScoreBits, 0u, d_score, nullptr);
}

int kmp_dev_pairs_rows_multi(kmp_postings* const* ws, const int* ks, uint32_t nk, const uint8_t* d_res,
                             const uint64_t* d_res_off, const uint16_t* d_class, uint32_t n, uint64_t slots,
                             uint32_t min_shared, int require_class_diff, uint32_t row_lo, uint32_t row_hi,
                             uint32_t* d_p, uint32_t* d_q, uint32_t* d_w, uint32_t* d_score, uint32_t* d_w0,
                             uint32_t* d_w1, uint64_t cap, uint64_t* n_edges, kmp_postings_stats* stats,
                             void* stream) {
    if (!ws || !ks || nk != 2 || !n_edges || row_lo > row_hi || row_hi > n) return KMP_EINVAL;
    if (!ws[0] || !ws[1] || ws[0] == ws[1] || ks[0] == ks[1]) return KMP_EINVAL;
    for (uint32_t j = 0; j < nk; ++j)
        if (ks[j] < 1 || ks[j] > kMaxK) return KMP_EINVAL;
    if (cap && (!d_p || !d_q || !d_w || !d_score || !d_w0 || !d_w1)) return KMP_EINVAL;
    if (row_hi - row_lo > kmp_dev_rows_max(n, 2)) return KMP_EINVAL;
    *n_edges = 0;
    if (stats) *stats = kmp_postings_stats{};
    if (row_lo == row_hi || n < 2) return KMP_OK;
    if (!d_res || !d_res_off || !d_class) return KMP_EINVAL;
    hipStream_t st = as_stream(stream);
    const bool ranged = !(row_lo == 0 && row_hi == n);
    // the tail's geometry and outputs (the same StepCfg fields the step uses)
    StepCfg c{};
    c.n = n;
    c.min_shared = std::max(1u, min_shared);
    c.ranged = ranged;
    c.row_lo = row_lo;
    c.row_hi = row_hi;
    c.d_p = d_p;
    c.d_q = d_q;
    c.d_w = d_w;
    c.cap = cap;
    c.stride = 1;
    c.sb = kScoreBits + 1;
    c.d_s = d_score;
    c.d_w1 = d_w1;
    c.d_w0 = d_w0;
    const std::vector<unsigned long long> call = {n, (unsigned long long)ks[0], (unsigned long long)ks[1], row_lo, row_hi,
                                                  c.min_shared, (unsigned long long)require_class_diff, slots,
                                                  (uintptr_t)d_res, (uintptr_t)ws[1]};
    if (ws[0]->pend_key == call) {  // the same call after KMP_EOVERFLOW: emit the staged runs again
        const int rc = tail_multi_emit(ws[0], c, n_edges, st);
        if (rc == KMP_OK) ws[0]->pend_key.clear();
        return rc;
    }
    ws[0]->pend_key.clear();
    uint64_t inc[2] = {0, 0};
    kmp_postings_stats s0{};
    const bool timed = stats != nullptr;  // stage_ms: [0] first k expanded, [1] second k, [2] the fused tail
    if (timed && !ws[0]->mev[0])
        for (auto& e : ws[0]->mev) PG(hipEventCreate(&e));
    if (timed) PG(hipEventRecord(ws[0]->mev[0], st));
    for (uint32_t j = 0; j < nk; ++j) {
        // expand only: every incidence keyed (pair << 8) | j << 7 | s(x)
        uint64_t unused = 0;
        int rc = residues_impl(ws[j], d_res, d_res_off, d_class, n, ks[j], slots, 0xFFFFFFFFu, 1, require_class_diff,
                               ranged, row_lo, row_hi, d_p, d_q, d_w, cap, &unused, j == 0 ? &s0 : nullptr, stream,
                               kScoreBits + 1, j << kScoreBits, d_score, d_w1, &inc[j]);
        if (rc != KMP_OK) return rc;
        if (timed) PG(hipEventRecord(ws[0]->mev[1 + j], st));
    }
    int rc = tail_multi(ws, nk, c, inc, n_edges, stats, st);
    if (rc == KMP_EOVERFLOW) ws[0]->pend_key = call;
    if (timed && (rc == KMP_OK || rc == KMP_EOVERFLOW)) {
        PG(hipEventRecord(ws[0]->mev[3], st));
        PG(hipEventSynchronize(ws[0]->mev[3]));
        for (int i = 0; i < 3; ++i) {
            float ms = 0.f;
            stats->stage_ms[i] = hipEventElapsedTime(&ms, ws[0]->mev[i], ws[0]->mev[i + 1]) == hipSuccess ? ms : -1.f;
        }
        (void)hipGetLastError();
        for (int i = 3; i < KMP_POSTINGS_STAGES; ++i) stats->stage_ms[i] = 0.f;
    }
    if (stats) {  // the first k's front statistics
        stats->sum_S = s0.sum_S;
        stats->distinct = s0.distinct;
        stats->repeat = s0.repeat;
        stats->sum_cdf2_light = s0.sum_cdf2_light;
        stats->max_df = s0.max_df;
        stats->heavy_entries = s0.heavy_entries;
    }
    return rc;
}

int kmp_dev_split_expand(kmp_postings* ws, const uint8_t* d_res, const uint64_t* d_res_off, const uint16_t* d_class,
                         uint32_t n, int k, uint64_t slots, uint32_t heavy_df, int require_class_diff, uint32_t part,
                         uint32_t parts, uint64_t cap, const uint32_t* learn, unsigned long long* d_send,
                         uint32_t* d_flags, unsigned long long* d_stats, void* stream) {
    if (!ws || !d_res || !d_res_off || !d_class || !d_send || !d_flags || !d_stats || k < 1 || k > kMaxK ||
        parts < 1 || parts > kSplitMax || part >= parts || cap < 1)
        return KMP_EINVAL;
    hipStream_t st = as_stream(stream);
    if (heavy_df < 2) heavy_df = 2;
    const Layout lay = make_layout(n, k, slots, true);
    if (!lay.bucketed) return KMP_ESTATE;
    const std::vector<unsigned long long> shape = {n, slots, (unsigned long long)k, parts};
    if (ws->split_shape != shape) {  // a new batch: learned capacities start over
        ws->split_shape = shape;
        ws->shard_cap = slots / 4 / kShards / parts + 4096;
        ws->bp_J_min = 0;
        ws->cur_on = ws->cur_mode;
        ws->shape.clear();
        ws->split_heavy = false;
        ws->fast_tail = ws->fast_mode;
    }
    if (learn) {  // the last call's flags, reduced over the ranks: every rank grows the same way
        if (learn[KMP_SPLIT_HEAVY]) ws->split_heavy = true;  // a rank spilled: the heavy path from now on
        // an eighth of slack: the fullest region varies by a few percent from call to call with the
        // heavy path on (3.8 % measured on uniprot k = 5 at G = 2), and a rerun costs a whole step
        if (learn[KMP_SPLIT_MAX_SHARD] > ws->shard_cap)
            ws->shard_cap = learn[KMP_SPLIT_MAX_SHARD] + learn[KMP_SPLIT_MAX_SHARD] / 8 + 256;
        if (learn[KMP_SPLIT_BIN_TILES]) ws->bp_J_min = std::max(ws->bp_J_min, learn[KMP_SPLIT_BIN_TILES] + 2);
        if (learn[KMP_SPLIT_CURSOR]) ws->cur_on = false;
    }
    if (ws->spill_cap == 0) ws->spill_cap = 1024;
    ws->front_ok = false;  // the front below holds one bucket range only
    StepCfg c{};
    c.slots = slots;
    c.lay = lay;
    c.n = n;
    c.heavy_df = heavy_df;
    c.min_shared = 1;
    c.require_diff = require_class_diff;
    c.row_hi = n;
    c.stride = 1;
    PtGeom g;
    if (!pt_geometry(ws, c, slots / 4, &g)) return KMP_EINVAL;
    {
        const int rc = step_reserve(ws, c, g, st);
        if (rc != KMP_OK) return rc;
    }
    PG(ws->split_cur.reserve((uint64_t)kSplitMax * kShards));
    const BpDigits dg = bp_digits(lay);
    ws->bin_lo = (uint32_t)((uint64_t)part * dg.nb1 / parts);
    ws->bin_hi = (uint32_t)((uint64_t)(part + 1) * dg.nb1 / parts);
    auto make_keys = [&](const Layout& l, hipStream_t s) {
        ws->parted = true;
        ws->cur_used = ws->cur_on && cur_geometry(l, &ws->cg);
        return bp_level1(ws, d_res, d_res_off, d_class, k, n, slots, l, s);
    };
    const ClearInKeys guard(ws);
    SplitRows rows{};
    rows.parts = parts;
    kmp_row_split(n, parts, rows.start);
    // the send cursors are cleared with the step's flags (by chunk_desc_kernel in the front); routed
    // (no heavy path): the bucket kernels write the send regions, pre-filled with kNoKey
    const bool routed = !ws->split_heavy;
    auto front = [&](hipStream_t s) -> int {
        const uint32_t ncur = routed ? parts * kShards : parts;
        ws->clear_extra = ws->split_cur.p;
        ws->clear_n = ncur;
        if (routed) {
            PG(hipMemsetAsync(d_send, 0xFF, (size_t)parts * cap * sizeof(unsigned long long), s));
            ws->route_send = d_send;
            ws->route_cap = cap;
            ws->route_rows = rows;
        }
        int rc = KMP_OK;
        if (ws->bin_hi > ws->bin_lo) rc = enqueue_front(ws, make_keys, c, true, s);
        else step_clear_kernel<<<1, 256, 0, s>>>(ws->flags.p, ws->bstats.p, ws->split_cur.p, ncur);  // no bins
        ws->clear_extra = nullptr;
        ws->clear_n = 0;
        ws->route_send = nullptr;
        return rc;
    };
    auto route = [&](hipStream_t s, int heavy_done) -> int {
        if (routed) {  // the bucket kernels routed the keys: the flags and statistics only
            split_pad_finish_kernel<<<dim3(1, 1), 256, 0, s>>>(d_send, cap, ws->split_cur.p, ws->bstats.p, ws->flags.p,
                                                                ws->shard_cap, parts, d_flags, d_stats, heavy_done, 1);
            PG(hipGetLastError());
            return KMP_OK;
        }
        const unsigned long long* cursor = ws->bstats.p + kRbCursor;
        split_route_kernel<<<dim3((uint32_t)((ws->shard_cap + kRtTile - 1) / kRtTile), kShards), kRtThreads, 0, s>>>(
            ws->inc_sorted.p, cursor, ws->shard_cap, bits_for(n), rows, cap, d_send, ws->split_cur.p);
        split_pad_finish_kernel<<<dim3((uint32_t)std::min<uint64_t>((cap + 1023) / 1024, 256), parts), 256, 0, s>>>(
            d_send, cap, ws->split_cur.p, ws->bstats.p, ws->flags.p, ws->shard_cap, parts, d_flags, d_stats,
            heavy_done, 0);
        PG(hipGetLastError());
        return KMP_OK;
    };
    if (ws->split_heavy) {
        // frequent k-mers (vertex.rs:59-140 at k = 5): the rank's front, one read-back, its spill
        // compacted, planned and expanded by the heavy path into the same shard regions (the heavy
        // pairs of the rank's k-mers, all rows), then routed like the light keys.  The spill regions
        // are the rank's own, so a spill overflow reruns the front here; every other capacity is
        // reported in the flags and grown identically on every rank.  Host-synchronous.
        int rc = KMP_OK;
        bool routed = false;
        for (int attempt = 0; attempt < 4; ++attempt) {
            if ((rc = step_reserve(ws, c, g, st)) != KMP_OK) break;
            if ((rc = front(st)) != KMP_OK) break;
            step_pack_kernel<<<1, 256, 0, st>>>(ws->bstats.p, ws->flags.p, nullptr, ws->hrb);
            PG(hipStreamSynchronize(st));
            const unsigned long long* rb = ws->hrb;
            unsigned long long acc[kStN], most, n_inc, spill_most, spill_total;
            sum_stats(rb, acc, &most, &n_inc, &spill_most, &spill_total);
            if (spill_most > ws->spill_cap) {
                ws->spill_cap = spill_most + spill_most / 8 + 1024;
                continue;
            }
            // a bin or cursor-region overflow: the flags rerun the step, no heavy work on it
            if (spill_total && !rb[kRbFlagBin] && !(rb[kRbFlagCur] && ws->cur_used)) {
                ws->heavy_ready = ws->hcur_valid = false;  // this call's front
                ws->h_segs = rb[kRbSegs];
                ws->h_segmax = rb[kRbSegMax];
                if ((rc = heavy_phase(ws, c, spill_total, true, st)) != KMP_OK) break;
            }
            rc = route(st, 1);
            routed = true;
            break;
        }
        ws->bin_lo = ws->bin_hi = 0;
        // every attempt grew the spill regions: the send buffer and flags were never written
        if (rc == KMP_OK && !routed) return KMP_EOVERFLOW;
        return rc;
    }
    auto enqueue = [&](hipStream_t s) -> int {
        const int rc = front(s);
        return rc != KMP_OK ? rc : route(s, 0);
    };
    const std::vector<unsigned long long> key = {
        n, slots, (unsigned long long)k, heavy_df, (unsigned long long)require_class_diff, part, parts, cap,
        (uintptr_t)d_res, (uintptr_t)d_res_off, (uintptr_t)d_class, (uintptr_t)d_send, (uintptr_t)d_flags,
        (uintptr_t)d_stats, ws->shard_cap, ws->spill_cap, ws->bp_J_min, ws->cur_on, ws->timing};
    const int rc = slot_launch(ws, ws->split_g[0], key, enqueue, st);
    ws->bin_lo = ws->bin_hi = 0;
    return rc;
}

int kmp_dev_split_edges(kmp_postings* ws, const unsigned long long* d_keys, uint64_t m, uint32_t n, uint32_t row_lo,
                        uint32_t row_hi, uint32_t min_shared, uint32_t* d_p, uint32_t* d_q, uint32_t* d_w,
                        uint64_t cap, uint64_t* n_edges, void* stream) {
    if (!ws || !n_edges || row_lo > row_hi || row_hi > n || (m && !d_keys) || (cap && (!d_p || !d_q || !d_w)))
        return KMP_EINVAL;
    *n_edges = 0;
    if (m == 0 || row_lo == row_hi) return KMP_OK;
    if (m > 0xFFFFFFFFull) return KMP_EINVAL;
    hipStream_t st = as_stream(stream);
    StepCfg c{};
    c.n = n;
    c.min_shared = std::max(1u, min_shared);
    c.ranged = true;
    c.row_lo = row_lo;
    c.row_hi = row_hi;
    c.d_p = d_p;
    c.d_q = d_q;
    c.d_w = d_w;
    c.cap = cap;
    c.stride = 1;
    for (int attempt = 0; attempt < 2; ++attempt) {
        PtGeom g;
        if (!pt_geometry(ws, c, m, &g)) return KMP_EINVAL;
        g.flat_n = m;  // the received regions, padded with kNoKey, read as one array
        g.nshards = 1;
        g.sc = m;
        g.jt = (uint32_t)((m + kPtTile - 1) / kPtTile);
        hipError_t e = hipSuccess;
        pt_bufs(ws, g, true, &e, st);
        PG(e);
        PG(ws->inc.reserve(pt_fast(ws, g) && !g.dense ? std::max<uint64_t>(m, (uint64_t)g.nrb * g.ftcap / 2) : m));  // u32 row-block keys
        PG(ws->uniq.reserve(m));  // staged p | q (u32 each)
        PG(ws->w.reserve(m));
        PG(ws->ovf.reserve((uint64_t)g.nrb + 1));
        PG(ws->small.reserve(16));
        PG(ws->flags.reserve(kFlN));
        PG(ws->bstats.reserve(kGsWords));
        if (!ws->hrb) PG(hipHostMalloc((void**)&ws->hrb, kRbWords * sizeof(unsigned long long), hipHostMallocCoherent));
        auto enqueue = [&](hipStream_t s) -> int {
            step_clear_kernel<<<1, 256, 0, s>>>(ws->flags.p, ws->bstats.p);  // flags (the expand's stats are out)
            return enqueue_tail_in(ws, c, g, d_keys, nullptr, m, s);
        };
        const std::vector<unsigned long long> key = {m, n, row_lo, row_hi, c.min_shared, cap, (uintptr_t)d_keys,
                                                     (uintptr_t)d_p, (uintptr_t)d_q, (uintptr_t)d_w, g.rbits,
                                                     ws->timing, ws->fast_tail};
        int rc = slot_launch(ws, ws->split_g[1], key, enqueue, st);
        if (rc != KMP_OK) return rc;
        PG(hipStreamSynchronize(st));
        const unsigned long long* rb = ws->hrb;
        if (rb[kRbFast]) {  // a fast-tail region overflowed: the counting tail (learned until a new shape)
            ws->fast_tail = false;
            continue;
        }
        uint64_t ne = rb[kRbRuns];
        if (rb[kRbOvf] && !pt_rowhist_ok(g)) {  // row blocks above the LDS capacity: the segmented sort, fewer rows per block next time
            if (g.rbits > 0) {
                const double over = (double)rb[kRbMaxBlock] / (0.8 * kPtCap);
                unsigned shrink = 1;
                while (shrink < 16 && (double)(1u << shrink) < over) ++shrink;
                ws->pt_rb_max = g.rbits > shrink ? g.rbits - shrink : 0u;
            }
            rc = pt_finish_overflow(ws, c, g, (uint32_t)rb[kRbOvf], &ne, st, m);
            if (rc != KMP_OK) return rc;
        }
        *n_edges = ne;
        return ne > cap ? KMP_EOVERFLOW : KMP_OK;
    }
    return KMP_EDEVICE;
}

// Row ranges of a split of the pair space: a pair belongs to its smaller protein, so row p owns
// about N - p pairs; range d starts at N * (1 - sqrt(1 - d/parts)) (equal expected pair counts).
void kmp_row_split(uint32_t n, uint32_t parts, uint32_t* start) {
    for (uint32_t d = 0; d <= parts; ++d) {
        const double x = 1.0 - std::sqrt(1.0 - (double)d / parts);
        start[d] = d == parts ? n : (uint32_t)std::min<double>(n, std::floor(x * n));
    }
}

}  // extern "C"

#undef PG
