// postings/tail.hip — row-block tails (combine_edges): counting tail, step read-back, fast tail.
// Part of kmp_postings.hip (included there; not a translation unit of its own).

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
constexpr uint32_t kPtThreads = 1024, kPtPer = 16, kPtTile = kPtThreads * kPtPer;  // partition tiles: 16,384 keys
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
// also clears the reduce's look-back words lb[0, nrb) and its ticket.  Tiles of 8,192 keys: twice the workgroups
// of the counting tail's 16,384-key tiles (which ran one per CU), at LDS for two per CU: 80 KB at
// most, so the histogram holds kFtScBlocks = kPtMaxBlocks - 16 row blocks (the fast tail's limit;
// the full 8,192 plus the scan's words was 36 B over, one workgroup per CU)
constexpr uint32_t kFtCap = 8192;  // fast tail, hash reduce: keys per row-block region
constexpr uint32_t kFtScThreads = 512, kFtScTile = kFtScThreads * 16, kFtScBlocks = kPtMaxBlocks - 16;
__global__ __launch_bounds__(kFtScThreads) void pt_scatter_capped_kernel(const unsigned long long* __restrict__ in,
                                                                         const unsigned long long* __restrict__ cursor,
                                                                         PtGeom g, uint32_t* __restrict__ cur,
                                                                         uint32_t* __restrict__ out,
                                                                         unsigned long long* __restrict__ lb,
                                                                         uint32_t* __restrict__ ticket, StepClear sc,
                                                                         uint32_t* __restrict__ flags) {
    constexpr uint32_t kThr = kFtScThreads, kPer = 16;
    __shared__ uint32_t lh[kFtScBlocks];
    __shared__ uint32_t S[kFtScTile];
    __shared__ uint16_t SR[kFtScTile];
    static_assert(sizeof(uint32_t) * (kFtScBlocks + kFtScTile + kFtScThreads / 64 + 1) +
                              sizeof(uint16_t) * kFtScTile <= 80 * 1024,
                  "two workgroups per CU");
    __shared__ uint32_t wave_tot[kThr / 64];
    __shared__ uint32_t s_n;
    const uint32_t j = blockIdx.x, s = blockIdx.y;
    if (j == 0 && s == 0) {
        for (uint32_t r = threadIdx.x; r < g.nrb; r += kThr) lb[r] = 0;
        if (threadIdx.x == 0) *ticket = 0;
        // (a tail-only call: the step's flags and statistics, which only the reduce reads)
        if (sc.flags)
            for (uint32_t i = threadIdx.x; i < sc.n_flags; i += kThr) sc.flags[i] = 0;
        if (sc.gstats)
            for (uint32_t i = threadIdx.x; i < sc.n_gstats; i += kThr) sc.gstats[i] = 0;
    }
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
        if (x[e] != kNoKey) x[e] -= base;  // rows from row0 (a row below it wraps past the span)
    }
    if (g.flat_n) {
        // received keys (the k-mer split's edges phase: another rank's output): a key outside the
        // call's row blocks is dropped and fails the call, never indexes past the histogram.  The
        // call's own bucket kernels (one GPU) write nothing else, so its step skips the test
        const unsigned long long span = (unsigned long long)g.nrb << sh;
        bool outside = false;
#pragma unroll
        for (uint32_t e = 0; e < kPer; ++e)
            if (x[e] != kNoKey && x[e] >= span) {
                outside = true;
                x[e] = kNoKey;
            }
        if (outside) flags[kFlRange] = 1;
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
    // block r's region: [r * ftcap, (r + 1) * ftcap); a run that does not fit is dropped whole (the
    // cursor still counts it: the reduce flags the block)
    uint32_t rabs[kQ];
#pragma unroll
    for (uint32_t t = 0; t < kQ; ++t) {
        const uint32_t r = threadIdx.x + t * kThr;
        rabs[t] = 0xFFFFFFFFu;
        if (cnt[t]) {
            if (rbase[t] + cnt[t] <= g.ftcap) rabs[t] = r * g.ftcap + rbase[t];
        }
    }
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
        // the run's position in out minus its staging start (all ones: dropped)
        if (r < g.nrb) lh[r] = rabs[t] == 0xFFFFFFFFu ? 0xFFFFFFFFu : rabs[t] - lh[r];
    }
    __syncthreads();
    const uint32_t placed = s_n;
    for (uint32_t i = threadIdx.x; i < placed; i += kThr) {
        const uint32_t a = lh[SR[i]];
        if (a != 0xFFFFFFFFu) out[a + i] = S[i];
    }
}

template <uint32_t kE>
using PtSort = rocprim::block_radix_sort<uint32_t, kPtRThreads, kE>;  // rocprim's digits (8 bits, match ranking)

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
constexpr uint32_t kBinMax = 64;
template <uint32_t kCap>  // bins at most
struct PtBinLdsT {
    uint32_t H[kCap];    // per bin: count, then first rank
    uint32_t S[kPtCap];  // the keys by bin
};
using PtBinLds = PtBinLdsT<8192>;
template <uint32_t kE, uint32_t kBinCap>
__device__ __forceinline__ bool pt_bin_sort(uint32_t (&k)[kE], uint32_t n, const PtGeom& g, uint32_t rowbase,
                                            PtBinLdsT<kBinCap>& b, uint32_t* red, uint32_t* s_flag,
                                            uint32_t* wave_tot) {
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
    // else bin = v nb / range as a multiply-high by nb 2^32 / range (< 2^32: nb < range), one
    // division per thread instead of a 64-bit division per key (~1,600 of the count launch's 2,060
    // VALU instructions per wave at config 5)
    const uint32_t mul = exact ? 0u : (uint32_t)(((uint64_t)nb << 32) / range);
    uint32_t br[kE];                 // bin | rank in it << 16 (bins, ranks < 2^14)
#pragma unroll
    for (uint32_t e = 0; e < kE; ++e) {
        br[e] = 0;
        if (threadIdx.x + e * kT < n) {
            const uint32_t v = pos(k[e]) - lo;
            const uint32_t bin = exact ? v : __umulhi(v, mul);
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
    // bin = pos nf / range: a multiply-high by nf 2^32 / range when the range fits 32 bits (pos < range;
    // a range within nf bins is its own binning), the 64-bit division only beyond
    const bool narrow = range <= 0xFFFFFFFFull;
    const uint32_t mul = narrow && range > nf ? (uint32_t)(((uint64_t)nf << 32) / range) : 0u;
    auto bin = [&](uint32_t k) -> uint32_t {
        const uint32_t q = (k >> g.sbits) & qm;
        const uint64_t pos = (uint64_t)(k >> rs) * span + (q > qlo ? q - qlo : 0u);
        if (narrow) return min(range > nf ? __umulhi((uint32_t)pos, mul) : (uint32_t)pos, nf - 1);
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
    kRbMaxBlock, kRbBinTiles, kRbFlagCur, kRbSegs, kRbSegMax, kRbFast, kRbList, kRbRange, kRbSegL, kRbSegW, kRbWords
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
        rb[kRbRange] = flags[kFlRange];
        rb[kRbSegL] = flags[kFlSegL];
        rb[kRbSegW] = flags[kFlSegW];
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
//                     instead (block radix sort + run-length encoding).  A block whose region
//                     overflowed, or above kFtCap keys, raises the read-back's kRbFast word: the
//                     caller learns the regions from the blocks' exact counts (fast_overflow), or
//                     takes fewer rows per block, and after kFregTries the counting tail for the shape.
//                     (A dense variant counting blocks above kFtCap in LDS bins over (row, q) was
//                     measured and removed in round 5: uniprot at k = 5 0.91 ms against 0.744 ms on
//                     the counting tail, and its 64 KB of bins held the reduce to two workgroups per CU.)
// The last block writes the edge count and the step's read-back.
constexpr uint32_t kFtThreads = 512, kFtHashMax = 6144, kFtSlots = 8192, kFtRowsMax = 1024, kFtRankMax = 256;
constexpr uint32_t kFtEmpty = 0xFFFFFFFFu;
constexpr uint32_t kFtSmallN = 2048;  // a block of at most this many keys hashes into kFtSlots / 2 slots
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
// Positions come from a ticket taken when the block starts, so every predecessor is resident or
// done: the polls end.
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
        uint32_t last[kFtThreads];  // the sort path: each thread's last sorted key
    };
    uint32_t RC[kFtRowsMax + 1];  // pairs per row -> row starts
    uint32_t wave_tot[kFtThreads / 64];
    uint32_t s_max, s_flag;
    unsigned long long s_excl;
};

// waves per SIMD the fast reduce is compiled for: 6, at most 80 VGPRs, so three 512-thread
// workgroups per CU (53 KB of LDS each): pair_sort_rle 0.083 -> 0.071 ms at config 3 (8 waves with a
// 4,096-slot table: 0.104 ms, round 6)
constexpr uint32_t kFtWaves = 6;
__global__ __launch_bounds__(kFtThreads, kFtWaves) void pt_reduce_fast_kernel(const uint32_t* __restrict__ keys,
                                                                    uint32_t* __restrict__ fcur, PtGeom g,
                                                                    unsigned long long* __restrict__ lb,
                                                                    uint32_t* __restrict__ ticket,
                                                                    uint32_t* __restrict__ d_p,
                                                                    uint32_t* __restrict__ d_q,
                                                                    uint32_t* __restrict__ d_w, uint64_t cap,
                                                                    uint32_t stride, PtPack pack,
                                                                    uint32_t* __restrict__ runs) {
    __shared__ __attribute__((aligned(16))) FtLds u;
    __shared__ uint32_t s_r, s_n;
    const uint32_t tid = threadIdx.x;
    const unsigned pb = g.pbits;
    const uint32_t R = 1u << g.rbits;
    // the row block = the look-back position = the order the workgroups started in (a ticket), so
    // every block a look-back polls is resident or done, whatever the dispatch order across XCDs and
    // whatever other kernels share the device.  One thread takes it, reads and re-zeroes the block's
    // cursor while the others clear the row counts; the hash table is cleared once the block's key
    // count is known: at most kFtSmallN keys (most blocks at config 3, mean ~1,700) take a table of
    // half the slots (half the clear and the slot reads), a sort-path block none
    if (tid == 0) {
        const uint32_t r0 = atomicAdd(ticket, 1u);
        s_r = r0;
        s_n = fcur[r0];
        fcur[r0] = 0;  // for the next call
        u.s_max = u.s_flag = 0;
    }
    for (uint32_t i = tid; i <= R; i += kFtThreads) u.RC[i] = 0;
    __syncthreads();
    const uint32_t r = s_r, nraw = s_n;
    // the block's region [r kFtCap, (r + 1) kFtCap); the largest block goes to the read-back (runs[2]
    // -> kRbMaxBlock: how many fewer rows per block an overflowing call takes)
    if (tid == 0 && nraw) atomicMax(&runs[2], nraw);
    bool ovf = nraw > kFtCap;
    const uint32_t n = ovf ? 0u : nraw;
    const unsigned tsh = n <= kFtSmallN ? 20u : 19u;  // hash shift: 12 or 13 slot bits
    const uint32_t nsl = 1u << (32 - tsh);
    if (n <= kFtHashMax) {
        for (uint32_t i = tid; i < nsl; i += kFtThreads) u.h.K[i] = kFtEmpty;
        for (uint32_t i = tid; i < nsl / 2; i += kFtThreads) reinterpret_cast<uint32_t*>(u.h.C)[i] = 0;
        __syncthreads();
    }
    const uint32_t* src = keys + (uint64_t)r * kFtCap;
    uint32_t D = 0;  // the block's kept pairs
    bool sort = n > kFtHashMax, published = false;
    if (!sort) {
        // ---- hash aggregation: pair -> slot, count per slot (the table was cleared above) ----
        uint32_t x[12];
#pragma unroll
        for (uint32_t e = 0; e < 12; ++e) {
            const uint32_t i = tid + e * kFtThreads;
            x[e] = i < n ? src[i] : kFtEmpty;
        }
        // the counts as non-returning adds: a 16-bit count cannot wrap, n <= kFtHashMax < 0xFFFF.
        // (Issuing every key's first probe before any collision loop measured slower: pair_sort_rle
        // 0.073 -> 0.117 ms at config 3, the probe arrays past the 80-VGPR budget of 6 waves)
        static_assert(kFtHashMax < 0xFFFFu, "hash-path counts fit 16 bits");
#pragma unroll
        for (uint32_t e = 0; e < 12; ++e) {
            if (x[e] == kFtEmpty) continue;
            uint32_t sl = (x[e] * 0x9E3779B1u) >> tsh;
            while (true) {
                const uint32_t old = atomicCAS(&u.h.K[sl], kFtEmpty, x[e]);
                if (old == kFtEmpty || old == x[e]) break;
                sl = (sl + 1) & (nsl - 1);
            }
            atomicAdd(reinterpret_cast<uint32_t*>(u.h.C) + (sl >> 1), 1u << (16 * (sl & 1)));
        }
        __syncthreads();
        // ---- kept pairs (w >= min_shared) counted per row, ranked in arrival order ----
        uint32_t ek[16], er[16];  // pair key | rank in its row << 16 | w
#pragma unroll
        for (uint32_t j = 0; j < 16; ++j) {
            const uint32_t sl = tid + j * kFtThreads;
            ek[j] = kFtEmpty;
            if (sl >= nsl) continue;  // (uniform per j)
            const uint32_t k = u.h.K[sl], w = u.h.C[sl];
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
                    // (four row words per 16-byte read measured no faster at config 3, and cost
                    // four more spilled VGPRs)
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
        __syncthreads();  // last aliases the sort storage
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
            runs[1] = atomicExch(&runs[2], 0u);  // the largest block, reset for the next call
        }
        __syncthreads();
        if (pack.rb) step_pack_body(pack.gstats, pack.flags, runs, pack.rb, any_ovf ? 1ull : 0ull);
    }
}
