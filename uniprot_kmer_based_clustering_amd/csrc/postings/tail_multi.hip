// postings/tail_multi.hip — the fused multi-k tail with in-place edges (config 5 passes).
// Part of kmp_postings.hip (included there; not a translation unit of its own).

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
// the count launch's: the sort (4,096 bins at most) and the run heads only, 50 KB — three
// workgroups per CU where PtDirectLds's 66 KB allowed two (the launch waits on its loads: ~60 % of
// a wave's cycles at config 5); compiled for 6 waves per SIMD (80 VGPRs) to match
struct PtCountLds {
    union {
        typename PtSort<2>::storage_type s2;
        typename PtSort<4>::storage_type s4;
        typename PtSort<8>::storage_type s8;
        typename PtSort<16>::storage_type s16;
        PtBinLdsT<4096> b;
        struct {
            uint32_t H[kPtCap + 1];  // each run's first rank | k-bit scan at it << 16
        } r;
    };
    uint32_t last[kPtRThreads];
    uint32_t wave_tot[kPtRThreads / 64];
};
static_assert(sizeof(PtCountLds) <= 160 * 1024 / 3, "three count workgroups per CU");

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
template <uint32_t kE, bool kKbit, bool kWrite, class Lds>
__device__ __forceinline__ void pt_direct_block(Lds& L, typename PtSort<kE>::storage_type& st,
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
                if constexpr (kWrite) L.r.P[base] = k[e] >> sb;
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
    if constexpr (!kWrite) {  // min_shared > 1: the kept runs
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
    } else {
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
__global__ __launch_bounds__(kPtRThreads, 6) void pt_reduce_count_kernel(uint32_t* __restrict__ keys, BlkSrc bs, PtGeom g,
                                                                      uint32_t* __restrict__ wc,
                                                                      unsigned long long* __restrict__ stat) {
    __shared__ PtCountLds L;
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
