// postings/partition.hip — the two-level bucket partition (level 1 from the residues, level 2 gather + cursor).
// Part of kmp_postings.hip (included there; not a translation unit of its own).

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

// workgroup size of the local level 1 (a 4,096-slot chunk either way; 512 threads own 8 slots each:
// twice the waves per CU at the same LDS; keys_level1 0.139 -> 0.127 ms at config 3)
constexpr uint32_t kL1Threads = 512;

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
// (chunk range [c_lo, c_hi) only, at desc[c - c_lo]: a rank of the k-mer split keys its own chunks)
__global__ void chunk_desc_kernel(const uint64_t* __restrict__ res_off, uint32_t n, uint64_t slots,
                                  uint32_t c_lo, uint32_t c_hi, int k, uint4* __restrict__ desc, uint32_t* __restrict__ cur,
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
    for (uint64_t c = max<uint64_t>((b + kKeyChunk - 1) / kKeyChunk, c_lo); c * kKeyChunk < e && c < c_hi; ++c) {
        desc[c - c_lo].x = p;
        desc[c - c_lo].z = (uint32_t)(off + min<uint64_t>(c * kKeyChunk - b, L));
    }
    // chunks whose last slot min((c + 1) * kKeyChunk, slots) - 1 lies in [b, e)
    for (uint64_t c = max<uint64_t>(b / kKeyChunk, c_lo); c < c_hi; ++c) {
        const uint64_t c1 = min<uint64_t>((c + 1) * kKeyChunk, slots);
        if (c1 - 1 >= e) break;
        if (c1 - 1 < b) continue;
        desc[c - c_lo].y = p;
        desc[c - c_lo].w = (uint32_t)(p < n ? off + min<uint64_t>(L, c1 - b + k - 1) : off);
    }
}

// The k-mer split with a sharded start (kmp_dev_split_keys): rank `part` holds the residues of its
// chunk range only, keys those chunks with the level-1 kernel below, and sends each chunk's keys
// of rank d's coarse bins (one contiguous digit-major piece of the ranked chunk) to region d of
// the send buffer; the all-to-all of the send buffers hands every rank the keys of its bins from
// every chunk, and its level 2 reads them where they landed (bp_scatter2g<.., kRecv>).
// Region d (cap u64 words): a run table of cm rows (the most chunks a rank holds), row i =
// {chunk i's piece: its u64 index in the RECEIVER's buffer (the sender is source `part`, whose
// region lands at part * cap) | start << 16 | count of each of d's bins, relative to it}, then the
// pieces, in kSendShards sub-regions of sub keys (chunk c's piece goes to sub-region c mod
// kSendShards, reserved on a cursor per (destination, sub-region): the fill of each sub-region
// depends on the chunks only, never on the order of the atomics).  A piece that does not fit is
// dropped with its counts (0) and raises kFlSend; the cursors still count it, so the rerun's
// region size is exact.
// 64 sub-regions: the returning reservation atomics of ~1,000 simultaneous chunks spread over 64 x
// parts cursors (16 sub-regions: 46 us for a rank's keys at G = 8, 64: 36 us; 128: 35 us)
constexpr uint32_t kSendShards = 64;
struct SendL1 {
    unsigned long long* send;  // parts regions of cap u64 words
    uint64_t cap, tb;          // region size; run-table words (u64) at its start
    uint32_t sub;              // keys per sub-region
    uint32_t* kcur;            // parts x kSendShards cursors
    uint32_t part, parts, c_lo, rowlen;  // rowlen: u32 words per table row (most bins a rank owns + 1)
    uint64_t res_base, res_end;  // the residue slice [res_base, res_end) at res
};
// coarse bins [bin_lo(d), bin_lo(d + 1)) belong to rank d (the k-mer split's share), and bin t to
// owner(t) = the largest d with bin_lo(d) <= t = ((t + 1) parts - 1) / nb1
__host__ __device__ __forceinline__ uint32_t split_bin_lo(uint32_t d, uint32_t nb1, uint32_t parts) {
    return (uint32_t)((uint64_t)d * nb1 / parts);
}

// waves per SIMD the persistent level 1 is compiled for (VGPR budget: 8 -> 64 registers and 24 B of
// scratch per lane, four 512-thread workgroups per CU; at 6 waves, 79 registers, a rank of the k-mer
// split at G = 8 spent 91 us in it against 86 us at 8; one GPU: the same)
constexpr uint32_t kL1pWaves = 8;
// Level 1, local, persistent: workgroup w takes chunks w, w + grid, ...; chunk c's keys of the
// call's digits [dlo, dhi) grouped by digit1 at out[c * kKeyChunk ...] (its own 4,096-key segment),
// its run table (start << 16 | count per own digit) in H1[c][digit - dlo].  The next chunk's
// residues and protein table are loaded into registers while this chunk is keyed, ranked and
// written (its descriptor one chunk earlier still), so the three dependent global round trips of
// a chunk (descriptor, protein offsets, residues) stay off the critical path: the one-chunk-per-
// workgroup kernel spent ~13 us per chunk waiting on them.
// kSend (the k-mer split's sharded start): the chunks are [sl.c_lo, sl.c_lo + G) of the batch (desc
// and the loop count them from 0), the residues a slice (SendL1.res_base / res_end), every digit is
// ranked and each rank's piece goes to the send buffer with its run-table row (SendL1 above)
// instead of the segment + H1.
// kPersist: a workgroup walks chunks blockIdx.x, + gridDim.x, ... with the next chunk's loads in
// flight (a rank's share of the bins, a grid of what fits the device); otherwise it keys chunk
// blockIdx.x alone (one GPU, and the sharded start: a grid of one workgroup per chunk), with no
// next-chunk registers held across the chunk's work
template <uint32_t kThr, bool kSend, bool kPersist, bool kTrans = false>
__global__ __launch_bounds__(kThr, kL1pWaves) void bp_scatter1p_kernel(
    const uint8_t* __restrict__ res, const uint64_t* __restrict__ res_off, const uint16_t* __restrict__ cls, int k,
    uint32_t n, uint64_t slots, uint32_t G, const uint4* __restrict__ desc, Layout lay, BpDigits dg, uint32_t pw21,
    uint32_t dlo, uint32_t dhi, uint32_t* __restrict__ H1, unsigned long long* __restrict__ out,
    uint32_t* __restrict__ flags, SendL1 sl) {
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
    // kTrans (one GPU: every bin, one chunk per workgroup): XCD-aware chunk order — workgroup L runs
    // on XCD L % 8, and XCD x keys the consecutive chunks [x per, (x + 1) per) — so the run table is
    // written transposed (H1T[digit][chunk], level 2's reading order) straight from here: the words
    // of one table row come from the consecutive chunks of one XCD and meet in its L2 (no bp_h1t)
    static_assert(!kTrans || (!kSend && !kPersist), "the transposed table: one chunk per workgroup");
    uint32_t c = blockIdx.x;
    if (kTrans) {
        const uint32_t per = (G + 7) / 8;
        c = (blockIdx.x % 8) * per + blockIdx.x / 8;
    }
    if (c >= G) return;
    for (uint32_t i = tid; i < 256; i += kThr) lut[i] = c_lut.v[i];
    __syncthreads();  // the table before the first staging reads it
    // residue i (absolute) is res[i - rb]: the whole batch, or (kSend) a slice starting at rb
    const uint64_t rb = kSend ? sl.res_base : 0ull, res_end = kSend ? sl.res_end : res_off[n];
    const bool vec_ok = ((uintptr_t)res & 15u) == 0 && (rb & 15u) == 0;
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
                pv = *reinterpret_cast<const uint4*>(res + (g - rb));
            } else {
                uint32_t w[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    w[q] = 0;
#pragma unroll
                    for (int bb = 0; bb < 4; ++bb) {
                        const uint64_t i = g + 4 * q + bb;
                        w[q] |= (uint32_t)(i >= rb && i < res_end ? res[i - rb] : 0) << (8 * bb);
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
    uint4 dnxt = kPersist && c + gridDim.x < G ? desc[c + gridDim.x] : make_uint4(0, 0, 0, 0);
    issue(dcur);
    const unsigned hs1 = dg.sh1 - lay.hshift;
    __shared__ uint32_t sd_base[kSend ? kSplitMax : 1], sd_start[kSend ? kSplitMax : 1];
    __shared__ uint32_t s_blo[kSend ? kSplitMax + 1 : 1];  // first bin of each rank (split_bin_lo)
    if (kSend)
        for (uint32_t d = tid; d <= sl.parts; d += kThr) s_blo[d] = split_bin_lo(d, dg.nb1, sl.parts);
    while (true) {
        const uint32_t gc = kSend ? c + sl.c_lo : c;  // the chunk's index in the batch
        const uint64_t c0 = (uint64_t)gc * kKeyChunk, c1 = min(c0 + kKeyChunk, slots);
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
        const uint32_t cn = kPersist ? c + gridDim.x : G;
        uint4 dnn = make_uint4(0, 0, 0, 0);
        if (kPersist && cn < G) {
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
        if (kTrans) {  // H1 is the transposed table here: row d - dlo holds the G chunks' runs of digit d
#pragma unroll
            for (uint32_t t = 0; t < kQ; ++t) {
                const uint32_t d = tid + t * kThr;
                if (d < nown) H1[(uint64_t)d * G + c] = lh[dlo + d] << 16 | cnt[t];
            }
        } else if (!kSend) {
            uint32_t* row = H1 + (uint64_t)c * nown;
#pragma unroll
            for (uint32_t t = 0; t < kQ; ++t) {
                const uint32_t d = tid + t * kThr;
                if (d < nown) row[d] = lh[dlo + d] << 16 | cnt[t];
            }
        }
#pragma unroll
        for (uint32_t e = 0; e < kPer; ++e)
            if (x[e] != kNoKey) u.S[lh[(uint32_t)(x[e] >> dg.sh1)] + r[e]] = x[e];
        __syncthreads();
        const uint32_t n_in = s_n;
        if (kSend) {
            // every digit is the call's (dlo = 0, dhi = nb1): rank d's piece is the chunk's keys of
            // its bins, contiguous in S; one reservation per destination
            const uint32_t nb1 = dg.nb1, l1 = __builtin_ctz(nb1);  // nb1 is a power of two
            // owner(t) = ((t + 1) parts - 1) / nb1: a multiply and a shift per key (split_owner)
            auto owner = [&](uint32_t t) { return ((t + 1) * sl.parts - 1) >> l1; };
            if (tid < sl.parts) {
                const uint32_t b0 = s_blo[tid], b1 = s_blo[tid + 1];
                const uint32_t s0 = b0 < nb1 ? lh[b0] : n_in, s1 = b1 < nb1 ? lh[b1] : n_in;
                const uint32_t size = s1 - s0, shard = gc % kSendShards;
                const uint32_t pos = size ? atomicAdd(&sl.kcur[tid * kSendShards + shard], size) : 0u;
                const bool fits = pos + size <= sl.sub;
                if (!fits) flags[kFlSend] = 1;
                sd_base[tid] = fits && sl.sub ? shard * sl.sub + pos : 0xFFFFFFFFu;
                sd_start[tid] = s0;
                // the row's first word: where the piece lands in the receiver's buffer (sub = 0: the
                // region cannot even hold the run table — nothing is written, the cursors count)
                if (sl.sub)
                    reinterpret_cast<uint32_t*>(sl.send + (uint64_t)tid * sl.cap)[(uint64_t)c * sl.rowlen] =
                        fits ? (uint32_t)((uint64_t)sl.part * sl.cap + sl.tb + shard * sl.sub + pos) : 0u;
            }
            __syncthreads();
#pragma unroll
            for (uint32_t t = 0; t < kQ; ++t) {
                const uint32_t dgt = tid + t * kThr;
                if (dgt < nb1 && sl.sub) {
                    const uint32_t d = owner(dgt);
                    const bool fits = sd_base[d] != 0xFFFFFFFFu;
                    uint32_t* row = reinterpret_cast<uint32_t*>(sl.send + (uint64_t)d * sl.cap) + (uint64_t)c * sl.rowlen;
                    row[1 + dgt - s_blo[d]] = fits ? (lh[dgt] - sd_start[d]) << 16 | cnt[t] : 0u;
                }
            }
            for (uint32_t i = tid; i < n_in; i += kThr) {
                const unsigned long long y = u.S[i];
                const uint32_t d = owner((uint32_t)(y >> dg.sh1));
                const uint32_t b = sd_base[d];
                if (b != 0xFFFFFFFFu) sl.send[(uint64_t)d * sl.cap + sl.tb + b + (i - sd_start[d])] = y;
            }
        } else {
            unsigned long long* seg = out + c0;  // c0 = chunk * kKeyChunk: 16-byte aligned
            for (uint32_t i = 2 * tid; i < n_in; i += 2 * kThr) {
                if (i + 1 < n_in)
                    *reinterpret_cast<ulonglong2*>(seg + i) = *reinterpret_cast<const ulonglong2*>(u.S + i);
                else
                    seg[i] = u.S[i];
            }
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
// takes the tiles [x * per, (x + 1) * per) of the tile list, tile-major: the
// consecutive workgroups of an XCD take adjacent bins of one chunk range, whose runs share the
// 128-B lines at their ends, so the second reader finds them in L2 (bp_scatter2g's fetch at config 3:
// 349 MB bin-major, 242 MB tile-major, for 235 MB of keys).
// kRecv (the k-mer split's sharded start): the runs are the received pieces — chunk row g of the
// G = parts * cm rows is row g mod cm of source g / cm's region (stride u32 words apart), rows past
// that source's chunk count are empty, and each row starts with the u64 index its runs are
// relative to (SendL1)
struct RecvTab {
    uint32_t cm;         // rows per source region (the most chunks a rank holds)
    uint32_t n_chunks;   // chunks of the batch (source s holds [s C / parts, (s + 1) C / parts))
    uint32_t parts;
    uint64_t stride;     // u32 words between source regions (2 x the region's u64 words)
    uint64_t tb;         // run-table u64 words at the start of a region
};
template <uint32_t kPer, uint32_t kThr, bool kVreg, bool kRecv>
__global__ __launch_bounds__(kThr) void bp_scatter2g_kernel(const unsigned long long* __restrict__ in,
                                                                   const uint32_t* __restrict__ H1T, uint32_t G,
                                                                   uint32_t hsb, uint32_t hsc,
                                                                   uint32_t T, uint32_t ntiles, uint32_t nbins,
                                                                   BpDigits dg, CurGeom cg,
                                                                   uint32_t* __restrict__ bcur,
                                                                   unsigned long long* __restrict__ out,
                                                                   uint32_t* __restrict__ flags, uint32_t c0,
                                                                   uint32_t dlo, RecvTab rt) {
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
    // tile-major: consecutive workgroups of an XCD take adjacent bins of one chunk range, whose runs
    // share their first and last 128-B lines, read by the next workgroup from L2
    const uint32_t c = c0 + w % nbins, ch0 = (w / nbins) * T;
    if (ch0 >= G) return;
    const uint32_t nch = min(T, G - ch0);
    const uint32_t* row = H1T + (uint64_t)(c - dlo) * hsb + (uint64_t)ch0 * hsc;
    const uint32_t q = (nch + kThr - 1) / kThr, b0 = threadIdx.x * q;
    uint32_t p[kQ], rbase[kRecv ? kQ : 1], v = 0;
#pragma unroll
    for (uint32_t t = 0; t < kQ; ++t) {
        if (kRecv) {
            const uint32_t g = ch0 + b0 + t, s = g / rt.cm, i = g - s * rt.cm;
            const uint32_t nsrc = s < rt.parts ? (uint32_t)((uint64_t)(s + 1) * rt.n_chunks / rt.parts -
                                                            (uint64_t)s * rt.n_chunks / rt.parts)
                                               : 0u;
            // a row past the region's table, or a run outside the source's key part, reads as empty
            // (only a sender's error path could produce one; nothing is read out of bounds)
            const bool ok = t < q && b0 + t < nch && i < nsrc && ((uint64_t)i + 1) * hsc <= 2 * rt.tb;
            const uint32_t* rw = H1T + s * rt.stride + (uint64_t)i * hsc;
            p[t] = ok ? rw[1 + c - dlo] : 0u;
            rbase[t] = ok ? rw[0] : 0u;
            const uint64_t lo = (uint64_t)s * (rt.stride / 2) + rt.tb, hi = (uint64_t)(s + 1) * (rt.stride / 2);
            if ((p[t] & 0xFFFFu) && (rbase[t] + (p[t] >> 16) < lo || rbase[t] + (p[t] >> 16) + (p[t] & 0xFFFFu) > hi)) {
                p[t] = 0;
                flags[kFlSend] = 1;
            }
        } else {
            p[t] = t < q && b0 + t < nch ? row[(uint64_t)(b0 + t) * hsc] : 0u;
        }
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
                src[b0 + t] = (kRecv ? rbase[t] : (ch0 + b0 + t) * kKeyChunk) + (p[t] >> 16) - excl;
                excl += p[t] & 0xFFFFu;
            }
        // key -> run map of the round's window [base, base + n_in)
        // each run marks its first position in the window (the run covering position base marks
        // 0), then a block-wide inclusive max-scan carries every mark over its run: run ids grow
        // with position.  (A thread filling its runs' positions in a loop ran as long as its wave's
        // longest runs: ~30-50 iterations per round.)
        static_assert(kTile == 16 * kThr, "16 map positions per thread");
        uint4* m4 = reinterpret_cast<uint4*>(map) + 2 * threadIdx.x;
        m4[0] = m4[1] = make_uint4(0, 0, 0, 0);
        __syncthreads();
        excl = excl0;
#pragma unroll
        for (uint32_t t = 0; t < kQ; ++t)
            if (t < q && b0 + t < nch) {
                const uint32_t e1 = excl + (p[t] & 0xFFFFu);
                const uint32_t lo = max(excl, base), hi = min(e1, base + n_in);
                if (lo < hi) map[lo - base] = (uint16_t)(b0 + t);
                excl = e1;
            }
        __syncthreads();
        {
            uint4 w0 = m4[0], w1 = m4[1];
            uint32_t wd[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
            uint32_t agg = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) agg = max(agg, max(wd[j] & 0xFFFFu, wd[j] >> 16));
            // inclusive max over the lanes, then the wave's lanes before this one, then earlier waves
            uint32_t inc = agg;
            inc = max(inc, dpp_mov<0x111>(inc));
            inc = max(inc, dpp_mov<0x112>(inc));
            inc = max(inc, dpp_mov<0x114>(inc));
            inc = max(inc, dpp_mov<0x118>(inc));
            inc = max(inc, dpp_mov<0x142, 0xA>(inc));
            inc = max(inc, dpp_mov<0x143, 0xC>(inc));
            const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
            uint32_t before = (uint32_t)__shfl_up((int)inc, 1);
            if (lane == 0) before = 0;
            if (lane == 63) wave_tot[wv] = inc;
            __syncthreads();
#pragma unroll
            for (uint32_t i = 0; i < kThr / 64; ++i)
                if (i < wv) before = max(before, wave_tot[i]);
            uint32_t run = before;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t lo16 = max(run, wd[j] & 0xFFFFu);
                run = max(lo16, wd[j] >> 16);
                wd[j] = lo16 | run << 16;
            }
            m4[0] = make_uint4(wd[0], wd[1], wd[2], wd[3]);
            m4[1] = make_uint4(wd[4], wd[5], wd[6], wd[7]);
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
// the small kernel over buckets [b0, b0 + nb)
template <bool kRows, bool kScore>
void launch_small(const BucketArgs& a, uint32_t b0, uint32_t nb, hipStream_t st) {
    if (!nb) return;
    if (a.lay.bbits >= kMergeMinBits && a.lay.mean_keys <= kBucketCap1024Mean)  // four keys per thread
        bucket_small_kernel<1024, kBucketSmallThreads, kBucketSmallTab, true, kRows, kScore>
            <<<nb, kBucketSmallThreads, 0, st>>>(a, b0);
    else if (a.lay.bbits >= kMergeMinBits)
        bucket_small_kernel<kBucketSmallCap, kBucketSmallThreads, kBucketSmallTab, true, kRows, kScore>
            <<<nb, kBucketSmallThreads, 0, st>>>(a, b0);
    else
        bucket_small_kernel<kBucketSmallCap, kBucketSmallThreads, kBucketSmallTab, false, kRows, kScore>
            <<<nb, kBucketSmallThreads, 0, st>>>(a, b0);
}
// buckets [b0, b0 + nb): the small kernel, then the large one over the buckets it listed
template <bool kRows, bool kScore>
void launch_buckets(const BucketArgs& a, uint32_t b0, uint32_t nb, uint32_t large_grid, hipStream_t st) {
    launch_small<kRows, kScore>(a, b0, nb, st);
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
