// postings/heavy.hip — the heavy path: frequent k-mers spilled by the bucket kernels.
// Part of kmp_postings.hip (included there; not a translation unit of its own).

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
// spilled keys per compaction tile (4,096 ran 249 workgroups at config 1: 11 + 15 us)
constexpr uint32_t kHvTile = 1024, kHvThreads = 256, kHvPer = kHvTile / kHvThreads;
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
// bucket, each holding every key of its k-mers.  Each put in order alone, in LDS, and written where
// the gather would have put it, is the whole sort the heavy path needs (k-mers contiguous, each
// sorted or in class runs): no global radix sort (eight onesweep passes over 1M keys at k = 5,
// 0.3 ms).  One workgroup per segment, in two size classes — config 1 has 3,808 one-k-mer segments
// (93 % of them at most 512 keys) and two whole buckets of ~4,600 keys:
//   heavy_seg_kernel<256, 0, 2048>      up to 2,048 keys: 256 threads, 17 KB of LDS
//   heavy_seg_kernel<1024, 2048, 8192>  2,049 - 8,192 keys: 1,024 threads, 64 KB; one workgroup per
//                                       listed large segment (list: spill_segment)
// (one 512-thread class kernel with a 64 KB hash set for every segment, a bitonic kernel and a
// radix kernel, each over every segment, took 55 + 5 + 56 us at config 1).
//
// A one-k-mer segment in class order: what the compaction and the class-order expansion need is
// class runs in ascending class, each protein once per run — not its proteins ascending (only plain
// order, the ranged calls', searches by protein).  So: a counting sort by class in LDS, a protein's
// later windows dropped through an LDS hash set on p sized to the segment (vertex.rs:59-140 counts a
// protein once per k-mer), and the segment's tail (as many slots as windows dropped) filled with
// copies of its last key, which the compaction sees as duplicates of their neighbour.  O(n) with
// four barriers.  A segment whose classes reach kScClasses sorts instead.
//
// Otherwise (a whole bucket, or plain order) a sort: bitonic in LDS up to 2,048 keys; above, a
// block radix sort (rocprim, 8-bit digits) of a compacted key (k-mer slot | the varying low bits:
// 4 passes instead of 8 at config 1).
constexpr uint32_t kSegLarge = 8192, kScClasses = 256;  // (kSegSmall: group.hip)
struct NoBlockSort {
    struct storage_type {
        char c;
    };
};
template <uint32_t kThr, uint32_t kLo, uint32_t kN>
__global__ __launch_bounds__(kThr) void heavy_seg_kernel(const unsigned long long* __restrict__ spill,
                                                         uint64_t spill_cap,
                                                         const unsigned long long* __restrict__ cursor,
                                                         const unsigned long long* __restrict__ seg,
                                                         const unsigned long long* __restrict__ list, HeavyOrder ho,
                                                         unsigned long long* __restrict__ out) {
    constexpr uint32_t kItems = kN / kThr;
    constexpr bool kRadix = kN > kSegSmall;
    using Sort = std::conditional_t<kRadix, rocprim::block_radix_sort<unsigned long long, kThr, kItems>, NoBlockSort>;
    __shared__ union {
        uint32_t P[2 * kN];                // hash set of the segment's proteins
        unsigned long long K[kN];          // an LDS bitonic sort's keys
        typename Sort::storage_type st;    // the radix sort's
    } u;
    __shared__ uint32_t CH[kScClasses];  // keys per class, then each class run's start
    __shared__ uint32_t HT[kRadix ? 2 * kN : 1];  // the radix sort's k-mer slots (h per slot)
    __shared__ uint32_t wave_tot[kThr / 64];
    __shared__ uint32_t s_maxc;
    __shared__ unsigned long long s_last, s_or;
    const unsigned long long sd = seg[kLo ? list[blockIdx.x] : blockIdx.x];
    const uint32_t cnt = (uint32_t)(sd >> 40) & 0x7FFFFFu;
    if (cnt <= kLo || cnt > kN) return;
    const bool whole = sd >> 63;
    const uint32_t tid = threadIdx.x;
    const uint64_t pos = sd & ((1ull << 40) - 1), shard = pos / spill_cap;
    uint64_t dst = pos - shard * spill_cap;
    for (uint64_t t = 0; t < shard; ++t) dst += cursor[t];
    const unsigned long long cm = (1ull << ho.cb) - 1, hm = ~((1ull << ho.hshift) - 1);
    // class order: [h | p | class] -> [h | class | p]
    auto order = [&](unsigned long long x) {
        return ho.cls ? (x & hm) | (x & cm) << ho.pbits | ((x & ~hm) >> ho.cb) : x;
    };
    if (tid == 0) {
        s_maxc = 0;
        s_or = 0;
    }
    // an LDS bitonic sort of the segment's keys (v: striped, thread t holds keys t + e * kThr)
    auto bitonic = [&](const unsigned long long* v) {
        uint32_t N = 1;
        while (N < cnt) N <<= 1;
        __syncthreads();  // u is free
        for (uint32_t i = tid; i < N; i += kThr) u.K[i] = ~0ull;  // padding sorts last
        __syncthreads();
#pragma unroll
        for (uint32_t e = 0; e < kItems; ++e) {
            const uint32_t i = tid + e * kThr;
            if (i < cnt) u.K[i] = v[e];
        }
        __syncthreads();
        for (uint32_t k = 2; k <= N; k <<= 1)
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t i = tid; i < N / 2; i += kThr) {
                    const uint32_t lo = 2 * j * (i / j) + (i % j), hi = lo + j;
                    const unsigned long long x = u.K[lo], y = u.K[hi];
                    if ((x > y) == !(lo & k)) {
                        u.K[lo] = y;
                        u.K[hi] = x;
                    }
                }
                __syncthreads();
            }
        for (uint32_t i = tid; i < cnt; i += kThr) out[dst + i] = u.K[i];
    };
    unsigned long long v[kItems];
    if (whole || !ho.cls) {
        if constexpr (kRadix) {
            // The sort key, compacted: the k-mer's slot in an LDS hash table of h (a segment's k-mers
            // only need to be contiguous, in any order) above the bits of the [class | p] (or
            // [p | class]) field that vary in the segment.  At config 1 a whole bucket sorts 13 + 18
            // bits (4 passes of 8 bits) instead of the 51 below its keys' highest differing bit (7).
            // Padding (all ones) sorts after every compacted key.  Every h of a segment shares h0's
            // top bit (a bucket is a range of top bits of h), so ~h0 marks an empty slot.
            const unsigned long long k0 = order(spill[pos]);
            const unsigned long long lowm = (1ull << ho.hshift) - 1;
            const uint32_t hempty = ~(uint32_t)(k0 >> ho.hshift);
            uint32_t lg = 6;  // slots: a power of two >= 2 cnt
            while ((1u << lg) < 2 * cnt) ++lg;
            const uint32_t nsl = 1u << lg;
            for (uint32_t i = tid; i < nsl; i += kThr) HT[i] = hempty;
            unsigned long long ox = 0;
#pragma unroll
            for (uint32_t e = 0; e < kItems; ++e) {  // blocked: thread t holds keys t * kItems + e
                const uint32_t i = tid * kItems + e;
                v[e] = ~0ull;
                if (i < cnt) {
                    v[e] = order(spill[pos + i]);
                    ox |= (v[e] ^ k0) & lowm;
                }
            }
#pragma unroll
            for (int o = 32; o; o >>= 1) ox |= __shfl_xor(ox, o);
            __syncthreads();  // s_or cleared, HT filled
            if ((tid & 63) == 0 && ox) atomicOr(&s_or, ox);
            __syncthreads();
            const unsigned long long dl = s_or;
            const uint32_t lb = dl ? 64u - (uint32_t)__clzll((long long)dl) : 0u;  // varying low bits [0, lb)
            const unsigned long long lbm = (1ull << lb) - 1;
#pragma unroll
            for (uint32_t e = 0; e < kItems; ++e) {
                if (v[e] == ~0ull) continue;
                const uint32_t h = (uint32_t)(v[e] >> ho.hshift);
                uint32_t sl = (h * 0x85EBCA6Bu) >> (32 - lg);
                for (;;) {
                    const uint32_t old = atomicCAS(&HT[sl], hempty, h);
                    if (old == hempty || old == h) break;
                    sl = (sl + 1) & (nsl - 1);
                }
                v[e] = (unsigned long long)sl << lb | (v[e] & lbm);
            }
            Sort().sort(v, u.st, 0, lg + lb);  // (barriers inside: HT complete before it is read)
            const unsigned long long fixed = k0 & lowm & ~lbm;
#pragma unroll
            for (uint32_t e = 0; e < kItems; ++e) {
                const uint32_t i = tid * kItems + e;
                if (i < cnt) out[dst + i] = (unsigned long long)HT[v[e] >> lb] << ho.hshift | fixed | (v[e] & lbm);
            }
        } else {
#pragma unroll
            for (uint32_t e = 0; e < kItems; ++e) {
                const uint32_t i = tid + e * kThr;
                v[e] = i < cnt ? order(spill[pos + i]) : ~0ull;
            }
            bitonic(v);
        }
        return;
    }
    // one k-mer, class order
    const uint32_t pm = (uint32_t)((1ull << ho.pbits) - 1);
    uint32_t mc = 0;
#pragma unroll
    for (uint32_t e = 0; e < kItems; ++e) {
        const uint32_t i = tid + e * kThr;
        v[e] = ~0ull;
        if (i < cnt) {
            v[e] = order(spill[pos + i]);
            mc = max(mc, (uint32_t)(v[e] >> ho.pbits) & (uint32_t)cm);
        }
    }
    uint32_t lg = 6;  // hash slots: a power of two >= 2 cnt
    while ((1u << lg) < 2 * cnt) ++lg;
    const uint32_t nsl = 1u << lg;
    for (uint32_t i = tid; i < nsl; i += kThr) u.P[i] = 0xFFFFFFFFu;
    for (uint32_t i = tid; i < kScClasses; i += kThr) CH[i] = 0;
    __syncthreads();
    const uint32_t wm = wave_max(mc);
    if ((tid & 63) == 0) atomicMax(&s_maxc, wm);
    __syncthreads();
    const uint32_t maxc = s_maxc;
    if (maxc >= kScClasses) {  // (uniform) many classes: sort the segment
        bitonic(v);
        return;
    }
    // a protein's first window in the segment keeps its key, later ones are dropped; each kept key
    // ranked in its class
    uint32_t rk[kItems];
#pragma unroll
    for (uint32_t e = 0; e < kItems; ++e) {
        rk[e] = ~0u;
        if (v[e] == ~0ull) continue;
        const uint32_t p = (uint32_t)v[e] & pm;
        uint32_t sl = (p * 0x9E3779B1u) >> (32 - lg);
        bool first = false;
        while (true) {
            const uint32_t old = atomicCAS(&u.P[sl], 0xFFFFFFFFu, p);
            if (old == 0xFFFFFFFFu) {
                first = true;
                break;
            }
            if (old == p) break;
            sl = (sl + 1) & (nsl - 1);
        }
        if (first) rk[e] = atomicAdd(&CH[(uint32_t)(v[e] >> ho.pbits) & (uint32_t)cm], 1u);
    }
    __syncthreads();
    lds_bins_scan<kThr>(CH, maxc + 1, wave_tot);  // CH: run starts; the kept count below
    uint32_t kept = 0;
#pragma unroll
    for (uint32_t e = 0; e < kItems; ++e)
        if (rk[e] != ~0u) {
            const uint32_t at = CH[(uint32_t)(v[e] >> ho.pbits) & (uint32_t)cm] + rk[e];
            out[dst + at] = v[e];
            ++kept;
        }
    // the segment's last kept key: the largest (class, position) — the highest class run's last slot
    uint32_t D, excl;
    block_scan_n<kThr>(kept, excl, D, wave_tot);
#pragma unroll
    for (uint32_t e = 0; e < kItems; ++e)
        if (rk[e] != ~0u && CH[(uint32_t)(v[e] >> ho.pbits) & (uint32_t)cm] + rk[e] == D - 1) s_last = v[e];
    __syncthreads();
    const unsigned long long last = s_last;
    for (uint32_t i = D + tid; i < cnt; i += kThr) out[dst + i] = last;
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
    unsigned long long v[kHvPer], u[kHvPer];  // every load issued before any is used
#pragma unroll
    for (uint32_t r = 0; r < kHvPer; ++r) {
        const uint64_t i = t0 + r * kHvThreads + threadIdx.x;
        v[r] = i < m ? x[i] : 0ull;
        u[r] = i < m && i ? x[i - 1] : ~0ull;
    }
#pragma unroll
    for (uint32_t r = 0; r < kHvPer; ++r) {
        if (t0 + r * kHvThreads + threadIdx.x >= m) break;
        ne += (v[r] >> es) != (u[r] >> es);
        ng += (v[r] >> ho.hshift) != (u[r] >> ho.hshift);
        nr += (v[r] >> ho.pbits) != (u[r] >> ho.pbits);
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
                                                         unsigned long long* __restrict__ tcount,
                                                         unsigned long long* __restrict__ ng_plan) {
    const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t ng = *ng_dev;  // k-mers; threads up to the bound ngb write empty plans
    // the k-mers the expansion walks: every one, within the arrays' bound (ngb - 1 k-mers + the scan's
    // end; the host's bound holds: the clamp only keeps a broken bound from reading past them)
    if (g == 0 && ng_plan) *ng_plan = ng < ngb ? ng : ngb - 1;
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

// The passes of a fused multi-k batch without the row-block partition (tail_multi_rows, step.hip):
// every pair key of a pass comes from the row-driven expansion (a spill-all front), so the row
// blocks' sizes can be counted before any key exists.  Phase 1 counts each row's kept keys; the
// host scans them into row blocks; phase 2 writes every key straight into its row block as the
// u32 row-block key — the u64 shard keys, the histogram pass over them (pt_hist) and their
// partition (pt_scatter) are gone: 20 of the ~50 bytes of tail traffic per key at config 5.
struct RowDirect {
    int phase;            // 1: count, 2: write
    uint32_t row0;        // the call's first row
    unsigned pbits, rbits;
    uint32_t* cnt;        // phase 1: kept keys per row of the call
    uint32_t* cur;        // phase 2: each row block's cursor (its start on entry)
    uint32_t* keys;       // phase 2: the row-block keys
    uint64_t cap;         // ... their capacity
    uint32_t* rec;        // per (workgroup, wave): phase 1's kept counts by row (the class test)
    bool ran;             // set by heavy_phase when its row-driven expansion took the call
};
// records per wave (row, kept); a wave over more rows marks its first record kRecFull and the
// write phase counts that workgroup itself
constexpr uint32_t kRecPer = 8, kRecFull = 0xFFFFFFFEu;
constexpr uint32_t kHrBatch = 4;  // partner loads a lane of the counting walk issues before using them
// (the same batching of the write walk measured slower: 406 -> 478 ms at config 5, as did pt_split's)

// Both phases, heavy_flat's work split (one workgroup per 256 active elements, their candidates in
// one contiguous slice per wave).  The elements come by protein, so the threads form runs of one
// row (phase 1) or one row block (phase 2; key (p - row0) >> shift): run r owns the candidates
// [rs[r], rs[r + 1]).  Kept counts per (wave, run): without the class test the slice's overlap
// with the run; with it, counted on a first walk (each lane's count held for its current run and
// added to LDS when the run changes) in phase 1, which records them per wave by row (rec: the
// slices are the same in both phases), so phase 2 sums its row blocks' counts from the records
// instead of walking the partners a third time.  Phase 1 adds each run's count to cnt[row].  Phase 2
// reserves each run's keys on its block cursor once, gives each wave its offset inside, and
// writes: a lane's position = its wave's offset in its run + the kept lanes before it in the
// same run (ballot), the offsets advanced by the last lane of each run segment.
template <bool kWrite>
__global__ __launch_bounds__(kHfThreads) void heavy_rows_kernel(
        const uint32_t* __restrict__ E, const uint64_t* __restrict__ GS, const uint32_t* __restrict__ KG,
        const uint32_t* __restrict__ GH, const uint32_t* __restrict__ PE, uint32_t a0, uint32_t a1, unsigned cb,
        int require_diff, uint32_t heavy_df, int k, unsigned sb, uint32_t sor, RowDirect rd,
        unsigned long long* __restrict__ gstats) {
    __shared__ uint32_t s_ex[kHfThreads + 1], s_e[kHfThreads], s_x[kHfThreads], s_f[kHfThreads];
    __shared__ uint32_t s_run[kHfThreads], s_rs[kHfThreads + 1], s_rb[kHfThreads], s_rr[kHfThreads];
    __shared__ uint32_t s_wk[kHfWaves][kHfThreads];  // kept per (wave, run); phase 2: then the write offsets
    __shared__ uint32_t wave_tot[kHfWaves];
    __shared__ uint32_t s_full;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t a = a0 + blockIdx.x * kHfThreads + tid;
    const unsigned shift = kWrite ? rd.rbits : 0u;
    uint32_t cand = 0, e = 0, x = 0, f = 0, rb = ~0u;
    if (a < a1) {
        e = PE[a];
        const uint32_t g = KG[e];
        const uint64_t gs0 = GS[g], gs1 = GS[g + 1];
        x = E[e];
        if (gs1 - gs0 <= heavy_df) cand = (uint32_t)(gs1 - e - 1);
        if (kWrite) f = sb ? sor | kmer_self_score(GH[g], k) : 0u;
        rb = ((x >> cb) - rd.row0) >> shift;
    }
    uint32_t ex, total;
    block_scan_n<kHfThreads>(cand, ex, total, wave_tot);
    s_ex[tid] = ex;
    s_e[tid] = e;
    s_x[tid] = x;
    s_f[tid] = f;
    s_rb[tid] = rb;
    if (tid == 0) s_ex[kHfThreads] = total;
    __syncthreads();
    if (total == 0) return;  // (uniform)
    // runs of threads (the valid threads are a prefix, their keys ascending)
    const bool head = a < a1 && (tid == 0 || s_rb[tid - 1] != rb);
    uint32_t ri, nruns;
    block_scan_n<kHfThreads>(head ? 1u : 0u, ri, nruns, wave_tot);
    if (head) {
        s_rs[ri] = ex;
        s_rr[ri] = rb;
    }
    if (tid == 0) s_rs[nruns] = total;  // (the invalid threads' ex)
    s_run[tid] = head ? ri : ri - 1u;
    const uint32_t S = (total + kHfWaves - 1) / kHfWaves;
    const uint32_t c0 = min(total, wv * S), c1 = min(total, c0 + S);
#pragma unroll
    for (uint32_t w = 0; w < kHfWaves; ++w) s_wk[w][tid] = 0;
    if (tid == 0) s_full = 0;
    __syncthreads();
    auto search = [&](uint32_t o) {  // the last row with s_ex[i] <= o (o < total: a row with candidates)
        uint32_t lo = 0, hi = kHfThreads;
        while (lo + 1 < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_ex[mid] <= o) lo = mid;
            else hi = mid;
        }
        return lo;
    };
    const uint32_t cmask = (1u << cb) - 1;
    uint32_t* const rec = rd.rec + (uint64_t)blockIdx.x * kHfWaves * kRecPer * 2;
    bool walk = require_diff;
    if (kWrite && require_diff) {  // phase 1's records, summed by row block
        if (tid < kHfWaves * kRecPer) {
            const uint32_t row = rec[2 * tid], n = rec[2 * tid + 1];
            if (row == kRecFull) {
                s_full = 1;
            } else if (n) {
                const uint32_t b = row >> rd.rbits;
                uint32_t lo = 0, hi = nruns;  // the run of block b (present: b is one of this workgroup's)
                while (lo + 1 < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (s_rr[mid] <= b) lo = mid;
                    else hi = mid;
                }
                atomicAdd(&s_wk[tid / kRecPer][lo], n);
            }
        }
        __syncthreads();
        walk = s_full != 0;  // (uniform)
        if (walk) {
#pragma unroll
            for (uint32_t w = 0; w < kHfWaves; ++w) s_wk[w][tid] = 0;
            __syncthreads();
        }
    }
    if (walk) {  // the first walk: kept per (wave, run)
        uint32_t i = c0 + lane < c1 ? search(c0 + lane) : 0u, cr = ~0u, acc = 0;
        for (uint32_t o0 = c0 + lane; o0 < c1; o0 += 64 * kHrBatch) {  // kHrBatch partner loads in flight
            uint32_t ib[kHrBatch], xb[kHrBatch];
#pragma unroll
            for (uint32_t b = 0; b < kHrBatch; ++b) {
                const uint32_t o = o0 + 64 * b;
                ib[b] = ~0u;
                if (o < c1) {
                    while (s_ex[i + 1] <= o) ++i;
                    ib[b] = i;
                    xb[b] = E[s_e[i] + 1 + (o - s_ex[i])];
                }
            }
#pragma unroll
            for (uint32_t b = 0; b < kHrBatch; ++b) {
                if (ib[b] == ~0u) continue;
                const uint32_t r = s_run[ib[b]];
                if (r != cr) {
                    if (acc) atomicAdd(&s_wk[wv][cr], acc);
                    cr = r;
                    acc = 0;
                }
                acc += ((xb[b] ^ s_x[ib[b]]) & cmask) != 0u;
            }
        }
        if (acc) atomicAdd(&s_wk[wv][cr], acc);
    } else if (!require_diff) {  // every candidate kept: the slices' overlaps with the runs
        for (uint32_t r = tid; r < nruns; r += kHfThreads)
#pragma unroll
            for (uint32_t w = 0; w < kHfWaves; ++w) {
                const uint32_t wc0 = min(total, w * S), wc1 = min(total, wc0 + S);
                const uint32_t lo = max(wc0, s_rs[r]), hi = min(wc1, s_rs[r + 1]);
                s_wk[w][r] = hi > lo ? hi - lo : 0u;
            }
    }
    __syncthreads();
    if (!kWrite) {
        if (require_diff && tid < kHfWaves * kRecPer) {  // this workgroup's records
            const uint32_t w = tid / kRecPer, i = tid % kRecPer;
            const uint32_t wc0 = min(total, w * S), wc1 = min(total, wc0 + S);
            uint32_t row = ~0u, n = 0;
            if (wc1 > wc0) {
                const uint32_t rf = s_run[search(wc0)], rl = s_run[search(wc1 - 1)];
                if (rl - rf >= kRecPer) {
                    row = kRecFull;
                } else if (rf + i <= rl) {
                    row = s_rr[rf + i];
                    n = s_wk[w][rf + i];
                }
            }
            rec[2 * tid] = row;
            rec[2 * tid + 1] = n;
        }
        for (uint32_t r = tid; r < nruns; r += kHfThreads) {
            uint32_t t = 0;
#pragma unroll
            for (uint32_t w = 0; w < kHfWaves; ++w) t += s_wk[w][r];
            if (t) atomicAdd(&rd.cnt[s_rr[r]], t);
        }
        return;
    }
    uint32_t K = 0;
    for (uint32_t r = tid; r < nruns; r += kHfThreads) {
        uint32_t t = 0;
#pragma unroll
        for (uint32_t w = 0; w < kHfWaves; ++w) t += s_wk[w][r];
        K += t;
        uint32_t at = t ? atomicAdd(&rd.cur[s_rr[r]], t) : 0u;
#pragma unroll
        for (uint32_t w = 0; w < kHfWaves; ++w) {
            const uint32_t v = s_wk[w][r];
            s_wk[w][r] = at;
            at += v;
        }
    }
    K = wave_sum(K);
    if (lane == 0 && K) {  // the incidences written (statistics: any shard's slot)
        uint32_t hx = (blockIdx.x * 0x9E3779B1u) ^ (a0 * 0x85EBCA6Bu) ^ wv;
        hx ^= hx >> 16;
        atomicAdd(&gstats[(uint64_t)((hx * 0x7FEB352Du) >> 26) * 8 + kStInc], (unsigned long long)K);
    }
    __syncthreads();
    const uint32_t rmask = (1u << rd.rbits) - 1;
    const unsigned long long below = (1ull << lane) - 1, upto = (2ull << lane) - 1;
    uint32_t i = c0 + lane < c1 ? search(c0 + lane) : 0u;
    for (uint32_t o0 = c0; o0 < c1; o0 += 64) {  // uniform over the wave (ballots)
        const uint32_t o = o0 + lane;
        bool keep = false;
        uint32_t key = 0, r = ~0u;
        if (o < c1) {
            while (s_ex[i + 1] <= o) ++i;
            const uint32_t xj = E[s_e[i] + 1 + (o - s_ex[i])], xi = s_x[i];
            keep = !require_diff || ((xj ^ xi) & cmask) != 0u;
            key = ((((xi >> cb) - rd.row0) & rmask) << rd.pbits | (xj >> cb)) << sb | s_f[i];
            r = s_run[i];
        }
        const unsigned long long m = __ballot(keep);
        const uint32_t pr = __shfl_up(r, 1), nr = __shfl_down(r, 1);
        const unsigned long long heads = __ballot(lane == 0 || pr != r);
        const unsigned long long seg = ~((1ull << (63 - __clzll(heads & upto))) - 1);  // lanes from the run's first
        if (keep) {
            const uint64_t pos = (uint64_t)s_wk[wv][r] + __popcll(m & below & seg);
            if (pos < rd.cap) rd.keys[pos] = key;
        }
        if ((lane == 63 || nr != r) && r != ~0u) s_wk[wv][r] += __popcll(m & upto & seg);
    }
}

// per-protein index of the compacted elements of proteins [lo, hi) (the batch's row span): counts,
// then (after a scan into PO) the scatter
__global__ void heavy_pcount_kernel(const uint32_t* __restrict__ E, const unsigned long long* __restrict__ tot,
                                    unsigned cb, uint32_t lo, uint32_t hi, uint32_t* __restrict__ cnt) {
    const uint64_t ne = tot[0];
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < ne; e += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t p = E[e] >> cb;
        if (p - lo < hi - lo) atomicAdd(&cnt[p], 1u);
    }
}
__global__ void heavy_pscatter_kernel(const uint32_t* __restrict__ E, const unsigned long long* __restrict__ tot,
                                      unsigned cb, uint32_t lo, uint32_t hi, const uint32_t* __restrict__ PO,
                                      uint32_t* __restrict__ cur, uint32_t* __restrict__ PE) {
    const uint64_t ne = tot[0];
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < ne; e += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t p = E[e] >> cb;
        if (p - lo < hi - lo) PE[PO[p] + atomicAdd(&cur[p], 1u)] = (uint32_t)e;
    }
}

// bucket kernels: capacity (keys), threads, log2 of the k-mer table (>= capacity)
constexpr int kBucketSmallCap = 1280, kBucketSmallThreads = 256, kBucketSmallTab = 11;
// larger buckets (up to 4,096 keys: four per thread, no register spills) take the large kernel;
// above that the whole bucket goes to the heavy path
constexpr int kBucketLargeCap = 4096, kBucketLargeThreads = 1024, kBucketLargeTab = 12;
// the large kernel grid-strides the list of large buckets (usually empty at config 3; most
// buckets of a k = 5 batch of real proteins): four workgroups per CU (one per CU measured 8 % slower)
constexpr int kBucketLargeGrid = 1024;
constexpr uint32_t kVregTries = 3;  // learned bucket layouts in a row before the counting partition
