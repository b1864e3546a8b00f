// postings/group.hip — bucket kernels: exact k-mer groups + pair expansion (Graph::new, update_graph_edges, the class filter).
// Part of kmp_postings.hip (included there; not a translation unit of its own).

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
// kFlRange: a pair key outside the call's row blocks reached the fast tail's scatter (dropped there;
// the call fails with KMP_EINVAL instead of writing out of bounds)
enum : uint32_t { kFlBin = 0, kFlClass = 1, kFlList = 2, kFlOvf = 3, kFlBinTiles = 4, kFlCur = 5, kFlSegs = 6, kFlSegMax = 7, kFlSend = 8, kFlSegL = 9, kFlSegW = 10, kFlRange = 11, kFlN = 12 };

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
    // flags[kFlSegs], the largest in flags[kFlSegMax]; the heavy path sorts each in LDS.  2 seg_cap
    // words: the second half lists the large segments (spill_segment)
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

// descriptor: spill index (40 bits) | keys (23 bits) << 40 | whole bucket (several k-mers) << 63.
// A segment above kSegSmall keys is also listed (its index) in seg[seg_cap + j], j counted in
// flags[kFlSegL]: the heavy path's large-segment kernel runs one workgroup per listed segment only.
constexpr uint32_t kSegSmall = 2048;
__device__ __forceinline__ void spill_segment(const BucketArgs& a, uint64_t pos, uint32_t keys, bool whole) {
    const uint32_t s = atomicAdd(&a.flags[kFlSegs], 1u);
    if (s < a.seg_cap)
        a.seg[s] = pos | (unsigned long long)min(keys, 0x7FFFFFu) << 40 | (unsigned long long)whole << 63;
    atomicMax(&a.flags[kFlSegMax], keys);
    if (whole) atomicAdd(&a.flags[kFlSegW], keys);  // (with the segment count: a bound on the spill's k-mers)
    if (keys > kSegSmall) {
        const uint32_t j = atomicAdd(&a.flags[kFlSegL], 1u);
        if (j < a.seg_cap) a.seg[a.seg_cap + j] = s;
    }
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
// (Measured and removed in round 5's clean-up: laying groups of 32+ keys out in class runs so an
// element's cross-class partners are a suffix — group_expand 0.222 -> 0.238 ms at config 3, 0.443 ->
// 0.452 ms at config 1)
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
    // the k-mer split's routed output (step F): per-destination reservation bases (a table of its
    // own: every LDS array above is still read by the partner walks between the count and the write)
    __shared__ uint32_t dbase[kSplitMax];
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
    if (!small) __syncthreads();  // LDS reuse across the buckets of one workgroup (the large kernel's loop)
    const unsigned hshift = lay.hshift, cb = lay.clsbits;
    const uint32_t lmask = (1u << hshift) - 1, cmask = (1u << cb) - 1;
    const uint32_t empty = ~b << (32 - lay.bbits);  // top bits differ from every h of bucket b
    const unsigned hb = 32 - lay.bbits;             // merged: low h bits kept in a slot
    const uint32_t hm = (1u << hb) - 1;
    constexpr uint32_t kFree = 0xFFFFFFFFu;          // merged empty slot (count field never all ones)
    if (kMerge && kPer % 4 == 0) {  // 16-byte stores
        uint4* h4 = reinterpret_cast<uint4*>(H + tid * kPer);
#pragma unroll
        for (int q = 0; q < kPer / 4; ++q) h4[q] = make_uint4(kFree, kFree, kFree, kFree);
    } else {
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            if (!kMerge) T[tid * kPer + q] = empty;
            H[tid * kPer + q] = kMerge ? kFree : 0u;
        }
    }
    for (uint32_t i = tid; i < kCap / 32; i += kThreads) dupw[i] = gdupw[i] = 0;
    for (uint32_t i = tid; i <= kHeavySub; i += kThreads) SZ[i] = 0;
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
        Bl[gs + rk[e]] = xl[e];
    }
    __syncthreads();
    // D. per position: group bounds, duplicate flag (same protein earlier in the group: the same
    // p << cb | class word); a group holding one marks its start in gdupw.
    // fwd (every pair of a group): one forward walk over the partners after i does
    // both D and E's partner test — the kept partners go to cnt (a bit mask in a group of at most 33
    // keys, else their count) and an equal word j > i marks j as a duplicate (rare: the group then
    // takes E's walk over the whole group).  No separate backward duplicate scan (config 3: 62 VALU
    // instructions per wave).
    uint32_t s[kE], en[kE], cnt[kE];
    constexpr bool kMask = kThreads <= 256;  // the large kernel measured slower with it (74 -> 80 us, config 1)
    const bool fwd = !kRows;
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
        for (uint32_t j = s[e]; j < i; ++j)
            if (Bl[j] == xl[e]) {
                atomicOr(&dupw[i >> 5], 1u << (i & 31));
                atomicOr(&gdupw[s[e] >> 5], 1u << (s[e] & 31));
                anydup = 1;
                break;
            }
    }
    __syncthreads();
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
    auto mask_mode = [&](int e) { return kMask && !gd[e] && en[e] - s[e] <= (kRows ? 32u : 33u); };
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
        // (SZ is dead after step C: per-destination counts and row starts; dbase: bases)
        uint32_t* dcnt = SZ;
        uint32_t* rst = SZ + 64;
        static_assert(kHeavySub + 1 >= 64 + kSplitMax + 1, "route tables");
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

// the small kernel's occupancy floor: 8 waves per SIMD, 64 VGPRs, 8 workgroups per CU (LDS allows 8):
// group_expand 0.238 -> 0.222 ms at config 3
constexpr int kBsWaves = 8;
template <int kCap, int kThreads, int kTabBits, bool kMerge, bool kRows, bool kScore>
__global__ __launch_bounds__(kThreads, kBsWaves * 256 / kThreads) void bucket_small_kernel(BucketArgs a, uint32_t b0) {
    process_bucket<kCap, kThreads, kTabBits, kMerge, kRows, kScore>(b0 + blockIdx.x, a, true);
}

// the buckets the small kernel listed (above its capacity), a grid-stride loop over the list
template <int kCap, int kThreads, int kTabBits, bool kRows, bool kScore>
__global__ __launch_bounds__(kThreads) void bucket_large_kernel(BucketArgs a) {
    const uint32_t m = *a.list_count;
    for (uint32_t i = blockIdx.x; i < m; i += gridDim.x)
        process_bucket<kCap, kThreads, kTabBits, false, kRows, kScore>(a.list[i], a, false);
}
