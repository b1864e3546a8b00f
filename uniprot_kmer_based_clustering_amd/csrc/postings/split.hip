// postings/split.hip — the multi-GPU k-mer split's device kernels.
// Part of kmp_postings.hip (included there; not a translation unit of its own).

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
// kShards x the fullest sub-region, so a grown cap gives every sub-region its need.  kcur (the sharded
// start): the keys phase's send cursors (nkc) and its flags (kFlN words after them) on this rank —
// MAX_KEYS = the region size that fits every sub-region (the cursors count every piece, dropped or
// not), RERUN when a piece was dropped — read and reset for the next keys phase.  A listed bucket
// with no large-bucket launch raises LARGE (and RERUN).
__global__ void split_pad_finish_kernel(unsigned long long* __restrict__ send, uint64_t cap,
                                        const unsigned long long* __restrict__ dcursor,
                                        const unsigned long long* __restrict__ gstats,
                                        const uint32_t* __restrict__ wflags, uint64_t sc, uint32_t parts,
                                        uint32_t* __restrict__ out, unsigned long long* __restrict__ stats,
                                        int heavy_done, int routed, int merge, uint32_t* __restrict__ kcur,
                                        uint32_t nkc, uint64_t tb, int large_launched) {
    const uint32_t d = blockIdx.y;
    if (!routed)
        for (uint64_t i = dcursor[d] + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap;
             i += (uint64_t)gridDim.x * blockDim.x)
            send[d * cap + i] = kNoKey;
    if (blockIdx.x || blockIdx.y) return;
    // one workgroup: the statistics and the fullest regions reduced over its threads (one thread
    // walking the parts x kShards cursors took 45 us at G = 8)
    const uint32_t t = threadIdx.x;
    __shared__ unsigned long long s_red[4][256 / 64];
    static_assert(kShards == 64 && kStN <= 8, "one wave per pair of statistics, a lane per shard");
    {
        // wave w (of 4) sums statistics w and w + 4 over the 64 shards (a lane per shard): every load
        // in flight at once (one thread walking the shards serialised 64 dependent loads)
        const uint32_t w = t >> 6, sh = t & 63;
#pragma unroll
        for (uint32_t j = 0; j < 2; ++j) {
            const uint32_t st = w + 4 * j;
            if (st >= kStN) continue;  // (uniform per wave)
            unsigned long long v = gstats[sh * 8 + st];
            for (int off = 32; off > 0; off >>= 1) {
                const unsigned long long o = (unsigned long long)__shfl_xor(v, off);
                v = st == kStMaxDf ? max(v, o) : v + o;
            }
            if (sh == 0) stats[st] = v;
        }
    }
    unsigned long long shard = 0, spill = 0, part = 0;
    for (uint32_t sh = t; sh < kShards; sh += blockDim.x) {
        shard = max(shard, gstats[kRbCursor + sh]);
        spill += gstats[kRbSpill + sh];
    }
    const uint32_t nq = routed ? parts * kShards : parts;
    for (uint32_t q = t; q < nq; q += blockDim.x) part = max(part, dcursor[q] * (routed ? kShards : 1u));
    unsigned long long kmax = 0;
    if (kcur)
        for (uint32_t q = t; q < nkc; q += blockDim.x) kmax = max(kmax, (unsigned long long)kcur[q]);
    for (int off = 32; off > 0; off >>= 1) {
        shard = max(shard, (unsigned long long)__shfl_xor(shard, off));
        spill += (unsigned long long)__shfl_xor(spill, off);
        part = max(part, (unsigned long long)__shfl_xor(part, off));
        kmax = max(kmax, (unsigned long long)__shfl_xor(kmax, off));
    }
    if ((t & 63) == 0) {
        s_red[0][t >> 6] = shard;
        s_red[1][t >> 6] = spill;
        s_red[2][t >> 6] = part;
        s_red[3][t >> 6] = kmax;
    }
    __syncthreads();
    if (t == 0) {
        shard = spill = part = kmax = 0;
        for (uint32_t w = 0; w < (blockDim.x + 63) / 64; ++w) {
            shard = max(shard, s_red[0][w]);
            spill += s_red[1][w];
            part = max(part, s_red[2][w]);
            kmax = max(kmax, s_red[3][w]);
        }
        const uint32_t clamp = 0xFFFFFFFFu;
        const uint32_t* kfl = kcur ? kcur + nkc : nullptr;  // the keys phase's flags
        const uint32_t k_rerun = kfl ? kfl[kFlSend] : 0u, k_class = kfl ? kfl[kFlClass] : 0u;
        const uint32_t k_keys = kcur ? (uint32_t)min<unsigned long long>(tb + kSendShards * kmax, clamp) : 0u;
        const uint32_t large = !large_launched && wflags[kFlList] ? 1u : 0u;
        out[KMP_SPLIT_CLASS] = wflags[kFlClass] | k_class;
        out[KMP_SPLIT_HEAVY] = spill != 0 && !heavy_done;  // spilled with the heavy path off: rerun with it on
        out[KMP_SPLIT_MAX_PART] = (uint32_t)min<unsigned long long>(part, clamp);
        out[KMP_SPLIT_MAX_SHARD] = (uint32_t)min<unsigned long long>(shard, clamp);
        out[KMP_SPLIT_BIN_TILES] = wflags[kFlBin] ? wflags[kFlBinTiles] : 0u;
        out[KMP_SPLIT_CURSOR] = wflags[kFlCur];
        out[KMP_SPLIT_RERUN] =
            (part > cap || shard > sc || wflags[kFlBin] || wflags[kFlCur] || wflags[kFlSend] || k_rerun || large) ? 1u
                                                                                                              : 0u;
        for (uint32_t i = KMP_SPLIT_CURSOR + 1; i < KMP_SPLIT_FLAGS; ++i) out[i] = 0;
        out[KMP_SPLIT_MAX_KEYS] = k_keys;
        out[KMP_SPLIT_LARGE] = large;
    }
    if (kcur) {  // read above (the reduction's barrier): cleared for the next keys phase
        __syncthreads();
        for (uint32_t q = t; q < nkc + kFlN; q += blockDim.x) kcur[q] = 0;
    }
}

