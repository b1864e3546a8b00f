// postings/step.hip — host orchestration of one step: geometry, buffers, front, heavy, tail, graphs.
// Part of kmp_postings.hip (included there; not a translation unit of its own).

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
constexpr double kFtTarget = 2275;  // the fast tail's average keys per row block (see pt_geometry)
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
    // average of ~1.1-2.3K keys (kFtTarget), twice that in the first rows
    const double target = (!c.sb && ws->fast_tail) ? kFtTarget : (double)kPtCap / 2.4;
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
    // the bin sort for scored blocks only (unscored at config 3: 0.130 -> 0.387 ms)
    g->binsort = g->sbits != 0;
    return true;
}

// ws->pt: T (totals) | fcur (fast-tail cursors) | cur | lb (fast-tail look-back, u64) | block starts
// (nrb + 1) | run counts (nrb) | edge offsets (nrb + 1) | the fast reduce's look-back ticket
struct PtBufs {
    uint32_t *T, *fcur, *cur, *bst, *counts, *eoff;  // row-block totals | fast cursors | scatter cursors | starts | runs | edge offsets
    unsigned long long* lb;
    uint32_t* ticket;
};
PtBufs pt_bufs(kmp_postings* ws, const PtGeom& g, bool reserve, hipError_t* e, hipStream_t st = nullptr) {
    PtBufs b{};
    if (reserve) {
        *e = ws->pt.reserve(5 * (uint64_t)kPtMaxBlocks + 3 * (uint64_t)g.nrb + 3);
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
    b.ticket = b.eoff + g.nrb + 1;
    return b;
}

// the fast row-block tail applies: unscored keys, at most kFtRowsMax rows per block, not turned off
// for the shape
bool pt_fast(const kmp_postings* ws, const PtGeom& g) {
    return ws->fast_tail && !g.sbits && g.rbits <= 10 && (1u << g.rbits) <= kFtRowsMax && g.nrb <= kFtScBlocks;
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

// ws->small (16 words), cleared when allocated (the fast tail's largest-block accumulator starts at 0)
hipError_t small_reserve(kmp_postings* ws, hipStream_t st) {
    hipError_t e = ws->small.reserve(16);
    if (e == hipSuccess && ws->small_zero_p != ws->small.p) {
        e = hipMemsetAsync(ws->small.p, 0, 16 * sizeof(uint32_t), st);
        ws->small_zero_p = ws->small.p;
    }
    return e;
}

// A fast-tail row block passed its kFtCap-key region (kRbFast): fewer rows per block, by the largest
// block's excess, at most kFastShrinks times; a single row above kFtCap, or blocks still too large
// after that, turn the counting tail on for the shape.  (Regions learned from the blocks' exact
// counts, with the blocks above kFtCap counted in LDS bins over (row, q), were measured and removed
// in round 5: uniprot at k = 5 0.91 ms against 0.744 ms on the counting tail.)
constexpr uint32_t kFastShrinks = 2;
void fast_overflow(kmp_postings* ws, const PtGeom& g, const unsigned long long* rb) {
    const uint64_t most = rb[kRbMaxBlock];
    if (ws->fast_tries >= kFastShrinks || g.rbits == 0) {
        ws->fast_tail = false;
        return;
    }
    ++ws->fast_tries;
    const double over = (double)most / (0.8 * kFtCap);
    unsigned shrink = 1;
    while (shrink < 16 && (double)(1u << shrink) < over) ++shrink;
    ws->pt_rb_max = g.rbits > shrink ? g.rbits - shrink : 0u;
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
    PG(small_reserve(ws, st));  // [1] run count, [2] largest row block, [3] its accumulator (fast tail)
    PG(ws->inc_sorted.reserve(total));
    if (!c.expand_only) {  // an expand-only call leaves the tail (and its staging) to tail_multi
        // u32 row-block keys (pt_scatter; the fast tail's fixed regions) ...
        PG(ws->inc.reserve(pt_fast(ws, g) ? std::max<uint64_t>(total, (uint64_t)g.nrb * g.ftcap / 2) : total));
        PG(ws->uniq.reserve(total));  // ... staged p | q (u32 each)
        PG(ws->w.reserve(total));     // ... staged w
        if (c.sb) PG(ws->stg2.reserve(2 * total));  // ... staged scores | second-k weights
    }
    PG(ws->spill.reserve(ws->spill_cap * kShards));
    PG(ws->hseg.reserve(2ull * seg_capacity(ws)));  // segments | the large ones' list
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
    const BpDigits dg = bp_digits(c.lay);
    uint32_t c0, c1;
    own_bins(ws, dg, &c0, &c1);
    if (keys) {  // else: the keys grouped by bucket of the last call (front reuse)
        PG(make_keys(c.lay, st));
        if (ws->defer_clear) {  // (a key path that did not take it)
            ws->defer_clear = false;
            return KMP_EINVAL;
        }
        ws->mark(1, st);
        // (level 2 and the bucket kernels of half the bins each on two streams, forked and joined
        // with events, measured no faster in round 5: config 3 level 2 + group 0.320 ms either way,
        // config 1 0.76 ms against 0.74 ms, a G = 8 rank 0.196 against 0.175 ms)
        int rc = bucket_group(ws, ws->keys.p, c.slots, c.lay, st);  // marks 2
        if (rc != KMP_OK) return rc;
    } else {
        ws->mark(1, st);
        ws->mark(2, st);
    }
    const BucketArgs a = bucket_args(ws, c, spill);
    const uint32_t b0 = c0 * dg.nb2, nbk = (c1 - c0) * dg.nb2;  // the call's buckets
    // the large-bucket kernel loops over its list: a grid sized from the last call's list (a
    // thousand idle 1,024-thread workgroups cost ~5 us); a bucket-range share of the k-mer split
    // lists about 1/parts of them
    // (a rank of the k-mer split: about 1/parts of them, and none at all until a call lists one)
    const uint32_t lg = ws->bin_hi ? (ws->split_large ? std::max<uint32_t>(64, kBucketLargeGrid * (c1 - c0) / dg.nb1) : 0u)
                                   : ws->large_grid;
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
        const uint32_t jt = (uint32_t)(((g.flat_n ? g.flat_n : g.sc) + kFtScTile - 1) / kFtScTile);
        // (the clear leaves kFlRange, which its own workgroups may set meanwhile: reset where it is read)
        const StepClear sc = ws->tail_clear ? StepClear{ws->flags.p, kFlRange, ws->bstats.p, kGsWords, nullptr, 0} : StepClear{};
        static_assert(kFlRange + 1 == kFlN, "the range flag is the last one");
        pt_scatter_capped_kernel<<<dim3(jt, g.nshards), kFtScThreads, 0, st>>>(in, cursor, g, b.fcur, keys32, b.lb,
                                                                                b.ticket, sc, ws->flags.p);
        ws->mark(4, st);
        pt_reduce_fast_kernel<<<g.nrb, kFtThreads, 0, st>>>(keys32, b.fcur, g, b.lb, b.ticket, c.d_p, c.d_q, c.d_w,
                                                             c.cap, c.stride,
                                                             PtPack{ws->bstats.p, ws->flags.p, nullptr, ws->hrb},
                                                             ws->small.p + 1);
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

// a side stream forked from st (its work after what st has queued) and joined back
bool side_fork(kmp_postings* ws, hipStream_t st) {
    if (!ws->side && hipStreamCreateWithFlags(&ws->side, hipStreamNonBlocking) != hipSuccess) {
        ws->side = nullptr;
        return false;
    }
    for (hipEvent_t* e : {&ws->sev[0], &ws->sev[1]})
        if (!*e && hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) {
            *e = nullptr;
            return false;
        }
    return hipEventRecord(ws->sev[0], st) == hipSuccess && hipStreamWaitEvent(ws->side, ws->sev[0], 0) == hipSuccess;
}
hipError_t side_join(kmp_postings* ws, hipStream_t st) {
    hipError_t e = hipEventRecord(ws->sev[1], ws->side);
    return e == hipSuccess ? hipStreamWaitEvent(st, ws->sev[1], 0) : e;
}

__global__ void copy_u64_kernel(unsigned long long* __restrict__ dst, const unsigned long long* __restrict__ src,
                                uint32_t n) {
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
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
            // a kernel, not a device-to-device copy: the blit and the launch after it left ~15 us of
            // idle GPU at config 1
            copy_u64_kernel<<<1, kShards, 0, st>>>(ws->hcur.p, ws->bstats.p + kRbSpill, kShards);
            ws->hcur_valid = true;
        }
        const unsigned long long* spill_cursor = ws->hcur.p;
        if (ws->h_segs && ws->h_segs <= seg_capacity(ws) && ws->h_segmax <= kSegLarge &&
            ws->h_segl <= seg_capacity(ws)) {
            const uint32_t ns = (uint32_t)ws->h_segs;
            static const bool trace = getenv("KMP_TRACE") != nullptr;
            hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
            if (trace && hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone) {
                // diagnostics: the segment sizes (one k-mer / whole bucket) by power-of-two class
                std::vector<unsigned long long> sd(ns);
                if (hipMemcpyAsync(sd.data(), ws->hseg.p, ns * 8ull, hipMemcpyDeviceToHost, st) == hipSuccess &&
                    hipStreamSynchronize(st) == hipSuccess) {
                    uint64_t n[2][15] = {}, k[2][15] = {};
                    for (unsigned long long d : sd) {
                        const uint32_t cnt = (uint32_t)(d >> 40) & 0x7FFFFFu, w = (uint32_t)(d >> 63);
                        uint32_t b = 0;
                        while (b < 14 && (1u << b) < cnt) ++b;
                        ++n[w][b];
                        k[w][b] += cnt;
                    }
                    for (int w = 0; w < 2; ++w)
                        for (int b = 0; b < 15; ++b)
                            if (n[w][b])
                                fprintf(stderr, "[kmp] segs %s <=%u: %llu segments, %llu keys\n",
                                        w ? "whole" : "kmer", 1u << b, (unsigned long long)n[w][b],
                                        (unsigned long long)k[w][b]);
                }
            }
            // the listed large segments on a side stream beside the small ones: a few workgroups'
            // latency (~40 us at config 1) under the small kernel's throughput (~25 us)
            hipStream_t ls = st;
            if (ws->h_segl && side_fork(ws, st)) ls = ws->side;
            if (ws->h_segl)
                heavy_seg_kernel<1024, kSegSmall, kSegLarge><<<(uint32_t)ws->h_segl, 1024, 0, ls>>>(
                    ws->spill.p, ws->spill_cap, spill_cursor, ws->hseg.p, ws->hseg.p + seg_capacity(ws), ho,
                    ws->hsorted.p);
            heavy_seg_kernel<256, 0, kSegSmall><<<ns, 256, 0, st>>>(ws->spill.p, ws->spill_cap, spill_cursor,
                                                                    ws->hseg.p, nullptr, ho, ws->hsorted.p);
            if (ls != st) PG(side_join(ws, st));
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
    {  // an index built for a row span that does not hold this call's rows: again, for every row
        const uint32_t lo = c.ranged ? c.row_lo : 0, hi = c.ranged ? c.row_hi : c.n;
        if (ws->h_flat_ready && (lo < ws->h_span_lo || hi > ws->h_span_hi)) ws->h_flat_ready = false;
    }
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
        // the proteins it covers: the batch's row span when it holds this call's rows (a rank's
        // share skips the other ranks' elements), else every one
        const bool spanned = ws->span_hi > ws->span_lo && c.ranged && c.row_lo >= ws->span_lo &&
                             c.row_hi <= ws->span_hi;
        ws->h_span_lo = spanned ? ws->span_lo : 0;
        ws->h_span_hi = spanned ? ws->span_hi : np;
        heavy_pcount_kernel<<<grid, 256, 0, st>>>(ws->hE.p, ws->h_tot, ho.cb, ws->h_span_lo, ws->h_span_hi, ws->hPC.p);
        size_t tb = 0;
        PG(rocprim::exclusive_scan(nullptr, tb, ws->hPC.p, ws->hPO.p, 0u, (size_t)np + 1, rocprim::plus<uint32_t>(), st));
        PG(ws->tmp.reserve(std::max(tb, ws->tmp.n)));
        PG(rocprim::exclusive_scan(ws->tmp.p, tb, ws->hPC.p, ws->hPO.p, 0u, (size_t)np + 1, rocprim::plus<uint32_t>(),
                                   st));
        PG(hipMemsetAsync(ws->hPC.p, 0, ((size_t)np + 1) * sizeof(uint32_t), st));
        heavy_pscatter_kernel<<<grid, 256, 0, st>>>(ws->hE.p, ws->h_tot, ho.cb, ws->h_span_lo, ws->h_span_hi, ws->hPO.p,
                                                    ws->hPC.p, ws->hPE.p);
        PG(hipGetLastError());
        ws->hPOh.resize((size_t)np + 1);
        PG(hipMemcpyAsync(ws->hPOh.data(), ws->hPO.p, ((size_t)np + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        PG(hipStreamSynchronize(st));
        ws->h_ng = ht[1];
        ws->h_flat_ready = true;
    }
    // bound on the k-mer count (device: h_tot[1]); exact once the flat index read it back.  Else the
    // spill's segments bound it: one k-mer per heavy group, at most one per key of a whole bucket
    // (config 1: 13,050 against the 1.0 M spilled keys that sized the plan, its scan and the expansion
    // grid before: 19 + 19 + 29 us)
    const uint64_t ngb = flat ? ws->h_ng : ws->h_segs ? std::min<uint64_t>(ws->h_m, ws->h_segs + ws->h_segw) : ws->h_m;
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
                nullptr, nullptr, nullptr, nullptr, nullptr);
        const uint32_t a0 = ws->hPOh[row_lo], a1 = ws->hPOh[row_hi];
        RowDirect* rd = ws->rdir;
        if (rd) {  // tail_multi_rows: its row counts, or its keys by row block
            rd->ran = true;
            const uint32_t grid = (a1 - a0 + kHfThreads - 1) / kHfThreads;
            PG(ws->hrec.reserve((uint64_t)grid * kHfWaves * kRecPer * 2 + 1));
            RowDirect rj = *rd;  // (the records are this workspace's: phase 2 reads what phase 1 wrote)
            rj.rec = ws->hrec.p;
            if (a1 > a0 && rd->phase == 1)
                heavy_rows_kernel<false><<<grid, kHfThreads, 0, st>>>(
                        ws->hE.p, GS, ws->hKG.p, ws->hGH.p, ws->hPE.p, a0, a1, ho.cb, c.require_diff, c.heavy_df, c.k,
                        c.sb, c.sor, rj, ws->bstats.p);
            else if (a1 > a0)
                heavy_rows_kernel<true><<<grid, kHfThreads, 0, st>>>(
                        ws->hE.p, GS, ws->hKG.p, ws->hGH.p, ws->hPE.p, a0, a1, ho.cb, c.require_diff, c.heavy_df, c.k,
                        c.sb, c.sor, rj, ws->bstats.p);
        } else if (a1 > a0)
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
    // row-block tables: k-mer g's blocks at GS[g] / kHvI + g (heavy_bbase), GS <= the elements <= h_m
    const uint64_t nbb = ngb + ws->h_m / kHvI + 2;
    PG(ws->hblk.reserve(2 * nbb));
    uint32_t* BT = ws->hblk.p;
    uint32_t* BP = BT + nbb;
    heavy_plan_kernel<<<(uint32_t)((ngb + 1 + 255) / 256), 256, 0, st>>>(
        ws->hE.p, GS, ngb + 1, ws->h_tot + 1, ho, RUN, RH, ho.cls && !c.ranged ? 1 : 0, row_lo, row_hi, c.heavy_df,
        stats ? 1 : 0, 1, ws->bstats.p, ws->hgi.p, BT, BP, ws->htc.p, ws->h_tot + 3);
    size_t t2 = 0;
    PG(rocprim::exclusive_scan(nullptr, t2, ws->htc.p, ws->htoff.p, 0ull, (size_t)ngb + 1,
                               rocprim::plus<unsigned long long>(), st));
    PG(ws->tmp.reserve(std::max(t2, ws->tmp.n)));
    PG(rocprim::exclusive_scan(ws->tmp.p, t2, ws->htc.p, ws->htoff.p, 0ull, (size_t)ngb + 1,
                               rocprim::plus<unsigned long long>(), st));
    // tiles = htoff[ng] (device); the grid strides them
    const uint32_t grid = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(ngb / 4, 256), 8192);
    heavy_expand_kernel<<<grid, kHvI, 0, st>>>(ws->hE.p, GS, ws->hgi.p, BT, BP, RUN, RH, ws->htoff.p, ws->h_tot + 3,
                                               ho, 1u << bits_for(c.n), c.require_diff, c.ranged ? 1 : 0, row_lo,
                                               row_hi, ws->inc_sorted.p, ws->shard_cap, ws->bstats.p + kRbCursor,
                                               ws->bstats.p, ws->hGH.p, c.k, c.sb, c.sor);
    PG(hipGetLastError());
    return KMP_OK;
}

// A captured sequence is replayed only if it holds kernel (and event) nodes alone.  Memset nodes
// replay wrongly on this stack: round 5's captured hipMemsetAsync of the split's send buffer was
// right on the capturing launch and filled the buffer with pointer-sized values on the first replay,
// and r05aq's fault (an aperture violation in rocPRIM's onesweep on the replay of a captured
// postings front, test_frequent_kmers_heavy_path[12000]) is the same input: rocPRIM's radix sort
// issues two hipMemsetAsync per call (its digit offsets and look-back states), and the captured
// front held them.  Every fill of this library's own captured sequences is a kernel; a sequence with
// a rocPRIM sort in it (the postings entry's front) runs plain instead.
bool graph_replayable(hipGraph_t gr) {
    size_t n = 0;
    if (hipGraphGetNodes(gr, nullptr, &n) != hipSuccess) return false;
    std::vector<hipGraphNode_t> nodes(n);
    if (n && hipGraphGetNodes(gr, nodes.data(), &n) != hipSuccess) return false;
    for (hipGraphNode_t x : nodes) {
        hipGraphNodeType t;
        if (hipGraphNodeGetType(x, &t) != hipSuccess) return false;
        if (t != hipGraphNodeTypeKernel && t != hipGraphNodeTypeEventRecord && t != hipGraphNodeTypeEmpty) {
            if (getenv("KMP_DEBUG")) fprintf(stderr, "kmp: captured sequence holds a node of type %d: run plain\n", (int)t);
            return false;
        }
    }
    return true;
}

// the kernel launches of a graph, in node order: function, grid, block, shared memory
std::vector<std::vector<unsigned long long>> graph_launches(hipGraph_t gr) {
    std::vector<std::vector<unsigned long long>> out;
    size_t n = 0;
    if (hipGraphGetNodes(gr, nullptr, &n) != hipSuccess) return out;
    std::vector<hipGraphNode_t> nodes(n);
    if (n && hipGraphGetNodes(gr, nodes.data(), &n) != hipSuccess) return out;
    for (hipGraphNode_t x : nodes) {
        hipGraphNodeType t;
        if (hipGraphNodeGetType(x, &t) != hipSuccess || t != hipGraphNodeTypeKernel) continue;
        hipKernelNodeParams kp{};
        if (hipGraphKernelNodeGetParams(x, &kp) != hipSuccess) continue;
        out.push_back({(uintptr_t)kp.func, kp.gridDim.x, kp.gridDim.y, kp.gridDim.z, kp.blockDim.x, kp.blockDim.y,
                       kp.blockDim.z, kp.sharedMemBytes});
    }
    return out;
}

// KMP_GRAPH_VERIFY=1: before a replay, the sequence is captured again (not launched) and its launches —
// function, grid, block, shared memory — must equal the replayed graph's, in order: a launch input
// the graph key missed (a grid from a read-back, a capacity) fails the call loudly instead of
// replaying stale launches.  Returns false on a mismatch.
template <class Enqueue>
bool graph_verify(kmp_postings* ws, const std::vector<std::vector<unsigned long long>>& want, Enqueue& enqueue) {
    if (!ws->cst) return true;
    hipGraph_t gr = nullptr;
    if (hipStreamBeginCapture(ws->cst, hipStreamCaptureModeRelaxed) != hipSuccess) {
        (void)hipGetLastError();
        return true;
    }
    const int rc = enqueue(ws->cst);
    if (hipStreamEndCapture(ws->cst, &gr) != hipSuccess || !gr) {
        (void)hipGetLastError();
        return rc == KMP_OK;
    }
    const auto got = graph_launches(gr);
    (void)hipGraphDestroy(gr);
    if (rc == KMP_OK && got == want) return true;
    fprintf(stderr, "kmp: graph replay check failed: %zu launches captured now, %zu in the replayed graph\n",
            got.size(), want.size());
    for (size_t i = 0; i < std::max(got.size(), want.size()); ++i)
        if (i >= got.size() || i >= want.size() || got[i] != want[i])
            fprintf(stderr, "kmp:   launch %zu: now grid %llu x %llu block %llu, graph grid %llu x %llu block %llu\n", i,
                    i < got.size() ? got[i][1] : 0ull, i < got.size() ? got[i][2] : 0ull,
                    i < got.size() ? got[i][4] : 0ull, i < want.size() ? want[i][1] : 0ull,
                    i < want.size() ? want[i][2] : 0ull, i < want.size() ? want[i][4] : 0ull);
    return false;
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
    static const bool trace = getenv("KMP_TRACE") != nullptr;
    if (trace)
        fprintf(stderr, "kmp-trace: slot %p key[0..2] %llu %llu %llu gen %llu: %s\n", (void*)&slot, key[0],
                key.size() > 1 ? key[1] : 0ull, key.size() > 2 ? key[2] : 0ull, key.back(),
                !ws->graph_on ? "plain (graphs off)"
                : (slot.gexec && slot.key == key) ? "replay"
                : slot.seen != key                ? "plain (first)"
                                                  : "capture");
    if (!ws->graph_on) return enqueue(st);
    if (slot.gexec && slot.key == key) {
        if (getenv("KMP_GRAPH_VERIFY") && !graph_verify(ws, slot.launches, enqueue)) return KMP_EDEVICE;
        PG(hipGraphLaunch(slot.gexec, st));
        ++ws->graph_replays;
        return KMP_OK;
    }
    if (slot.seen != key || slot.plain == key) {  // (plain: its capture held a node that does not replay)
        slot.seen = key;
        return enqueue(st);
    }
    if (slot.gexec) (void)hipGraphExecDestroy(slot.gexec);
    slot.gexec = nullptr;
    slot.key.clear();
    slot.launches.clear();
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
    const bool ok = rc == KMP_OK && e == hipSuccess && gr && gen == g_grow_gen.load();
    if (ok && graph_replayable(gr)) {
        slot.launches = graph_launches(gr);
        e = hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0);
    } else {
        if (ok) slot.plain = key;
        if (e == hipSuccess) e = hipErrorUnknown;
    }
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
    if (ws->async_slot >= 0) {
        // a submission: its slot's graph (the key holds the slot's read-back, so the two slots'
        // graphs differ); replayed without a host wait when it matches, else plain or captured and
        // finished synchronously by the caller
        kmp_postings::GraphSlot& gs = ws->fg[ws->async_slot];
        std::vector<unsigned long long> kg = key;
        kg.push_back((uintptr_t)ws->hrb);
        std::vector<unsigned long long> kr = kg;
        kr.push_back(g_grow_gen.load());  // (slot_launch's own last word)
        if (ws->graph_on && gs.gexec && gs.key == kr) {
            if (getenv("KMP_GRAPH_VERIFY") && !graph_verify(ws, gs.launches, enqueue)) return KMP_EDEVICE;
            PG(hipGraphLaunch(gs.gexec, st));
            ++ws->graph_replays;
            PG(hipEventRecord(ws->done_ev[ws->async_slot], st));
            ws->async_launched = true;
            ws->async_geom = g;
            return KMP_OK;
        }
        // a shape that already finished clean (ok_key, either slot or a synchronous call) is captured
        // on the slot's first use, so both slots replay from the third submission of a shape on
        if (ws->ok_key == key) gs.seen = kr;
        return slot_launch(ws, gs, kg, enqueue, st);
    }
    if (!ws->graph_on) return enqueue(st);
    if (ws->gexec && ws->gkey == key) {
        if (getenv("KMP_GRAPH_VERIFY") && !graph_verify(ws, ws->glaunches, enqueue)) return KMP_EDEVICE;
        PG(hipGraphLaunch(ws->gexec, st));
        ++ws->graph_replays;
        return KMP_OK;
    }
    if (ws->gkey_seen != key || ws->gkey_plain == key) {  // (plain: its capture held a node that does not replay)
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
    const bool ok = rc == KMP_OK && e == hipSuccess && gr && gen == g_grow_gen.load();
    if (ok && !graph_replayable(gr)) {  // this sequence runs plain (the workspace keeps its graphs)
        (void)hipGraphDestroy(gr);
        ws->gkey_plain = key;
        return enqueue(st);
    }
    if (ok) {
        ws->glaunches = graph_launches(gr);
        e = hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0);
    } else if (e == hipSuccess) {
        e = hipErrorUnknown;
    }
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

// The fused step's read-back asks for nothing more: no fallback, rerun, learned capacity, overflow
// finish or error (then fused_finish completes the call; a submission checks this at its wait)
bool fused_clean(const kmp_postings* ws, const PtGeom& g, const unsigned long long* rb) {
    unsigned long long acc[kStN], most, n_inc, spill_most, spill_total;
    sum_stats(rb, acc, &most, &n_inc, &spill_most, &spill_total);
    return !rb[kRbFlagClass] && !(rb[kRbList] && ws->large_used == 0) && !(rb[kRbFlagCur] && ws->cur_used) &&
           !rb[kRbFlagBin] && spill_most <= ws->spill_cap && !spill_total && most <= ws->shard_cap && !rb[kRbFast] &&
           !rb[kRbRange] && !(rb[kRbOvf] && !pt_rowhist_ok(g));
}

// a clean fused step (fused_clean): what it teaches the next call, its statistics and edge count
int fused_finish(kmp_postings* ws, const StepCfg& c, const PtGeom& g, const unsigned long long* rb, uint64_t* n_edges,
                 kmp_postings_stats* stats) {
    unsigned long long acc[kStN], most, n_inc, spill_most, spill_total;
    sum_stats(rb, acc, &most, &n_inc, &spill_most, &spill_total);
    ws->pt_inc = n_inc;  // sizes the next call's row blocks
    ws->last_fast = pt_fast(ws, g);
    ws->vreg_tries = 0;  // a call without a region overflow
    {  // the large-bucket grid of the next call: twice the listed buckets, 64 .. kBucketLargeGrid;
       // none listed: not launched (an idle 64-workgroup launch cost ~5 us of the config-3 step)
        uint32_t lg = rb[kRbList] ? 64u : 0u;
        while (lg && lg < kBucketLargeGrid && lg < 2 * rb[kRbList]) lg *= 2;
        ws->large_grid = lg;
    }
    const uint64_t ne = rb[kRbRuns];
    ws->last_ovf = (uint32_t)rb[kRbOvf];
    ws->shard_cap = most + most / 64 + 256;  // learned for the next call
    fill_stats(stats, acc);
    if (stats) {
        stats->incidences = n_inc;
        stats->pairs = ne;
    }
    ws->last_heavy = ws->heavy_ready;
    ws->last_fused = true;
    if (c.front_key) {
        ws->front_ok = true;
        ws->front_key = *c.front_key;
    }
    *n_edges = ne;
    return ne > c.cap ? KMP_EOVERFLOW : KMP_OK;
}

// KMP_HOSTPROF=1 (diagnostic): host time of the fused step's phases, averaged over 50 calls on stderr
struct HostProf {
    bool on = getenv("KMP_HOSTPROF") != nullptr;
    std::chrono::steady_clock::time_point t[5];
    double acc[4] = {0, 0, 0, 0};
    int n = 0;
    void mark(int i) {
        if (on) t[i] = std::chrono::steady_clock::now();
    }
    void done() {
        if (!on) return;
        for (int i = 0; i < 4; ++i) acc[i] += std::chrono::duration<double, std::micro>(t[i + 1] - t[i]).count();
        if (++n == 50) {
            fprintf(stderr, "kmp-hostprof: us per call: prep %.1f launch %.1f sync %.1f finish %.1f\n", acc[0] / n,
                    acc[1] / n, acc[2] / n, acc[3] / n);
            n = 0;
            for (double& a : acc) a = 0;
        }
    }
};
HostProf g_hprof;

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
        ws->fast_tries = 0;
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
        if (attempt) ++ws->reruns;
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
            key.push_back(ws->bp_J_min);  // (the counting level 2's tile budget, learned from a bin overflow)
            g_hprof.mark(1);
            ws->cur_key = key;
            int rc = fused_launch(ws, make_keys, key, c, g, st);
            g_hprof.mark(2);
            key.resize(key.size() - 10);
            if (rc != KMP_OK) return rc;
            if (ws->async_launched) return KMP_OK;  // a submission in flight: kmp_postings_wait checks it
            PG(hipStreamSynchronize(st));
            g_hprof.mark(3);
        } else {
            // (the split step's front as a graph of its own measured no faster at config 1: 0.624-0.629
            // ms against 0.618 with plain launches, tools/front_probe.py; it runs plain)
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
                    ws->h_segl = rb[kRbSegL];
                    ws->h_segw = rb[kRbSegW];
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
                // (the row-count path: no shard keys, its expansion counts what it wrote)
                *c.n_inc_out = ws->rdir ? acc[kStInc] : n_inc;
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
        if (!split && !rerun && fused_clean(ws, g, rb)) {
            ws->ok_key = ws->cur_key;
            return fused_finish(ws, c, g, rb, n_edges, stats);
        }
        if (rb[kRbFast]) {  // a fast-tail row block passed its region: fewer rows per block, or the counting tail
            if (debug)
                fprintf(stderr, "kmp: fast tail region overflow (rows per block %u, largest block %llu, try %u)\n",
                        1u << g.rbits, rb[kRbMaxBlock], ws->fast_tries);
            fast_overflow(ws, g, rb);
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
        if (rb[kRbRange]) {  // a pair key outside the call's rows (a device fault upstream)
            PG(hipMemsetAsync(ws->flags.p + kFlRange, 0, sizeof(uint32_t), st));
            PG(hipStreamSynchronize(st));
            return KMP_EDEVICE;
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

int tail_multi_cut(kmp_postings* const* ws, uint32_t nk, const StepCfg& c, const PtGeom& g, uint64_t T,
                   uint64_t total, const PtBufs& b, const std::vector<uint32_t>& hb, bool learn_shards,
                   uint64_t* n_edges, kmp_postings_stats* stats, hipStream_t st);

// the fused tail's geometry and buffers for T keys: *g, *total (the staging capacity), *b
int tail_multi_prep(kmp_postings* const* ws, uint32_t nk, const StepCfg& c, uint64_t T, PtGeom* g, uint64_t* total,
                    PtBufs* b, hipStream_t st) {
    kmp_postings* w0 = ws[0];
    if (!pt_geometry(w0, c, std::max<uint64_t>(T, 1), g)) return KMP_EINVAL;
    // staging capacity: every key of the pass (the row-block positions); a stream's planned pass
    // size at least, so the staging arrays are allocated once, not regrown as the passes vary
    *total = T + 1;
    for (uint32_t j = 0; j < nk; ++j) *total = std::max<uint64_t>(*total, ws[j]->stage_floor);
    PG(w0->inc.reserve(*total / 2 + 1));  // u32 keys in a u64 buffer
    if (!w0->direct_tail) {  // staged runs (the direct reduce writes the edges in place)
        PG(w0->uniq.reserve(*total));
        PG(w0->w.reserve(*total));
        PG(w0->stg2.reserve(2 * *total));
    }
    PG(w0->ovf.reserve((uint64_t)g->nrb + 1));
    PG(small_reserve(w0, st));
    hipError_t e = hipSuccess;
    *b = pt_bufs(w0, *g, true, &e, st);
    PG(e);
    PG(hipMemsetAsync(w0->flags.p + kFlOvf, 0, sizeof(uint32_t), st));
    return KMP_OK;
}

int tail_multi(kmp_postings* const* ws, uint32_t nk, const StepCfg& c, const uint64_t* inc, uint64_t* n_edges,
               kmp_postings_stats* stats, hipStream_t st) {
    kmp_postings* w0 = ws[0];
    uint64_t T = 0;
    for (uint32_t j = 0; j < nk; ++j) T += inc[j];
    PtGeom g;
    uint64_t total = 0;
    PtBufs b{};
    if (int rc = tail_multi_prep(ws, nk, c, T, &g, &total, &b, st)) return rc;
    uint32_t* keys32 = reinterpret_cast<uint32_t*>(w0->inc.p);
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
    std::vector<uint32_t> hb(g.nrb + 1);
    PG(hipMemcpyAsync(hb.data(), b.bst, (g.nrb + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    PG(hipStreamSynchronize(st));
    return tail_multi_cut(ws, nk, c, g, T, total, b, hb, true, n_edges, stats, st);
}

// tail_multi after the partition: the row blocks' keys in w0->inc at their starts hb (host copy;
// b.bst on the device) -> sub-blocks (a block above kPtCap cut into pieces the LDS reduce takes),
// the reduce and the edges.  learn_shards: size the inputs' next shard regions from this call's.
int tail_multi_cut(kmp_postings* const* ws, uint32_t nk, const StepCfg& c, const PtGeom& g, uint64_t T,
                   uint64_t total, const PtBufs& b, const std::vector<uint32_t>& hb, bool learn_shards,
                   uint64_t* n_edges, kmp_postings_stats* stats, hipStream_t st) {
    kmp_postings* w0 = ws[0];
    uint32_t* keys32 = reinterpret_cast<uint32_t*>(w0->inc.p);
    uint32_t* stage_p = reinterpret_cast<uint32_t*>(w0->uniq.p);
    uint32_t* stage_q = stage_p + total;
    const bool direct = w0->direct_tail != 0;
    std::vector<uint32_t> hd(g.nrb + 1);
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
        if (learn_shards)
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
    if (learn_shards)
        for (uint32_t j = 0; j < nk; ++j) ws[j]->shard_cap = ws[j]->last_most + ws[j]->last_most / 4 + 256;
    w0->pt_inc = T;
    if (stats) {
        stats->incidences = T;
        stats->pairs = ne;
    }
    *n_edges = ne;
    return ne > c.cap ? KMP_EOVERFLOW : KMP_OK;
}

// The fused passes' row-count path (heavy_rowcount / heavy_flat_rows, heavy.hip): expand(j, rd)
// runs input j's expand-only call with ws[j]->rdir = rd.  Phase 1 counts each row's keys, the
// host scans them into row blocks (the geometry from their exact total), phase 2 writes the keys
// into their blocks and tail_multi_cut reduces them: no shard keys, no pt_hist / pt_tscan /
// pt_scatter.  *taken false: a call the path does not cover (a front that left pair keys in its
// shard regions, an expansion that is not row-driven): nothing of the tail ran, and the caller
// takes the partition path (expand, tail_multi).
template <class Expand>
int tail_multi_rows(kmp_postings* const* ws, uint32_t nk, const StepCfg& c, Expand&& expand, uint64_t* inc,
                    bool* taken, uint64_t* n_edges, kmp_postings_stats* stats, hipStream_t st) {
    kmp_postings* w0 = ws[0];
    *taken = false;
    const uint32_t rows = c.row_hi - c.row_lo;
    PG(w0->rcnt.reserve((uint64_t)rows + 1));
    PG(hipMemsetAsync(w0->rcnt.p, 0, (size_t)rows * sizeof(uint32_t), st));
    RowDirect rd{};
    rd.phase = 1;
    rd.row0 = c.row_lo;
    rd.cnt = w0->rcnt.p;
    for (uint32_t j = 0; j < nk; ++j) {
        rd.ran = false;
        if (int rc = expand(j, &rd)) return rc;
        if (!rd.ran || ws[j]->last_most) return KMP_OK;  // keys outside the row-driven expansion
    }
    std::vector<uint32_t> hc(rows);
    PG(hipMemcpyAsync(hc.data(), w0->rcnt.p, (size_t)rows * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    PG(hipStreamSynchronize(st));
    uint64_t T = 0;
    for (uint32_t v : hc) T += v;
    if (T >= 0xFFFFFFFFull) return KMP_OK;  // (u32 key positions: the partition path reports it)
    PtGeom g;
    uint64_t total = 0;
    PtBufs b{};
    if (int rc = tail_multi_prep(ws, nk, c, T, &g, &total, &b, st)) return rc;
    std::vector<uint32_t> hb(g.nrb + 1, 0);
    {
        uint64_t at = 0;
        for (uint32_t r = 0; r < g.nrb; ++r) {
            hb[r] = (uint32_t)at;
            const uint64_t r0 = (uint64_t)r << g.rbits, r1 = std::min<uint64_t>(rows, (uint64_t)(r + 1) << g.rbits);
            for (uint64_t i = r0; i < r1; ++i) at += hc[i];
        }
        hb[g.nrb] = (uint32_t)at;
    }
    PG(hipMemcpyAsync(b.bst, hb.data(), (g.nrb + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, st));
    PG(hipMemcpyAsync(b.cur, hb.data(), g.nrb * sizeof(uint32_t), hipMemcpyHostToDevice, st));
    rd.phase = 2;
    rd.pbits = g.pbits;
    rd.rbits = g.rbits;
    rd.cur = b.cur;
    rd.keys = reinterpret_cast<uint32_t*>(w0->inc.p);
    rd.cap = total;
    uint64_t got = 0;
    for (uint32_t j = 0; j < nk; ++j) {
        rd.ran = false;
        if (int rc = expand(j, &rd)) return rc;
        if (!rd.ran || ws[j]->last_most) {  // (phase 1 took this front)
            if (getenv("KMP_DEBUG"))
                fprintf(stderr, "kmp: row-count path, input %u: expansion %d, shard keys %llu\n", j, (int)rd.ran,
                        (unsigned long long)ws[j]->last_most);
            return KMP_EDEVICE;
        }
        got += inc[j];
    }
    if (got != T) {  // the writes disagree with the counts
        if (getenv("KMP_DEBUG"))
            fprintf(stderr, "kmp: row-count path wrote %llu keys, counted %llu\n", (unsigned long long)got,
                    (unsigned long long)T);
        return KMP_EDEVICE;
    }
    *taken = true;
    return tail_multi_cut(ws, nk, c, g, T, total, b, hb, false, n_edges, stats, st);
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
    PG(small_reserve(ws, st));
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
    if (!ws->timing || !stats || ws->async_launched) return;
    (void)hipStreamSynchronize(st);
    for (int s = 0; s < KMP_POSTINGS_STAGES; ++s) {
        float ms = 0.f;
        stats->stage_ms[s] = hipEventElapsedTime(&ms, ws->evp[s], ws->evp[s + 1]) == hipSuccess ? ms : -1.f;
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
    g_hprof.mark(0);
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
            g_hprof.mark(4);
            if (rc == KMP_OK && ws->last_fused && !ws->async_launched) g_hprof.done();
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
