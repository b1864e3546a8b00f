// postings/api.hip — the extern "C" entry points of the postings engine (include/kmerpair.h).
// Part of kmp_postings.hip (included there; not a translation unit of its own).

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

int kmp_postings_set_row_span(kmp_postings* ws, uint32_t lo, uint32_t hi) {
    if (!ws || lo > hi) return KMP_EINVAL;
    ws->span_lo = lo;
    ws->span_hi = hi;
    return KMP_OK;
}

int kmp_postings_set_direct(kmp_postings* ws, int enable) {
    if (!ws) return KMP_EINVAL;
    ws->direct_tail = enable ? 1 : 0;
    return KMP_OK;
}

int kmp_postings_set_tail(kmp_postings* ws, int mode) {
    if (!ws || (mode != KMP_TAIL_FAST && mode != KMP_TAIL_COUNT)) return KMP_EINVAL;
    ws->fast_mode = mode != KMP_TAIL_COUNT;
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
uint64_t kmp_postings_reruns(const kmp_postings* ws) { return ws ? ws->reruns : 0; }

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

}  // extern "C"

// pipelined submissions (kmp_dev_pairs_residues_submit / kmp_postings_wait), held in ws->async
struct AsyncSub {
    bool used = false, launched = false;  // launched: in flight without a host wait (else finished at submit)
    uint64_t ticket = 0;
    int rc = KMP_OK;
    uint64_t n_edges = 0;
    kmp_postings_stats stats{};
    const uint8_t* d_res = nullptr;
    const uint64_t* d_res_off = nullptr;
    const uint16_t* d_class = nullptr;
    uint32_t n = 0;
    int k = 0;
    uint64_t slots = 0;
    uint32_t heavy_df = 0, min_shared = 0;
    int require_class_diff = 0;
    uint32_t *d_p = nullptr, *d_q = nullptr, *d_w = nullptr;
    uint64_t cap = 0;
    void* stream = nullptr;
    PtGeom g{};
};
struct AsyncState {
    AsyncSub sub[2];
    uint64_t next = 1;
};

extern "C" {

int kmp_dev_pairs_residues_submit(kmp_postings* ws, const uint8_t* d_res, const uint64_t* d_res_off,
                                  const uint16_t* d_class, uint32_t n, int k, uint64_t slots, uint32_t heavy_df,
                                  uint32_t min_shared, int require_class_diff, uint32_t* d_p, uint32_t* d_q,
                                  uint32_t* d_w, uint64_t cap, void* stream, uint64_t* ticket) {
    if (!ws || !ticket) return KMP_EINVAL;
    if (!ws->async) ws->async = std::make_shared<AsyncState>();
    auto* as = static_cast<AsyncState*>(ws->async.get());
    const int s = !as->sub[0].used ? 0 : !as->sub[1].used ? 1 : -1;
    if (s < 0) return KMP_ESTATE;  // two outstanding: wait for one first
    if (!ws->hrb_slot[s])
        PG(hipHostMalloc((void**)&ws->hrb_slot[s], kRbWords * sizeof(unsigned long long), hipHostMallocCoherent));
    if (!ws->done_ev[s]) PG(hipEventCreateWithFlags(&ws->done_ev[s], hipEventDisableTiming));
    if (ws->timing)
        for (auto& e : ws->evs[s])
            if (!e) PG(hipEventCreate(&e));
    AsyncSub& a = as->sub[s];
    a = AsyncSub{};
    a.d_res = d_res, a.d_res_off = d_res_off, a.d_class = d_class, a.n = n, a.k = k, a.slots = slots;
    a.heavy_df = heavy_df, a.min_shared = min_shared, a.require_class_diff = require_class_diff;
    a.d_p = d_p, a.d_q = d_q, a.d_w = d_w, a.cap = cap, a.stream = stream;
    // the call on the slot's read-back and stage events; its step graph is the slot's own
    unsigned long long* const rb_sync = ws->hrb;
    ws->hrb = ws->hrb_slot[s];
    ws->evp = ws->evs[s];
    ws->async_slot = s;
    ws->async_launched = false;
    a.rc = residues_impl(ws, d_res, d_res_off, d_class, n, k, slots, heavy_df, min_shared, require_class_diff, false, 0,
                         n, d_p, d_q, d_w, cap, &a.n_edges, &a.stats, stream);
    a.launched = ws->async_launched;
    a.g = ws->async_geom;
    ws->hrb = rb_sync;
    ws->evp = ws->ev;
    ws->async_slot = -1;
    ws->async_launched = false;
    if (!a.launched && a.rc != KMP_OK && a.rc != KMP_EOVERFLOW) return a.rc;  // (the slot stays free)
    a.used = true;
    a.ticket = as->next++;
    *ticket = a.ticket;
    return KMP_OK;
}

int kmp_postings_wait(kmp_postings* ws, uint64_t ticket, uint64_t* n_edges, kmp_postings_stats* stats) {
    if (!ws || !n_edges || !ws->async) return KMP_EINVAL;
    auto* as = static_cast<AsyncState*>(ws->async.get());
    int s = -1;
    for (int i = 0; i < 2; ++i)
        if (as->sub[i].used && as->sub[i].ticket == ticket) s = i;
    if (s < 0) return KMP_EINVAL;
    AsyncSub& a = as->sub[s];
    a.used = false;
    if (!a.launched) {  // finished at submit
        *n_edges = a.n_edges;
        if (stats) *stats = a.stats;
        return a.rc;
    }
    PG(hipEventSynchronize(ws->done_ev[s]));
    const unsigned long long* rb = ws->hrb_slot[s];
    if (!fused_clean(ws, a.g, rb)) {
        // the read-back asks for more (a rerun with a grown capacity, a fallback): the stream
        // drained (the other submission too, so nothing in flight uses a buffer that may grow),
        // then this step again, synchronously
        PG(hipStreamSynchronize(as_stream(a.stream)));
        return residues_impl(ws, a.d_res, a.d_res_off, a.d_class, a.n, a.k, a.slots, a.heavy_df, a.min_shared,
                             a.require_class_diff, false, 0, a.n, a.d_p, a.d_q, a.d_w, a.cap, n_edges, stats, a.stream);
    }
    if (stats) *stats = kmp_postings_stats{};
    // the call's configuration as run_postings built it (what fused_finish reads: cap, the front key)
    const uint32_t hd = std::max(2u, a.heavy_df);
    const std::vector<unsigned long long> front_key = {a.n, (unsigned long long)a.k, a.slots, hd,
                                                       (unsigned long long)a.require_class_diff, 1,
                                                       (uintptr_t)a.d_res, (uintptr_t)a.d_res_off, (uintptr_t)a.d_class};
    StepCfg c{};
    c.n = a.n;
    c.slots = a.slots;
    c.cap = a.cap;
    c.front_key = &front_key;
    const int rc = fused_finish(ws, c, a.g, rb, n_edges, stats);
    ws->last_bucketed = true;
    if (ws->timing && stats)
        for (int i = 0; i < KMP_POSTINGS_STAGES; ++i) {
            float ms = 0.f;
            stats->stage_ms[i] = hipEventElapsedTime(&ms, ws->evs[s][i], ws->evs[s][i + 1]) == hipSuccess ? ms : -1.f;
        }
    (void)hipGetLastError();
    return rc;
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
    // expand only: every incidence keyed (pair << 8) | j << 7 | s(x); rd: the row-count path's
    // phase (the front's statistics from the call that computes it: phase 1 or the partition path)
    auto expand = [&](uint32_t j, RowDirect* rd) -> int {
        uint64_t unused = 0;
        ws[j]->rdir = rd;
        const bool front = !rd || rd->phase == 1;
        const int rc = residues_impl(ws[j], d_res, d_res_off, d_class, n, ks[j], slots, 0xFFFFFFFFu, 1,
                                     require_class_diff, ranged, row_lo, row_hi, d_p, d_q, d_w, cap, &unused,
                                     j == 0 && front ? &s0 : nullptr, stream, kScoreBits + 1, j << kScoreBits, d_score,
                                     d_w1, &inc[j]);
        ws[j]->rdir = nullptr;
        if (rc == KMP_OK && timed && (!rd || rd->phase == 2)) PG(hipEventRecord(ws[0]->mev[1 + j], st));
        return rc;
    };
    // the passes of a batch (a row range, the in-place reduce): the row-count path
    int rc = KMP_OK;
    bool taken = false;
    if (ranged && ws[0]->direct_tail)
        rc = tail_multi_rows(ws, nk, c, expand, inc, &taken, n_edges, stats, st);
    if (rc == KMP_OK && !taken) {
        for (uint32_t j = 0; j < nk && rc == KMP_OK; ++j) rc = expand(j, nullptr);
        if (rc == KMP_OK) rc = tail_multi(ws, nk, c, inc, n_edges, stats, st);
    }
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

// the key source of a split expand: the whole batch's residues (every rank keys every window and
// keeps its bins: kmp_dev_split_expand) or the pieces every rank sent (kmp_dev_split_group)
struct SplitSrc {
    const uint8_t* d_res;
    const uint64_t* d_res_off;
    const uint16_t* d_class;
    const unsigned long long* d_krecv;  // non-null: the received pieces (kcap u64 words per source)
    uint64_t kcap;
};

static int split_expand_impl(kmp_postings* ws, const SplitSrc& src, uint32_t n, int k, uint64_t slots,
                             uint32_t heavy_df, int require_class_diff, uint32_t part, uint32_t parts, uint64_t cap,
                             const uint32_t* learn, unsigned long long* d_send, uint32_t* d_flags,
                             unsigned long long* d_stats, void* stream) {
    hipStream_t st = as_stream(stream);
    if (heavy_df < 2) heavy_df = 2;
    const Layout lay = make_layout(n, k, slots, true);
    if (!lay.bucketed) return KMP_ESTATE;
    const bool recv = src.d_krecv != nullptr;
    const std::vector<unsigned long long> shape = {n, slots, (unsigned long long)k, parts, recv};
    if (ws->split_shape != shape) {  // a new batch: learned capacities start over
        ws->split_shape = shape;
        ws->shard_cap = slots / 4 / kShards / parts + 4096;
        ws->bp_J_min = 0;
        ws->cur_on = ws->cur_mode;
        ws->shape.clear();
        ws->split_heavy = false;
        ws->fast_tail = ws->fast_mode;
        ws->vreg_on = false;
    }
    const uint32_t nb = 1u << lay.bbits;
    if (learn) {  // the last call's flags, reduced over the ranks: every rank grows the same way
        if (learn[KMP_SPLIT_HEAVY]) ws->split_heavy = true;  // a rank spilled: the heavy path from now on
        // an eighth of slack: the fullest region varies by a few percent from call to call with the
        // heavy path on (3.8 % measured on uniprot k = 5 at G = 2), and a rerun costs a whole step
        if (learn[KMP_SPLIT_MAX_SHARD] > ws->shard_cap)
            ws->shard_cap = learn[KMP_SPLIT_MAX_SHARD] + learn[KMP_SPLIT_MAX_SHARD] / 8 + 256;
        if (learn[KMP_SPLIT_BIN_TILES]) ws->bp_J_min = std::max(ws->bp_J_min, learn[KMP_SPLIT_BIN_TILES] + 2);
        if (learn[KMP_SPLIT_LARGE]) ws->split_large = true;
        if (learn[KMP_SPLIT_CURSOR]) {
            if (recv && ws->cur.p) {
                // a bucket region overflowed on some rank: this rank's regions from its last call's
                // exact bucket counts (the cursors count dropped keys too; cleared only by the next
                // front), its own bins only — the layout is the rank's own business
                PG(ws->vreg.reserve(nb + 1));
                vreg_kernel<<<1, 1024, 0, st>>>(ws->cur.p, nb, ws->vreg.p);
                uint32_t tot = 0;
                PG(hipMemcpyAsync(&tot, ws->vreg.p + nb, 4, hipMemcpyDeviceToHost, st));
                PG(hipStreamSynchronize(st));
                if ((uint64_t)tot + 2 * kBpTile >= (1ull << 32)) return KMP_EINVAL;
                ws->vreg_total = tot;
                ws->vreg_on = true;
            } else {
                ws->cur_on = false;  // the residue source: the counting partition
            }
        }
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
    ws->bin_lo = split_bin_lo(part, dg.nb1, parts);
    ws->bin_hi = split_bin_lo(part + 1, dg.nb1, parts);
    // key regions too small for their run tables carry nothing readable (the keys phase sent no
    // table and raised RERUN with the size that fits): this step groups nothing
    if (recv && src.kcap < split_geom(lay, slots, parts).tb + kSendShards) ws->bin_hi = ws->bin_lo;
    auto make_keys = [&](const Layout& l, hipStream_t s) {
        ws->parted = true;
        if (recv) {
            // the cursor level 2 always (the counting partition needs level 1's own output)
            if (!cur_geometry(l, &ws->cg)) return hipErrorInvalidValue;
            if (ws->vreg_on) {
                ws->cg.vreg = ws->vreg.p;
                const hipError_t e = ws->sorted.reserve(ws->vreg_total);
                if (e != hipSuccess) return e;
            }
            ws->cur_used = true;
            return bp_level1_recv(ws, src.d_krecv, src.kcap, parts, l, slots, s);
        }
        ws->cur_used = ws->cur_on && cur_geometry(l, &ws->cg);
        return bp_level1(ws, src.d_res, src.d_res_off, src.d_class, k, n, slots, l, s);
    };
    const ClearInKeys guard(ws);
    SplitRows rows{};
    rows.parts = parts;
    kmp_row_split(n, parts, rows.start);
    // the send cursors are cleared with the step's flags (by the front's first kernel); routed (no
    // heavy path): the bucket kernels write the send regions, pre-filled with kNoKey
    const bool routed = !ws->split_heavy;
    auto front = [&](hipStream_t s) -> int {
        const uint32_t ncur = routed ? parts * kShards : parts;
        ws->clear_extra = ws->split_cur.p;
        ws->clear_n = ncur;
        const bool bins = ws->bin_hi > ws->bin_lo;
        if (routed) {
            // the send regions pre-filled with kNoKey: by the received front's clear kernel, else here
            // (a kernel, never a memset node: this sequence is captured as a HIP graph, and a captured
            // hipMemsetAsync of the send buffer measured correct on the capturing launch but filled the
            // whole buffer with pointer-sized garbage on the graph's first replay)
            const uint64_t nfill = (uint64_t)parts * cap;
            if (recv && bins) {
                ws->fill_p = d_send;
                ws->fill_n = nfill;
            } else {
                const uint32_t grid = (uint32_t)std::min<uint64_t>(nfill / 2 / 256 / 8 + 1, 2048);
                split_recv_clear_kernel<<<grid, 256, 0, s>>>(nullptr, 0, StepClear{}, d_send, nfill);
                PG(hipGetLastError());
            }
            ws->route_send = d_send;
            ws->route_cap = cap;
            ws->route_rows = rows;
        }
        int rc = KMP_OK;
        if (bins) rc = enqueue_front(ws, make_keys, c, true, s);
        else step_clear_kernel<<<1, 256, 0, s>>>(ws->flags.p, ws->bstats.p, ws->split_cur.p, ncur);  // no bins
        ws->clear_extra = nullptr;
        ws->clear_n = 0;
        ws->route_send = nullptr;
        ws->fill_p = nullptr;
        ws->fill_n = 0;
        return rc;
    };
    // the sharded start's keys phase (this rank's send cursors and flags): read and reset by the finish
    uint32_t* kcur = recv && ws->kcur_dirty ? ws->split_kcur.p : nullptr;
    const uint32_t nkc = parts * kSendShards;
    const uint64_t ktb = recv ? split_geom(lay, slots, parts).tb : 0;
    auto route = [&](hipStream_t s, int heavy_done) -> int {
        // merge: the keys phase wrote this step's key-exchange flags into d_flags first
        const int merge = recv ? 1 : 0;
        const int large = ws->large_used != 0 || ws->bin_hi <= ws->bin_lo;
        if (routed) {  // the bucket kernels routed the keys: the flags and statistics only
            split_pad_finish_kernel<<<dim3(1, 1), 256, 0, s>>>(d_send, cap, ws->split_cur.p, ws->bstats.p, ws->flags.p,
                                                                ws->shard_cap, parts, d_flags, d_stats, heavy_done, 1,
                                                                merge, kcur, nkc, ktb, large);
            PG(hipGetLastError());
            return KMP_OK;
        }
        const unsigned long long* cursor = ws->bstats.p + kRbCursor;
        split_route_kernel<<<dim3((uint32_t)((ws->shard_cap + kRtTile - 1) / kRtTile), kShards), kRtThreads, 0, s>>>(
            ws->inc_sorted.p, cursor, ws->shard_cap, bits_for(n), rows, cap, d_send, ws->split_cur.p);
        split_pad_finish_kernel<<<dim3((uint32_t)std::min<uint64_t>((cap + 1023) / 1024, 256), parts), 256, 0, s>>>(
            d_send, cap, ws->split_cur.p, ws->bstats.p, ws->flags.p, ws->shard_cap, parts, d_flags, d_stats,
            heavy_done, 0, merge, kcur, nkc, ktb, large);
        PG(hipGetLastError());
        return KMP_OK;
    };
    auto unbind = [&]() {
        ws->bin_lo = ws->bin_hi = 0;
        ws->l1_in = nullptr;
        ws->l2_tab = nullptr;
        ws->cg.vreg = nullptr;
    };
    if (ws->split_heavy) {
        // frequent k-mers (vertex.rs:59-140 at k = 5): the rank's front, one read-back, its spill
        // compacted, planned and expanded by the heavy path into the same shard regions (the heavy
        // pairs of the rank's k-mers, all rows), then routed like the light keys.  The spill regions
        // are the rank's own, so a spill overflow reruns the front here; every other capacity is
        // reported in the flags and grown identically on every rank.  Host-synchronous.
        int rc = KMP_OK;
        bool routed_done = false;
        for (int attempt = 0; attempt < 4; ++attempt) {
            if (attempt) ++ws->reruns;
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
                ws->h_segl = rb[kRbSegL];
                ws->h_segw = rb[kRbSegW];
                if ((rc = heavy_phase(ws, c, spill_total, true, st)) != KMP_OK) break;
            }
            rc = route(st, 1);
            routed_done = true;
            break;
        }
        unbind();
        if (kcur && routed_done) ws->kcur_dirty = false;
        ws->last_bucketed = true;
        ws->last_heavy = true;
        if (rc == KMP_OK && !routed_done) {
            // every attempt grew the spill regions: no keys are sent and the flags ask every rank for
            // a rerun, so the ranks stay in lockstep through the collectives (an error returned here
            // on one rank alone would leave the others waiting in the all-to-all); the grown regions
            // are this rank's own and stay for the rerun.  The flags are this step's alone, RERUN
            // (with the sharded start too: d_flags still held the last step's reduced flags, and the
            // keys phase's own flags sit in its cursor words, which the rerun's keys phase clears)
            PG(hipMemsetAsync(d_send, 0xFF, (size_t)parts * cap * sizeof(unsigned long long), st));
            PG(hipMemsetAsync(d_flags, 0, KMP_SPLIT_FLAGS * sizeof(uint32_t), st));
            PG(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_flags + KMP_SPLIT_RERUN), 1, 1, st));
            PG(hipMemsetAsync(d_stats, 0, 8 * sizeof(unsigned long long), st));
        }
        return rc;
    }
    auto enqueue = [&](hipStream_t s) -> int {
        const int rc = front(s);
        return rc != KMP_OK ? rc : route(s, 0);
    };
    const std::vector<unsigned long long> key = {
        n, slots, (unsigned long long)k, heavy_df, (unsigned long long)require_class_diff, part, parts, cap,
        (uintptr_t)src.d_res, (uintptr_t)src.d_res_off, (uintptr_t)src.d_class, (uintptr_t)src.d_krecv, src.kcap,
        (uintptr_t)d_send, (uintptr_t)d_flags, (uintptr_t)d_stats, ws->shard_cap, ws->spill_cap, ws->bp_J_min,
        ws->cur_on, ws->timing, ws->vreg_on ? ws->vreg_total + 1 : 0, (uintptr_t)kcur, ws->split_large};
    if (getenv("KMP_TRACE"))
        fprintf(stderr, "kmp-trace: split_expand n %u part %u/%u cap %llu recv %d kcap %llu routed %d large %d shard_cap %llu\n",
                n, part, parts, (unsigned long long)cap, (int)recv, (unsigned long long)src.kcap, (int)routed,
                (int)ws->split_large, (unsigned long long)ws->shard_cap);
    const int rc = slot_launch(ws, ws->split_g[0], key, enqueue, st);
    if (getenv("KMP_TRACE") && rc == KMP_OK) {  // diagnostics: every routed key inside its region's rows
        PG(hipStreamSynchronize(st));
        std::vector<unsigned long long> h((size_t)parts * cap);
        PG(hipMemcpy(h.data(), d_send, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        const unsigned pb = bits_for(n);
        uint64_t bad = 0, keys = 0;
        unsigned long long first = 0;
        for (uint32_t d = 0; d < parts; ++d)
            for (uint64_t i = 0; i < cap; ++i) {
                const unsigned long long x = h[(size_t)d * cap + i];
                if (x == kNoKey) continue;
                ++keys;
                const uint64_t p = x >> pb, q = x & ((1ull << pb) - 1);
                if (p < rows.start[d] || p >= rows.start[d + 1] || q <= p || q >= n) {
                    if (!bad++) first = x;
                }
            }
        fprintf(stderr, "kmp-trace: split_expand part %u sent %llu keys, %llu outside their rows (first %llx)\n", part,
                (unsigned long long)keys, (unsigned long long)bad, first);
    }
    unbind();
    if (kcur) ws->kcur_dirty = false;
    ws->last_bucketed = true;
    ws->last_heavy = false;
    return rc;
}

int kmp_dev_split_expand(kmp_postings* ws, const uint8_t* d_res, const uint64_t* d_res_off, const uint16_t* d_class,
                         uint32_t n, int k, uint64_t slots, uint32_t heavy_df, int require_class_diff, uint32_t part,
                         uint32_t parts, uint64_t cap, const uint32_t* learn, unsigned long long* d_send,
                         uint32_t* d_flags, unsigned long long* d_stats, void* stream) {
    if (!ws || !d_res || !d_res_off || !d_class || !d_send || !d_flags || !d_stats || k < 1 || k > kMaxK ||
        parts < 1 || parts > kSplitMax || part >= parts || cap < 1)
        return KMP_EINVAL;
    return split_expand_impl(ws, SplitSrc{d_res, d_res_off, d_class, nullptr, 0}, n, k, slots, heavy_df,
                             require_class_diff, part, parts, cap, learn, d_send, d_flags, d_stats, stream);
}

int kmp_split_plan(const uint64_t* offsets, uint32_t n, int k, uint32_t part, uint32_t parts, kmp_split_span* out) {
    if (!offsets || !out || k < 1 || k > kMaxK || parts < 1 || parts > kSplitMax || part >= parts) return KMP_EINVAL;
    *out = kmp_split_span{};
    const uint64_t total = offsets[n];
    const uint64_t slots = kmp_set_capacity(n, total);
    if (slots > 0xFFFFFFFFull) return KMP_EINVAL;
    const Layout lay = make_layout(n, k, slots, true);
    if (!lay.bucketed) return KMP_ESTATE;
    const SplitGeom sg = split_geom(lay, slots, parts);
    const uint32_t c_lo = split_chunk_lo(sg, part, parts), c_hi = split_chunk_lo(sg, part + 1, parts);
    out->slots = slots;
    out->n_chunks = sg.n_chunks;
    out->c_lo = c_lo;
    out->c_hi = c_hi;
    // the protein whose slot region [set_base(off[p], p), set_base(off[p + 1], p + 1)) holds slot s
    // (n: the tail past the last region) — chunk_desc_kernel's view of a chunk's ends
    auto prot = [&](uint64_t s) {
        uint32_t lo = 0, hi = n;  // largest p in [0, n] with base(p) <= s
        while (lo < hi) {
            const uint32_t mid = (uint32_t)(((uint64_t)lo + hi + 1) / 2);
            if (set_base(offsets[mid], mid) <= s) lo = mid;
            else hi = mid - 1;
        }
        return lo;
    };
    if (c_hi > c_lo) {
        const uint64_t s0 = (uint64_t)c_lo * kKeyChunk, s1 = std::min<uint64_t>((uint64_t)c_hi * kKeyChunk, slots);
        uint32_t p = prot(s0);
        uint64_t L = p < n ? offsets[p + 1] - offsets[p] : 0, b = set_base(offsets[p], p);
        const uint64_t r0 = offsets[p] + std::min<uint64_t>(s0 - b, L);
        p = prot(s1 - 1);
        L = p < n ? offsets[p + 1] - offsets[p] : 0;
        b = set_base(offsets[p], p);
        const uint64_t r1 = p < n ? offsets[p] + std::min<uint64_t>(L, s1 - b + k - 1) : offsets[p];
        out->res_lo = r0 & ~15ull;  // the level-1 kernel's 16-byte loads start on 16-byte boundaries
        out->res_hi = std::max(r1, out->res_lo);
    }
    out->key_table_words = sg.tb;
    // a region: the table plus kSendShards sub-regions of a fair share of the windows with 1/16 slack
    const uint64_t per = slots / parts / parts / kSendShards;
    out->key_cap = sg.tb + kSendShards * (per + per / 16 + 256);
    return KMP_OK;
}

int kmp_dev_split_keys(kmp_postings* ws, const uint8_t* d_res, uint64_t res_lo, uint64_t res_hi,
                       const uint64_t* d_res_off, const uint16_t* d_class, uint32_t n, int k, uint64_t slots,
                       uint32_t part, uint32_t parts, uint64_t kcap, unsigned long long* d_ksend, uint32_t* d_flags,
                       void* stream) {
    if (!ws || !d_res_off || !d_class || !d_ksend || !d_flags || k < 1 || k > kMaxK || parts < 1 ||
        parts > kSplitMax || part >= parts || res_hi < res_lo || (res_lo & 15u) || (res_hi > res_lo && !d_res))
        return KMP_EINVAL;
    if (slots > 0xFFFFFFFFull || (uint64_t)parts * kcap >= (1ull << 32)) return KMP_EINVAL;
    hipStream_t st = as_stream(stream);
    const Layout lay = make_layout(n, k, slots, true);
    if (!lay.bucketed) return KMP_ESTATE;
    const SplitGeom sg = split_geom(lay, slots, parts);
    // a region too small for its run table: nothing is sent, the flags report the size that fits
    const uint64_t sub64 = kcap >= sg.tb + kSendShards ? (kcap - sg.tb) / kSendShards : 0;
    const uint32_t sub = (uint32_t)std::min<uint64_t>(sub64, 0xFFFFFFFFull);
    const uint32_t c_lo = split_chunk_lo(sg, part, parts), c_hi = split_chunk_lo(sg, part + 1, parts);
    const uint32_t G = c_hi - c_lo, nkc = parts * kSendShards;
    PG(ws->split_desc.reserve(std::max(1u, G)));
    // the send cursors | the keys phase's flags: zero when allocated, and reset by the group phase
    // that reads them (kmp_dev_split_group's finish), so this call clears nothing
    PG(ws->split_kcur.reserve(nkc + kFlN));
    if (ws->kcur_zero_p != ws->split_kcur.p || ws->kcur_dirty) {
        PG(hipMemsetAsync(ws->split_kcur.p, 0, ws->split_kcur.n * sizeof(uint32_t), st));
        ws->kcur_zero_p = ws->split_kcur.p;
    }
    ws->kcur_dirty = true;
    const BpDigits dg = bp_digits(lay);
    const uint32_t pw21 = (uint32_t)pow21(k - 1);
    // the rank's chunk descriptors depend on the batch's offsets only: computed once per batch
    const std::vector<unsigned long long> dkey = {(uintptr_t)d_res_off, n, slots, (unsigned long long)k, c_lo, c_hi,
                                                  (uintptr_t)ws->split_desc.p};
    if (ws->split_desc_key != dkey) {
        chunk_desc_kernel<<<(n + 1 + 255) / 256, 256, 0, st>>>(d_res_off, n, slots, c_lo, c_hi, k, ws->split_desc.p,
                                                               nullptr, 0, StepClear{});
        PG(hipGetLastError());
        ws->split_desc_key = dkey;
    }
    auto enqueue = [&](hipStream_t s) -> int {
        if (G) {
            const SendL1 sl{d_ksend, kcap, sg.tb, sub, ws->split_kcur.p, part, parts, c_lo, sg.rowlen, res_lo, res_hi};
            // one workgroup per chunk (every digit ranked: the single-GPU geometry; two or four chunks
            // per persistent workgroup measured 5 and 30 % slower at G = 8); its flags go to the words
            // after the cursors
            bp_scatter1p_kernel<kL1Threads, true, false><<<G, kL1Threads, 0, s>>>(
                d_res, d_res_off, d_class, k, n, slots, G, ws->split_desc.p, lay, dg, pw21, 0u, dg.nb1, nullptr,
                nullptr, ws->split_kcur.p + nkc, sl);
        }
        PG(hipGetLastError());
        return KMP_OK;
    };
    const std::vector<unsigned long long> key = {n, slots, (unsigned long long)k, part, parts, kcap, res_lo, res_hi,
                                                 (uintptr_t)d_res, (uintptr_t)d_res_off, (uintptr_t)d_class,
                                                 (uintptr_t)d_ksend, (uintptr_t)d_flags, (uintptr_t)ws->split_kcur.p,
                                                 (uintptr_t)ws->split_desc.p};
    return slot_launch(ws, ws->split_g[2], key, enqueue, st);
}

int kmp_dev_split_group(kmp_postings* ws, const unsigned long long* d_krecv, uint64_t kcap, uint32_t n, int k,
                        uint64_t slots, uint32_t heavy_df, int require_class_diff, uint32_t part, uint32_t parts,
                        uint64_t cap, const uint32_t* learn, unsigned long long* d_send, uint32_t* d_flags,
                        unsigned long long* d_stats, void* stream) {
    if (!ws || !d_krecv || !d_send || !d_flags || !d_stats || k < 1 || k > kMaxK || parts < 1 || parts > kSplitMax ||
        part >= parts || cap < 1 || (uint64_t)parts * kcap >= (1ull << 32))
        return KMP_EINVAL;
    return split_expand_impl(ws, SplitSrc{nullptr, nullptr, nullptr, d_krecv, kcap}, n, k, slots, heavy_df,
                             require_class_diff, part, parts, cap, learn, d_send, d_flags, d_stats, stream);
}

int kmp_dev_split_edges(kmp_postings* ws, const unsigned long long* d_keys, uint64_t m, uint32_t n, uint32_t row_lo,
                        uint32_t row_hi, uint32_t min_shared, uint32_t* d_p, uint32_t* d_q, uint32_t* d_w,
                        uint64_t cap, uint64_t* n_edges, void* stream) {
    if (!ws || !n_edges || row_lo > row_hi || row_hi > n || (m && !d_keys) || (cap && (!d_p || !d_q || !d_w)))
        return KMP_EINVAL;
    *n_edges = 0;
    hipStream_t st = as_stream(stream);
    if (m == 0 || row_lo == row_hi) {  // nothing to reduce; still synchronous, as the full path is
        PG(hipStreamSynchronize(st));
        return KMP_OK;
    }
    if (m > 0xFFFFFFFFull) return KMP_EINVAL;
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
    for (int attempt = 0; attempt < 8; ++attempt) {
        if (attempt) ++ws->reruns;
        PtGeom g;
        if (!pt_geometry(ws, c, m, &g)) return KMP_EINVAL;
        g.flat_n = m;  // the received regions, padded with kNoKey, read as one array
        g.nshards = 1;
        g.sc = m;
        g.jt = (uint32_t)((m + kPtTile - 1) / kPtTile);
        hipError_t e = hipSuccess;
        pt_bufs(ws, g, true, &e, st);
        PG(e);
        // u32 row-block keys (the fast tail's fixed or learned regions)
        PG(ws->inc.reserve(pt_fast(ws, g) ? std::max<uint64_t>(m, (uint64_t)g.nrb * g.ftcap / 2) : m));
        PG(ws->uniq.reserve(m));  // staged p | q (u32 each)
        PG(ws->w.reserve(m));
        PG(ws->ovf.reserve((uint64_t)g.nrb + 1));
        PG(small_reserve(ws, st));
        PG(ws->flags.reserve(kFlN));
        PG(ws->bstats.reserve(kGsWords));
        if (!ws->hrb) PG(hipHostMalloc((void**)&ws->hrb, kRbWords * sizeof(unsigned long long), hipHostMallocCoherent));
        auto enqueue = [&](hipStream_t s) -> int {
            // the step's flags and statistics cleared (the expand's stats are out): by the fast tail's
            // scatter kernel, or a kernel of its own before the counting tail
            if (pt_fast(ws, g)) {
                ws->tail_clear = true;
            } else {
                step_clear_kernel<<<1, 256, 0, s>>>(ws->flags.p, ws->bstats.p);
            }
            const int rc = enqueue_tail_in(ws, c, g, d_keys, nullptr, m, s);
            ws->tail_clear = false;
            return rc;
        };
        const std::vector<unsigned long long> key = {m, n, row_lo, row_hi, c.min_shared, cap, (uintptr_t)d_keys,
                                                     (uintptr_t)d_p, (uintptr_t)d_q, (uintptr_t)d_w, g.rbits,
                                                     ws->timing, ws->fast_tail};
        if (getenv("KMP_TRACE")) {
            fprintf(stderr,
                    "kmp-trace: split_edges m %llu n %u rows [%u, %u) cap %llu rbits %u nrb %u fast %d inc %llu pt %llu\n",
                    (unsigned long long)m, n, row_lo, row_hi, (unsigned long long)cap, g.rbits, g.nrb,
                    (int)pt_fast(ws, g), (unsigned long long)ws->inc.n, (unsigned long long)ws->pt.n);
            PG(hipStreamSynchronize(st));
            std::vector<unsigned long long> h(m);
            PG(hipMemcpy(h.data(), d_keys, m * sizeof(unsigned long long), hipMemcpyDeviceToHost));
            const unsigned pb = bits_for(n);
            uint64_t bad = 0, keys = 0;
            unsigned long long first = 0;
            for (const unsigned long long x : h) {
                if (x == kNoKey) continue;
                ++keys;
                const uint64_t p = x >> pb, q = x & ((1ull << pb) - 1);
                if (p < row_lo || p >= row_hi || q <= p || q >= n)
                    if (!bad++) first = x;
            }
            fprintf(stderr, "kmp-trace: split_edges received %llu keys, %llu outside rows (first %llx)\n",
                    (unsigned long long)keys, (unsigned long long)bad, first);
        }
        int rc = slot_launch(ws, ws->split_g[1], key, enqueue, st);
        if (rc != KMP_OK) return rc;
        PG(hipStreamSynchronize(st));
        const unsigned long long* rb = ws->hrb;
        if (rb[kRbFast]) {  // a fast-tail region overflowed: fewer rows per block, or the counting tail
            fast_overflow(ws, g, rb);
            continue;
        }
        if (rb[kRbRange]) {  // a received key outside [row_lo, row_hi): nothing written out of bounds
            PG(hipMemsetAsync(ws->flags.p + kFlRange, 0, sizeof(uint32_t), st));
            PG(hipStreamSynchronize(st));
            return KMP_EINVAL;
        }
        uint64_t ne = rb[kRbRuns];
        ws->last_fast = pt_fast(ws, g);
        ws->last_ovf = (uint32_t)rb[kRbOvf];
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
