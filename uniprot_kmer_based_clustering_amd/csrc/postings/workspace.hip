// postings/workspace.hip — the workspace (struct kmp_postings) and its buffers.
// Part of kmp_postings.hip (included there; not a translation unit of its own).

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
    bool fast_tail = true;      // unscored calls take the fast row-block tail (off for a shape whose
                                // row blocks still pass kFtCap after kFastShrinks tries: kRbFast)
    uint32_t fast_tries = 0;    // ... fewer rows per block tried so far
    const uint32_t* small_zero_p = nullptr;  // the ws->small allocation that was cleared
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
    // level 2 over received pieces (the k-mer split's sharded start, kmp_dev_split_group): the
    // receive buffer (keys) and its run tables; nullptr: level 1's own output (ws->keys, ws->bp)
    const unsigned long long* l1_in = nullptr;
    const uint32_t* l2_tab = nullptr;
    RecvTab l2_rt{};
    bool tail_clear = false;  // the fast tail's scatter clears the step's flags and statistics first
    unsigned long long* fill_p = nullptr;  // filled with kNoKey by the received front's clear kernel
    uint64_t fill_n = 0;
    Grow<uint32_t> split_kcur;  // the key pieces' send cursors (parts x kSendShards) | kFlSend | kFlClass
    const uint32_t* kcur_zero_p = nullptr;  // the split_kcur allocation that was cleared
    bool kcur_dirty = false;    // a keys phase's cursors not yet read (and reset) by a group phase
    bool split_large = false;   // the k-mer split launches the large-bucket kernel (a call listed one)
    Grow<uint4> split_desc;     // the sharded keys phase's chunk descriptors (per batch and rank)
    std::vector<unsigned long long> split_desc_key;
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
    // kmp_postings_set_row_span: the batch's ranged calls' rows (span_hi 0: any); the index's rows
    uint32_t span_lo = 0, span_hi = 0, h_span_lo = 0, h_span_hi = 0;
    // tail_multi_rows: the phase its calls run (set around them; nullptr otherwise), and the pass's
    // per-row key counts (ws[0]'s)
    RowDirect* rdir = nullptr;
    Grow<uint32_t> rcnt, hrec;  // hrec: this workspace's heavy_rows records (phase 1 -> phase 2)
    uint64_t h_ng = 0;  // k-mers of the compaction (read back with the index)
    uint64_t spill_cap = 0;     // keys per spill shard region
    bool heavy = false;         // this workspace's batches spill: run the split step
    bool heavy_ready = false;   // hE / hGS hold the current front's compacted spill
    uint64_t h_m = 0;                // spill keys behind hE (the bound on elements and k-mers)
    // the front's spill segments (read-back): count, largest, large ones, keys in whole buckets
    uint64_t h_segs = 0, h_segmax = 0, h_segl = 0, h_segw = 0;
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
        std::vector<unsigned long long> key, seen, plain;  // plain: a key whose capture does not replay
        std::vector<std::vector<unsigned long long>> launches;  // its kernel launches (KMP_GRAPH_VERIFY check)
        void reset() {
            if (gexec) (void)hipGraphExecDestroy(gexec);
            gexec = nullptr;
            key.clear();
            seen.clear();
            plain.clear();
            launches.clear();
        }
    } split_g[3];  // the k-mer split's phases (expand or group, edges, keys)
    // pipelined submissions (kmp_dev_pairs_residues_submit / kmp_postings_wait): a submission whose
    // step graph replays goes out without a host wait; it has a slot of its own (two), with its own
    // read-back, stage events, completion event and captured graph, so the next submission can be
    // queued behind it before its read-back is checked
    GraphSlot fg[2];
    unsigned long long* hrb_slot[2] = {nullptr, nullptr};
    hipEvent_t evs[2][KMP_POSTINGS_STAGES + 1] = {};
    hipEvent_t done_ev[2] = {};
    int async_slot = -1;          // the slot of the submission being enqueued (-1: a synchronous call)
    bool async_launched = false;  // ... its step went out without a host wait (async_geom: its tail geometry)
    PtGeom async_geom{};
    std::shared_ptr<void> async;  // the submissions (AsyncState, api.hip)
    // the fused step's graph key of this call, and of the last call that finished clean
    std::vector<unsigned long long> cur_key, ok_key;
    hipGraphExec_t gexec = nullptr;
    hipStream_t cst = nullptr;  // capture stream
    hipStream_t side = nullptr;   // side_fork: the heavy path's large segment sorts
    hipEvent_t sev[2] = {};

    std::vector<unsigned long long> gkey, gkey_seen, gkey_plain;  // gkey_plain: a key whose capture does not replay
    std::vector<std::vector<unsigned long long>> glaunches;  // the fused graph's kernel launches (KMP_DEBUG check)
    uint64_t graph_replays = 0;
    uint64_t reruns = 0;  // calls (or a split call's phases) run again with a grown capacity
    // read-back of a step (kRb* layout), written by the pack kernel into coherent pinned memory
    unsigned long long* hrb = nullptr;
    hipEvent_t ev[KMP_POSTINGS_STAGES + 1] = {};
    hipEvent_t* evp = ev;  // the stage events a call's marks record into (a submission: its slot's)
    hipEvent_t mev[4] = {};  // kmp_dev_pairs_rows_multi: start, first k expanded, second k, tail done
    const uint32_t* pt_zero_p = nullptr;  // the pt allocation whose totals T were cleared
    size_t pt_zero_n = 0;
    ~kmp_postings() {
        for (auto* g : {&keys, &sorted, &inc, &inc_sorted, &uniq, &bstats, &btot, &boff, &spill, &hkeys, &hsorted,
                        &hGS, &htc, &htoff, &hoff, &hRH, &hseg, &hcur, &ovk, &ovx, &split_cur, &dlb})
            g->release();
        for (auto* g : {&w, &keep, &pos, &small, &cnt, &flags, &chunk_first, &chunk_desc, &bp, &pt, &ovf, &ovr, &ova, &stg2, &k2, &dsc, &hE, &hgi, &hcnt,
                        &hrun, &hblk, &cur, &hGH, &split_kcur, &hKG, &hPE, &hPO, &hPC, &rcnt, &hrec, &doff, &vreg})
            g->release();
        for (auto* g : {&split_desc})
            g->release();
        tmp.release();
        for (auto& e : ev)
            if (e) (void)hipEventDestroy(e);
        for (auto& e : mev)
            if (e) (void)hipEventDestroy(e);
        if (hrb) (void)hipHostFree(hrb);
        for (int i = 0; i < 2; ++i) {
            if (hrb_slot[i]) (void)hipHostFree(hrb_slot[i]);
            for (auto& e : evs[i])
                if (e) (void)hipEventDestroy(e);
            if (done_ev[i]) (void)hipEventDestroy(done_ev[i]);
            fg[i].reset();
        }
        if (gexec) (void)hipGraphExecDestroy(gexec);
        for (auto& g : split_g) g.reset();
        if (cst) (void)hipStreamDestroy(cst);
        if (side) (void)hipStreamDestroy(side);
        for (auto& e : sev)
            if (e) (void)hipEventDestroy(e);
    }
    void mark(int stage, hipStream_t st) {
        if (timing) (void)hipEventRecord(evp[stage], st);
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
