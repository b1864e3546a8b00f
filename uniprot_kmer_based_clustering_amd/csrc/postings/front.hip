// postings/front.hip — host side of the front: level 1 / level 2 / bucket launches.
// Part of kmp_postings.hip (included there; not a translation unit of its own).

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
        chunk_desc_kernel<<<(n + 1 + 255) / 256, 256, 0, st>>>(d_res_off, n, slots, 0u, G, k,
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
        if (!per_cu && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, bp_scatter1p_kernel<kL1Threads, false, true>,
                                                                     kL1Threads, 0) != hipSuccess ||
                        per_cu < 1))
            per_cu = 2;
        // every bin owned (one GPU): one workgroup per chunk, in order (bp_scatter1p 112 -> 103 us at
        // config 3); a share of the bins (a rank of the k-mer split, little work per chunk): persistent
        const uint32_t grid = nown >= dg.nb1 ? G : std::min<uint32_t>(G, (uint32_t)per_cu * device_cus());
        if (nown) {
            const uint4* desc = reinterpret_cast<const uint4*>(ws->chunk_desc.p);
            if (nown >= dg.nb1) {
                // every bin (one GPU): the run table written transposed by the level-1 workgroups
                // themselves (XCD-aware chunk order; 8 * ceil(G / 8) workgroups, the few past G return)
                bp_scatter1p_kernel<kL1Threads, false, false, true><<<8 * ((G + 7) / 8), kL1Threads, 0, st>>>(
                    d_res, d_res_off, d_class, k, n, slots, G, desc, lay, dg, pw21, dlo, dhi, H1 + h1, ws->keys.p,
                    ws->flags.p, SendL1{});
            } else {
                if (grid < G)
                    bp_scatter1p_kernel<kL1Threads, false, true><<<grid, kL1Threads, 0, st>>>(
                        d_res, d_res_off, d_class, k, n, slots, G, desc, lay, dg, pw21, dlo, dhi, H1, ws->keys.p,
                        ws->flags.p, SendL1{});
                else
                    bp_scatter1p_kernel<kL1Threads, false, false><<<grid, kL1Threads, 0, st>>>(
                        d_res, d_res_off, d_class, k, n, slots, G, desc, lay, dg, pw21, dlo, dhi, H1, ws->keys.p,
                        ws->flags.p, SendL1{});
                if (!direct)
                    bp_h1t_kernel<<<dim3((G + 31) / 32, (nown + 31) / 32), 256, 0, st>>>(H1, G, nown, 0, nown, H1 + h1);
            }
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

// workgroup size of the level-2 gather (a 4,096-key round either way).  512 threads x 8 keys (82
// VGPRs, 6 waves per SIMD instead of 3) measured no faster at config 3 (buckets_level2 0.159-0.164 ms
// vs 0.149-0.160 ms), so 256 x 16 stays
constexpr uint32_t kGatherThreads = 256;
// the cursor level 2's buffers (before any launch of the call's front)
int bp_level2c_reserve(kmp_postings* ws, const Layout& lay) {
    const uint32_t nb = 1u << lay.bbits;
    PG(ws->cur.reserve(nb));
    PG(ws->sorted.reserve(ws->cg.vreg ? ws->vreg_total : (uint64_t)nb * ws->cg.capb));
    PG(ws->cnt.reserve(2 * (uint64_t)nb + 2));  // the large-bucket list
    return KMP_OK;
}

// the level-2 gather of coarse bins [a, b) (of the call's bins [c0, c1), whose run table level 1
// wrote from bin c0): a local level 1's output or the received pieces
int bp_level2c_bins(kmp_postings* ws, const Layout& lay, uint32_t a, uint32_t b, hipStream_t st) {
    const BpDigits dg = bp_digits(lay);
    uint32_t c0, c1;
    own_bins(ws, dg, &c0, &c1);
    if (b > a) {
        const uint32_t ntiles = (ws->bp_G + ws->bp_T - 1) / ws->bp_T, per = (ntiles * (b - a) + 7) / 8;
        constexpr uint32_t kGp = kBpGatherTile / kGatherThreads, kGt = kGatherThreads;
        // level 1's output: this call's own segments, or (the k-mer split's sharded start) the
        // pieces every rank sent (ws->l2_tab: their run tables in the receive buffer)
        const bool recv = ws->l2_tab != nullptr;
        const unsigned long long* in = recv ? ws->l1_in : ws->keys.p;
        const uint32_t* tab = recv ? ws->l2_tab : ws->bp.p + ws->bp_h1t;
        const uint32_t grid = 8 * per;
#define KMP_L2G(V, R)                                                                                           \
    bp_scatter2g_kernel<kGp, kGt, V, R><<<grid, kGt, 0, st>>>(in, tab, ws->bp_G, ws->bp_hsb, ws->bp_hsc, ws->bp_T, \
                                                              ntiles, b - a, dg, ws->cg, ws->cur.p, ws->sorted.p,     \
                                                              ws->flags.p, a, c0, ws->l2_rt)
        if (recv) {
            if (ws->cg.vreg) KMP_L2G(true, true);
            else KMP_L2G(false, true);
        } else {
            if (ws->cg.vreg) KMP_L2G(true, false);
            else KMP_L2G(false, false);
        }
#undef KMP_L2G
    }
    PG(hipGetLastError());
    return KMP_OK;
}

// Level 2, cursor variant: ws->keys (level 1) -> the bucket regions of ws->sorted, counts in ws->cur.
int bp_level2c(kmp_postings* ws, const Layout& lay, hipStream_t st) {
    const BpDigits dg = bp_digits(lay);
    const uint32_t nb = 1u << lay.bbits;
    uint32_t* C1 = ws->bp.p + ws->bp_c1;
    const int rc = bp_level2c_reserve(ws, lay);
    if (rc != KMP_OK) return rc;
    uint32_t c0, c1;
    own_bins(ws, dg, &c0, &c1);
    if (!ws->bp_local)  // the local level 1 cleared the counts with its chunk_first
        bp_cur_clear_kernel<<<std::min<uint32_t>((nb + 1023) / 1024, 1024), 1024, 0, st>>>(ws->cur.p, nb);
    if (c1 > c0 && ws->bp_local) {
        return bp_level2c_bins(ws, lay, c0, c1, st);
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

// ---- the k-mer split with a sharded start (kmp_dev_split_keys / kmp_dev_split_group) ----
// geometry every rank derives alike from (batch, k, parts): chunks, the most chunks a rank holds,
// the run-table row length (the most bins a rank owns + 1) and the table's u64 words per region
struct SplitGeom {
    uint32_t n_chunks, cm, rowlen, nb1;
    uint64_t tb;
};
SplitGeom split_geom(const Layout& lay, uint64_t slots, uint32_t parts) {
    SplitGeom g{};
    g.n_chunks = (uint32_t)((slots + kKeyChunk - 1) / kKeyChunk);
    g.cm = (g.n_chunks + parts - 1) / parts;
    g.nb1 = bp_digits(lay).nb1;
    g.rowlen = (g.nb1 + parts - 1) / parts + 1;
    g.tb = ((uint64_t)g.cm * g.rowlen + 1) / 2;
    return g;
}
uint32_t split_chunk_lo(const SplitGeom& g, uint32_t part, uint32_t parts) {
    return (uint32_t)((uint64_t)part * g.n_chunks / parts);
}

// clears the bucket counts of the cursor level 2 and (sc) the step's flags: the front of a call
// whose level 1 ran elsewhere (the received pieces)
// and fills [fill, fill + nfill) with kNoKey (the routed send regions)
__global__ void split_recv_clear_kernel(uint32_t* __restrict__ cur, uint32_t ncur, StepClear sc,
                                        unsigned long long* __restrict__ fill, uint64_t nfill) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    for (uint32_t i = t; i < ncur; i += gridDim.x * blockDim.x) cur[i] = 0;
    ulonglong2* f2 = reinterpret_cast<ulonglong2*>(fill);  // 16-B aligned (a device allocation)
    for (uint64_t i = t; i < nfill / 2; i += (uint64_t)gridDim.x * blockDim.x) f2[i] = make_ulonglong2(kNoKey, kNoKey);
    if (t == 0 && (nfill & 1)) fill[nfill - 1] = kNoKey;
    if (blockIdx.x == 0 && sc.flags) {
        for (uint32_t i = threadIdx.x; i < sc.n_gstats; i += blockDim.x) sc.gstats[i] = 0;
        for (uint32_t i = threadIdx.x; i < sc.n_flags; i += blockDim.x) sc.flags[i] = 0;
        for (uint32_t i = threadIdx.x; i < sc.n_extra; i += blockDim.x) sc.extra[i] = 0;
    }
}

// level 1 of a call over received pieces: nothing to compute, only the clears and level 2's
// geometry (bp_level2c reads the pieces where they landed)
hipError_t bp_level1_recv(kmp_postings* ws, const unsigned long long* krecv, uint64_t kcap, uint32_t parts,
                          const Layout& lay, uint64_t slots, hipStream_t st) {
    const BpDigits dg = bp_digits(lay);
    const SplitGeom sg = split_geom(lay, slots, parts);
    const uint32_t nb = 1u << lay.bbits;
    hipError_t e = ws->cur.reserve(nb);
    if (e != hipSuccess) return e;
    StepClear sc{};
    if (ws->defer_clear) {
        sc = StepClear{ws->flags.p, kFlN, ws->bstats.p, kShards * 10, ws->clear_extra, ws->clear_n};
        ws->defer_clear = false;
    }
    const uint32_t grid = (uint32_t)std::min<uint64_t>(std::max<uint64_t>((nb + 255) / 256, ws->fill_n / 2 / 256 / 8 + 1), 2048);
    split_recv_clear_kernel<<<grid, 256, 0, st>>>(ws->cur.p, nb, sc, ws->fill_p, ws->fill_n);
    ws->bp_local = true;
    ws->bp_G = parts * sg.cm;
    ws->bp_T = std::min<uint32_t>(kBpGatherMax, std::max<uint32_t>(1, kBpGatherTile * 7 / 4 * dg.nb1 / kKeyChunk));
    ws->bp_hsb = 0;
    ws->bp_hsc = sg.rowlen;
    ws->l1_in = krecv;
    ws->l2_tab = reinterpret_cast<const uint32_t*>(krecv);
    ws->l2_rt = RecvTab{sg.cm, sg.n_chunks, parts, 2 * kcap, sg.tb};
    return hipGetLastError();
}
