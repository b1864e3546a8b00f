// kmp_api.cpp — host-buffer C ABI (include/kmerpair.h: context … edges).  Each call is
// synchronous, like the reference's Graph methods; every device step goes through the
// kmp_dev_* stages of kmp_kernels.hip on the context's own stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "kmerpair.h"
#include "kmp_df.hpp"
#include "kmp_edges.hpp"
#include "kmp_internal.hpp"
#include "kmp_merge.hpp"
#include "kmp_mphf.hpp"
#include "kmp_multi.hpp"
#include "kmp_stream.hpp"
#include "kmp_threads.hpp"

using namespace kmp;

namespace {


struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    hipError_t reserve(size_t b) {
        if (b <= bytes && p) return hipSuccess;
        release();
        hipError_t e = hipMalloc(&p, b ? b : 16);
        if (e == hipSuccess) bytes = b ? b : 16;
        return e;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
    void swap(DevBuf& o) {
        std::swap(p, o.p);
        std::swap(bytes, o.bytes);
    }
    void adopt(void* q, size_t b) {  // take ownership of a hipMalloc'd buffer
        release();
        p = q;
        bytes = q ? b : 0;
    }
};

}  // namespace

// one k of a multi-k / streamed call: the sets (scores of the tiles engine), a workspace whose front
// is kept across the passes, and the pass's edges
struct kmp_kset {
    int k = 0;
    DevBuf set, set_len, rep, rep_len, ep, eq, ew, score;
    uint64_t cap = 0;
    std::vector<uint32_t> h_set_len, h_rep_len;
    kmp_postings* ws = nullptr;
    ~kmp_kset() { kmp_postings_destroy(ws); }
};

// one rank of a multi-GPU context: its device, stream, workspace and pair buffers; ranks
// other than 0 also hold their copy of the packed batch (rank 0 uses the context's)
struct kmp_rank {
    int device = 0;
    hipStream_t stream = nullptr;  // rank 0: the context's
    bool own_stream = false;
    DevBuf res, off, cls, ep, eq, ew;
    DevBuf send, recv, sflags, sstats;  // k-mer split: exchange regions, flags, statistics
    uint64_t cap = 0;
    kmp_postings* ws = nullptr;
    // streamed passes (kmp_pairs_stream) of this rank's rows: per-k workspaces, merged arrays, summary
    std::vector<std::unique_ptr<kmp_kset>> ksets;
    DevBuf mscore, mwk, mscratch, dacc;
    ~kmp_rank() {
        (void)hipSetDevice(device);
        ksets.clear();
        if (own_stream && stream) {
            (void)hipStreamSynchronize(stream);
            (void)hipStreamDestroy(stream);
        }
        kmp_postings_destroy(ws);
        res.release();
        off.release();
        cls.release();
        ep.release();
        eq.release();
        ew.release();
        send.release();
        recv.release();
        sflags.release();
        sstats.release();
    }
};

struct kmp_ctx {
    int device = 0;
    int threads = 1;
    std::string err;
    std::mutex err_mu;  // err is written from the rank threads of a multi-GPU stream
    hipStream_t stream = nullptr;

    uint32_t n = 0;
    uint64_t total_res = 0;
    uint32_t max_len = 0;
    bool loaded = false;
    std::vector<uint64_t> h_off;
    std::vector<uint16_t> h_cls;
    DevBuf res, off, cls;

    int k_codes = 0;
    DevBuf codes;

    int k_sets = 0;
    DevBuf set, set_len, rep, rep_len, bits, scratch;
    DevBuf escore;  // per-edge BLOSUM scores (u32) from the scored reduction, or f32 from edge_blosum_device
    std::vector<uint32_t> h_set_len, h_rep_len;
    kmp_counters counters{};

    DevBuf items, dense_off, dense, long_ids, ep, eq, ew, ecount, sort_tmp;
    uint64_t edge_cap = 0;
    kmp_postings* postings = nullptr;

    // repeat index of the current sets (kmp_get_df …): MPHF over the df >= 2 codes
    bool rep_index = false, hash_kmers = false;
    kmp_mphf* rep_mphf = nullptr;
    uint64_t n_repeat = 0;
    DevBuf code_by_id, df_by_id, hk_ids;
    std::vector<uint64_t> h_hk_off;
    void drop_repeat_index() {
        kmp_mphf_free(rep_mphf);
        rep_mphf = nullptr;
        rep_index = hash_kmers = false;
        n_repeat = 0;
        code_by_id.release();
        df_by_id.release();
        hk_ids.release();
        h_hk_off.clear();
    }
    // bounded-memory passes: pair keys per pass (0: auto from free device memory), passes of the
    // last kmp_pairs / kmp_pairs_multi_k
    uint64_t pass_keys = 0;
    // the auto budget (plain, fused), from the free memory at the batch's first passed call: later
    // calls hold that call's pass buffers (cached across streams) and plan the same passes
    uint64_t budget[2] = {0, 0};
    std::mutex budget_mu;  // (the ranks of a multi-GPU stream plan from their own threads)
    uint32_t last_passes = 0;
    int direct_tail = 1;  // kmp_ctx_set_direct_tail: the fused tail writes its edges in place
    int flat_heavy = 1;   // kmp_ctx_set_flat_heavy: passes expand frequent k-mers by rows
    uint64_t last_windows = 0;  // kmp_ctx_last_tail_windows
    // kmp_ctx_set_rows: the rows kmp_pairs_stream covers ([0, 0): all) — a process's share of a
    // multi-process split (one process per GPU)
    uint32_t rows_lo = 0, rows_hi = 0;
    // kmp_pairs_multi_k: per k, the sets (scores), a workspace (front kept across passes) and
    // the pass's edges; the merged list
    using KSet = kmp_kset;
    std::vector<std::unique_ptr<KSet>> ksets;
    DevBuf mscore, mwk, mscratch;
    // multi-GPU (kmp_ctx_create_multi): the ranks of the row split and the gather's transport
    std::vector<std::unique_ptr<kmp_rank>> ranks;
    std::unique_ptr<kmp::Transport> transport;
    uint64_t split_cap = 0;   // k-mer split: keys per exchange region (learned per batch)
    const char* last_split = "";  // the flow of the last multi-GPU kmp_pairs: "kmer" or "rows"
    bool split_rows = false;  // the batch spills frequent k-mers: the row split
    ~kmp_ctx() {
        ranks.clear();
        (void)hipSetDevice(device);
        ksets.clear();
        transport.reset();
        (void)hipSetDevice(device);
        kmp_postings_destroy(postings);
        kmp_mphf_free(rep_mphf);
    }
};


namespace {

// the context's error text; the ranks of a multi-GPU stream report from their own threads
void note_error(kmp_ctx* c, const std::string& msg, bool keep_first) {
    std::lock_guard<std::mutex> lk(c->err_mu);
    if (!keep_first || c->err.empty()) c->err = msg;
}

int fail(kmp_ctx* c, int status, const char* fmt, ...) {
    if (c) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        std::vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        note_error(c, buf, false);
    }
    return status;
}

#define KMP_HIP(ctx, expr)                                                                   \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return fail((ctx), e_ == hipErrorOutOfMemory ? KMP_ENOMEM : KMP_EDEVICE, "%s: %s", \
                        #expr, hipGetErrorString(e_));                                       \
    } while (0)

#define KMP_TRY(ctx, expr)                                                                    \
    do {                                                                                      \
        int s_ = (expr);                                                                      \
        if (s_ != KMP_OK) {                                                                   \
            note_error((ctx), std::string(#expr) + ": " + kmp_status_string(s_), true);       \
            return s_;                                                                        \
        }                                                                                     \
    } while (0)

int use_device(kmp_ctx* c) {
    KMP_HIP(c, hipSetDevice(c->device));
    return KMP_OK;
}

uint64_t protein_len(const kmp_ctx* c, uint32_t p) { return c->h_off[p + 1] - c->h_off[p]; }

// canonical order (tiles: device sort; postings: already sorted), copy out, scores, counters
// The host pass over a returned edge list (bounds check of every device edge, score fill, the
// n_align / sum_w_diff counters), split over the context's host threads: at config 5 the list
// holds ~5e8 edges and one thread spent seconds here.
struct EdgeScan {
    uint64_t nalign = 0, wdiff = 0, bad = ~0ull;
};
template <class F>
EdgeScan scan_edges(uint64_t count, int threads, F body) {
    const uint64_t kMinPer = 1u << 20;
    int t = (int)std::min<uint64_t>(std::max(threads, 1), std::max<uint64_t>(1, count / kMinPer));
    std::vector<EdgeScan> part(t);
    auto run = [&](int r) {
        const uint64_t a = count * r / t, b = count * (r + 1) / t;
        EdgeScan& s = part[r];
        for (uint64_t i = a; i < b; ++i)
            if (!body(i, s)) {
                s.bad = i;
                return;
            }
    };
    run_parts(t, run);
    EdgeScan out;
    for (const EdgeScan& s : part) {
        out.nalign += s.nalign;
        out.wdiff += s.wdiff;
        out.bad = std::min(out.bad, s.bad);
    }
    return out;
}

// scored: the BLOSUM scores are in c->escore as u32 (the scored reduction); otherwise a BLOSUM
// call computes them here per edge (edge_blosum_device: the tiles and set-postings engines)
int finish_edges(kmp_ctx* c, const kmp_pair_opts& o, uint64_t count, bool needs_sort, kmp_edges** out,
                 bool scored = false) {
    if (needs_sort) {
        const uint64_t tmp = kmp_dev_sort_edges_tmp_bytes(count, c->n);
        KMP_HIP(c, c->sort_tmp.reserve(tmp));
        KMP_TRY(c, kmp_dev_sort_edges(c->ep.as<uint32_t>(), c->eq.as<uint32_t>(), c->ew.as<uint32_t>(), count, c->n,
                                      c->sort_tmp.p, c->sort_tmp.bytes, c->stream));
    }
    std::unique_ptr<kmp_edges> e(new (std::nothrow) kmp_edges);
    if (!e) return fail(c, KMP_ENOMEM, "edges");
    e->p.resize(count);
    e->q.resize(count);
    e->w.resize(count);
    if (count) {
        KMP_HIP(c, hipMemcpyAsync(e->p.data(), c->ep.p, count * 4, hipMemcpyDeviceToHost, c->stream));
        KMP_HIP(c, hipMemcpyAsync(e->q.data(), c->eq.p, count * 4, hipMemcpyDeviceToHost, c->stream));
        KMP_HIP(c, hipMemcpyAsync(e->w.data(), c->ew.p, count * 4, hipMemcpyDeviceToHost, c->stream));
    }
    hvec<uint32_t> iscore;  // scored: the u32 scores, converted below
    if (o.score == KMP_SCORE_BLOSUM && count && scored) {
        iscore.resize(count);
        KMP_HIP(c, hipMemcpyAsync(iscore.data(), c->escore.p, count * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                  c->stream));
    } else if (o.score == KMP_SCORE_BLOSUM && count) {
        KMP_HIP(c, c->escore.reserve(count * sizeof(float)));
        e->score.resize(count);
        KMP_TRY(c, edge_blosum_device(c->rep.as<uint32_t>(), c->rep_len.as<uint32_t>(), c->off.as<uint64_t>(),
                                      c->ep.as<uint32_t>(), c->eq.as<uint32_t>(), c->ew.as<uint32_t>(), count,
                                      c->k_sets, c->escore.as<float>(), c->stream));
        KMP_HIP(c, hipMemcpyAsync(e->score.data(), c->escore.p, count * sizeof(float), hipMemcpyDeviceToHost,
                                  c->stream));
    }
    KMP_HIP(c, hipStreamSynchronize(c->stream));
    e->score.resize(count);
    kmp_edges* E = e.get();
    const EdgeScan sc = scan_edges(count, c->threads, [&](uint64_t i, EdgeScan& s) {
        const uint32_t p = E->p[i], q = E->q[i], w = E->w[i];
        if (p >= q || q >= c->n) return false;
        if (c->h_cls[p] != c->h_cls[q]) s.wdiff += w;
        if (w > o.align_threshold) ++s.nalign;
        if (o.score == KMP_SCORE_JACCARD) {
            const uint64_t uni = (uint64_t)c->h_set_len[p] + c->h_set_len[q] - w;
            E->score[i] = uni ? (float)w / (float)uni : 0.0f;  // exact operands (< 2^24), one rounding
        } else if (o.score == KMP_SCORE_BLOSUM) {
            if (scored) E->score[i] = (float)iscore[i];  // an integer below 2^24: exact
        } else {
            E->score[i] = (float)w;
        }
        return true;
    });
    if (sc.bad != ~0ull)
        return fail(c, KMP_EDEVICE, "device edge %llu = (%u, %u) is not a pair of the batch",
                    (unsigned long long)sc.bad, E->p[sc.bad], E->q[sc.bad]);
    c->counters.n_edges = count;
    c->counters.n_align = sc.nalign;
    c->counters.sum_w_diff = sc.wdiff;
    *out = e.release();
    return KMP_OK;
}


// the repeat MPHF and code/df by id (main.rs:127-149,187-193), from a df pass that keeps its runs
int ensure_repeat_index(kmp_ctx* c) {
    if (c->rep_index) return KMP_OK;
    DfCounters dc{};
    uint32_t *uniq = nullptr, *counts = nullptr;
    KMP_TRY(c, device_df_counters(c->set.as<uint32_t>(), c->h_set_len.data(), c->h_off.data(), c->off.as<uint64_t>(),
                                  c->n, c->k_sets, c->stream, &dc, c->err, &uniq, &counts));
    kmp_mphf* m = nullptr;
    uint32_t *cb = nullptr, *db = nullptr;
    uint64_t R = 0;
    const int rc = repeat_mphf_build(uniq, counts, dc.distinct, 3.0, c->stream, &m, &cb, &db, &R);
    if (uniq) (void)hipFree(uniq);
    if (counts) (void)hipFree(counts);
    if (rc != KMP_OK) return fail(c, rc, "repeat MPHF build: %s", kmp_status_string(rc));
    c->rep_mphf = m;
    c->n_repeat = R;
    c->code_by_id.adopt(cb, R * 4);
    c->df_by_id.adopt(db, R * 4);
    c->rep_index = true;
    return KMP_OK;
}

int ensure_hash_kmers(kmp_ctx* c) {
    KMP_TRY(c, ensure_repeat_index(c));
    if (c->hash_kmers) return KMP_OK;
    uint32_t* ids = nullptr;
    const int rc = hash_kmers_device(c->rep_mphf, c->res.as<uint8_t>(), c->off.as<uint64_t>(), c->h_off.data(), c->n,
                                     c->k_sets, c->code_by_id.as<uint32_t>(), c->n_repeat, c->stream, &ids, c->h_hk_off);
    if (rc != KMP_OK) return fail(c, rc, "hash k-mers: %s", kmp_status_string(rc));
    c->hk_ids.adopt(ids, c->h_hk_off.back() * 4);
    c->hash_kmers = true;
    return KMP_OK;
}

// copy `total` u32 from device to a caller buffer with the cap / EOVERFLOW convention
int copy_out_u32(kmp_ctx* c, const uint32_t* src, uint64_t total, uint32_t* out, uint64_t cap, uint64_t* n) {
    *n = total;
    if (cap < total) return KMP_EOVERFLOW;
    if (total == 0) return KMP_OK;
    if (!out) return fail(c, KMP_EINVAL, "out is NULL");
    KMP_HIP(c, hipMemcpyAsync(out, src, total * 4, hipMemcpyDeviceToHost, c->stream));
    KMP_HIP(c, hipStreamSynchronize(c->stream));
    return KMP_OK;
}

int repeat_prologue(kmp_ctx* c, const void* n) {
    if (!c || !n) return KMP_EINVAL;
    c->err.clear();
    if (!c->k_sets) return fail(c, KMP_ESTATE, "kmp_build_sets first");
    KMP_TRY(c, use_device(c));
    return KMP_OK;
}

}  // namespace

extern "C" {

int kmp_version(void) { return KMP_ABI_VERSION; }

const char* kmp_status_string(int s) {
    switch (s) {
        case KMP_OK: return "ok";
        case KMP_EINVAL: return "invalid argument";
        case KMP_ENOMEM: return "out of memory";
        case KMP_EDEVICE: return "device error";
        case KMP_ERCCL: return "collective error";
        case KMP_EOVERFLOW: return "buffer too small";
        case KMP_ESTATE: return "call out of order";
        case KMP_EIO: return "i/o error";
        default: return "unknown status";
    }
}

void kmp_pair_opts_default(kmp_pair_opts* o) {
    if (!o) return;
    o->min_shared = 1;
    o->require_class_diff = 1;
    o->align_threshold = 10;
    o->score = KMP_SCORE_COUNT;
    o->engine = KMP_ENGINE_AUTO;
}

int kmp_ctx_create(kmp_ctx** out, int device, int cpu_threads) {
    if (!out) return KMP_EINVAL;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return KMP_EDEVICE;
    if (device < 0 || device >= count) return KMP_EINVAL;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return KMP_EDEVICE;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return KMP_EDEVICE;  // kernels are gfx950-only
    kmp_ctx* c = new (std::nothrow) kmp_ctx;
    if (!c) return KMP_ENOMEM;
    c->device = device;
    c->threads = cpu_threads < 1 ? 1 : cpu_threads;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return KMP_EDEVICE;
    }
    *out = c;
    return KMP_OK;
}

int kmp_ctx_create_multi(kmp_ctx** out, int n_gpus, const int* devices, int cpu_threads) {
    if (!out || n_gpus < 1 || n_gpus > 64) return KMP_EINVAL;
    *out = nullptr;
    std::vector<int> dev(n_gpus);
    for (int g = 0; g < n_gpus; ++g) dev[g] = devices ? devices[g] : g;
    kmp_ctx* c = nullptr;
    int rc = kmp_ctx_create(&c, dev[0], cpu_threads);
    if (rc != KMP_OK) return rc;
    std::unique_ptr<kmp_ctx> guard(c);
    bool distinct = true;
    for (int g = 0; g < n_gpus; ++g) {
        for (int h = 0; h < g; ++h) distinct &= dev[h] != dev[g];
        if (g) {  // every device must pass the same checks as the first
            kmp_ctx* probe = nullptr;
            rc = kmp_ctx_create(&probe, dev[g], 1);
            if (rc != KMP_OK) return rc;
            kmp_ctx_destroy(probe);
        }
        std::unique_ptr<kmp_rank> r(new (std::nothrow) kmp_rank);
        if (!r) return KMP_ENOMEM;
        r->device = dev[g];
        if (hipSetDevice(dev[g]) != hipSuccess) return KMP_EDEVICE;
        if (g == 0) {
            r->stream = c->stream;
        } else {
            if (hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) != hipSuccess) return KMP_EDEVICE;
            r->own_stream = true;
        }
        if (kmp_postings_create(&r->ws) != KMP_OK) return KMP_ENOMEM;
        c->ranks.push_back(std::move(r));
    }
    (void)hipSetDevice(dev[0]);
    if (n_gpus > 1) {
        if (distinct) {
            c->transport = kmp::make_rccl_transport(dev, &c->err);
            if (!c->transport) return KMP_ERCCL;
        } else {
            c->transport = kmp::make_copy_transport(dev);
        }
    }
    *out = guard.release();
    return KMP_OK;
}

int kmp_ctx_gpus(const kmp_ctx* c) { return c ? std::max<int>(1, (int)c->ranks.size()) : 0; }

const char* kmp_ctx_transport(const kmp_ctx* c) {
    if (!c) return "none";
    return c->transport ? c->transport->name() : "local";
}

const char* kmp_ctx_last_split(const kmp_ctx* c) { return c ? c->last_split : ""; }

void kmp_ctx_destroy(kmp_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* kmp_last_error(const kmp_ctx* c) { return c ? c->err.c_str() : "null context"; }

int kmp_load_proteins(kmp_ctx* c, const uint8_t* residues, const uint64_t* offsets, uint32_t n,
                      const uint16_t* class_id) {
    if (!c) return KMP_EINVAL;
    c->err.clear();
    if (!offsets) return fail(c, KMP_EINVAL, "offsets is NULL");
    for (uint32_t p = 0; p < n; ++p)
        if (offsets[p + 1] < offsets[p]) return fail(c, KMP_EINVAL, "offsets not monotone at %u", p);
    const uint64_t total = offsets[n] - offsets[0];
    if (total && !residues) return fail(c, KMP_EINVAL, "residues is NULL");
    KMP_TRY(c, use_device(c));
    c->loaded = false;
    c->k_codes = c->k_sets = 0;
    c->drop_repeat_index();
    c->budget[0] = c->budget[1] = 0;
    c->n = n;
    c->total_res = total;
    c->h_off.resize(n + 1);
    c->max_len = 0;
    for (uint32_t p = 0; p <= n; ++p) c->h_off[p] = offsets[p] - offsets[0];
    for (uint32_t p = 0; p < n; ++p) {
        const uint64_t L = c->h_off[p + 1] - c->h_off[p];
        if (L > 0xFFFFFFFFull) return fail(c, KMP_EINVAL, "protein %u longer than 2^32 residues", p);
        c->max_len = std::max<uint32_t>(c->max_len, (uint32_t)L);
    }
    c->h_cls.assign(n, 0);
    if (class_id) std::copy(class_id, class_id + n, c->h_cls.begin());
    KMP_HIP(c, c->res.reserve(total + 16));
    KMP_HIP(c, c->off.reserve((n + 1) * sizeof(uint64_t)));
    KMP_HIP(c, c->cls.reserve((n + 1) * sizeof(uint16_t)));
    if (total) KMP_HIP(c, hipMemcpyAsync(c->res.p, residues + offsets[0], total, hipMemcpyHostToDevice, c->stream));
    KMP_HIP(c, hipMemcpyAsync(c->off.p, c->h_off.data(), (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
    if (n) KMP_HIP(c, hipMemcpyAsync(c->cls.p, c->h_cls.data(), n * sizeof(uint16_t), hipMemcpyHostToDevice, c->stream));
    KMP_HIP(c, hipStreamSynchronize(c->stream));
    for (size_t g = 1; g < c->ranks.size(); ++g) {  // multi-GPU: every rank holds the whole batch
        kmp_rank& r = *c->ranks[g];
        KMP_HIP(c, hipSetDevice(r.device));
        KMP_HIP(c, r.res.reserve(total + 16));
        KMP_HIP(c, r.off.reserve((n + 1) * sizeof(uint64_t)));
        KMP_HIP(c, r.cls.reserve((n + 1) * sizeof(uint16_t)));
        if (total) KMP_HIP(c, hipMemcpyAsync(r.res.p, residues + offsets[0], total, hipMemcpyHostToDevice, r.stream));
        KMP_HIP(c, hipMemcpyAsync(r.off.p, c->h_off.data(), (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, r.stream));
        if (n) KMP_HIP(c, hipMemcpyAsync(r.cls.p, c->h_cls.data(), n * sizeof(uint16_t), hipMemcpyHostToDevice, r.stream));
        KMP_HIP(c, hipStreamSynchronize(r.stream));
    }
    KMP_TRY(c, use_device(c));
    c->counters = kmp_counters{};
    c->counters.n_proteins = n;
    c->loaded = true;
    c->split_cap = 0;
    c->split_rows = false;
    return KMP_OK;
}

int kmp_extract(kmp_ctx* c, int k) {
    if (!c) return KMP_EINVAL;
    c->err.clear();
    if (!c->loaded) return fail(c, KMP_ESTATE, "kmp_load_proteins first");
    if (k < 1 || k > kMaxK) return fail(c, KMP_EINVAL, "k must be in 1..7, got %d", k);
    KMP_TRY(c, use_device(c));
    KMP_HIP(c, c->codes.reserve(kmp_set_capacity(c->n, c->total_res) * sizeof(uint32_t)));
    KMP_TRY(c, kmp_dev_extract(c->res.as<uint8_t>(), c->off.as<uint64_t>(), c->n, k, c->codes.as<uint32_t>(), c->stream));
    KMP_HIP(c, hipStreamSynchronize(c->stream));
    c->k_codes = k;
    return KMP_OK;
}

int kmp_get_kmers(kmp_ctx* c, uint32_t p, uint32_t* out, uint64_t cap, uint64_t* n) {
    if (!c || !n) return KMP_EINVAL;
    c->err.clear();
    if (!c->k_codes) return fail(c, KMP_ESTATE, "kmp_extract first");
    if (p >= c->n) return fail(c, KMP_EINVAL, "protein %u out of range", p);
    const uint64_t nw = n_windows(protein_len(c, p), c->k_codes);
    *n = nw;
    if (cap < nw) return KMP_EOVERFLOW;
    if (nw == 0) return KMP_OK;
    if (!out) return fail(c, KMP_EINVAL, "out is NULL");
    KMP_TRY(c, use_device(c));
    KMP_HIP(c, hipMemcpyAsync(out, c->codes.as<uint32_t>() + set_base(c->h_off[p], p), nw * sizeof(uint32_t),
                              hipMemcpyDeviceToHost, c->stream));
    KMP_HIP(c, hipStreamSynchronize(c->stream));
    return KMP_OK;
}

int kmp_build_sets(kmp_ctx* c, int k) {
    if (!c) return KMP_EINVAL;
    c->err.clear();
    if (!c->loaded) return fail(c, KMP_ESTATE, "kmp_load_proteins first");
    if (k < 1 || k > kMaxK) return fail(c, KMP_EINVAL, "k must be in 1..7, got %d", k);
    KMP_TRY(c, use_device(c));
    c->k_sets = 0;
    c->drop_repeat_index();
    // the multi-GPU flow and exchange capacity are learned per (batch, k): a k that spills
    // frequent k-mers must not pin the row split on another k of the same batch
    c->split_cap = 0;
    c->split_rows = false;
    const uint64_t capacity = kmp_set_capacity(c->n, c->total_res);
    const uint64_t words = kmp_dev_repeat_bitmap_words(k);
    KMP_HIP(c, c->set.reserve(capacity * sizeof(uint32_t)));
    KMP_HIP(c, c->rep.reserve(capacity * sizeof(uint32_t)));
    KMP_HIP(c, c->set_len.reserve((c->n + 1) * sizeof(uint32_t)));
    KMP_HIP(c, c->rep_len.reserve((c->n + 1) * sizeof(uint32_t)));
    KMP_HIP(c, c->bits.reserve(2 * words * sizeof(uint32_t)));
    const bool long_path = n_windows(c->max_len, k) > KMP_LDS_SORT_MAX;
    if (long_path) KMP_HIP(c, c->scratch.reserve(capacity * sizeof(uint32_t)));
    KMP_TRY(c, kmp_dev_build_sets(c->res.as<uint8_t>(), c->off.as<uint64_t>(), c->n, k, c->max_len,
                                  c->set.as<uint32_t>(), c->set_len.as<uint32_t>(),
                                  long_path ? c->scratch.as<uint32_t>() : nullptr, c->stream));
    KMP_TRY(c, kmp_dev_filter_repeats(c->set.as<uint32_t>(), c->set_len.as<uint32_t>(), c->off.as<uint64_t>(), c->n,
                                      k, c->bits.as<uint32_t>(), c->rep.as<uint32_t>(), c->rep_len.as<uint32_t>(),
                                      c->stream));
    c->h_set_len.resize(c->n);
    c->h_rep_len.resize(c->n);
    if (c->n) {
        KMP_HIP(c, hipMemcpyAsync(c->h_set_len.data(), c->set_len.p, c->n * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                  c->stream));
        KMP_HIP(c, hipMemcpyAsync(c->h_rep_len.data(), c->rep_len.p, c->n * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                  c->stream));
    }
    KMP_HIP(c, hipStreamSynchronize(c->stream));
    kmp_counters& ct = c->counters;
    ct = kmp_counters{};
    ct.n_proteins = c->n;
    for (uint32_t p = 0; p < c->n; ++p) {
        ct.n_windows += n_windows(protein_len(c, p), k);
        ct.sum_S += c->h_set_len[p];
    }
    // device df over all sets (main.rs:77-149): distinct / repeat / Σ C(df,2) / max df
    DfCounters dc{};
    KMP_TRY(c, device_df_counters(c->set.as<uint32_t>(), c->h_set_len.data(), c->h_off.data(), c->off.as<uint64_t>(), c->n, k, c->stream, &dc,
                                  c->err));
    ct.distinct = dc.distinct;
    ct.repeat = dc.repeat;
    ct.sum_cdf2 = dc.sum_cdf2;
    ct.max_df = dc.max_df;
    c->k_sets = k;
    return KMP_OK;
}

int kmp_get_set(kmp_ctx* c, uint32_t p, uint32_t* out, uint64_t cap, uint64_t* n) {
    if (!c || !n) return KMP_EINVAL;
    c->err.clear();
    if (!c->k_sets) return fail(c, KMP_ESTATE, "kmp_build_sets first");
    if (p >= c->n) return fail(c, KMP_EINVAL, "protein %u out of range", p);
    const uint64_t m = c->h_set_len[p];
    *n = m;
    if (cap < m) return KMP_EOVERFLOW;
    if (m == 0) return KMP_OK;
    if (!out) return fail(c, KMP_EINVAL, "out is NULL");
    KMP_TRY(c, use_device(c));
    KMP_HIP(c, hipMemcpyAsync(out, c->set.as<uint32_t>() + set_base(c->h_off[p], p), m * sizeof(uint32_t),
                              hipMemcpyDeviceToHost, c->stream));
    KMP_HIP(c, hipStreamSynchronize(c->stream));
    return KMP_OK;
}

int kmp_counters_get(kmp_ctx* c, kmp_counters* out) {
    if (!c || !out) return KMP_EINVAL;
    *out = c->counters;
    return KMP_OK;
}

int kmp_get_df(kmp_ctx* c, uint32_t* df_by_id, uint64_t cap, uint64_t* n) {
    KMP_TRY(c, repeat_prologue(c, n));
    KMP_TRY(c, ensure_repeat_index(c));
    return copy_out_u32(c, c->df_by_id.as<uint32_t>(), c->n_repeat, df_by_id, cap, n);
}

int kmp_get_repeat_codes(kmp_ctx* c, uint32_t* code_by_id, uint64_t cap, uint64_t* n) {
    KMP_TRY(c, repeat_prologue(c, n));
    KMP_TRY(c, ensure_repeat_index(c));
    return copy_out_u32(c, c->code_by_id.as<uint32_t>(), c->n_repeat, code_by_id, cap, n);
}

int kmp_get_hash_kmers(kmp_ctx* c, uint32_t p, uint32_t* ids, uint64_t cap, uint64_t* n) {
    KMP_TRY(c, repeat_prologue(c, n));
    if (p >= c->n) return fail(c, KMP_EINVAL, "protein %u out of range", p);
    KMP_TRY(c, ensure_hash_kmers(c));
    const uint64_t b = c->h_hk_off[p];
    return copy_out_u32(c, c->hk_ids.as<uint32_t>() + b, c->h_hk_off[p + 1] - b, ids, cap, n);
}

int kmp_get_hash_kmers_all(kmp_ctx* c, uint32_t* ids, uint64_t cap, uint64_t* offsets, uint64_t* n) {
    KMP_TRY(c, repeat_prologue(c, n));
    KMP_TRY(c, ensure_hash_kmers(c));
    if (offsets) std::copy(c->h_hk_off.begin(), c->h_hk_off.end(), offsets);
    return copy_out_u32(c, c->hk_ids.as<uint32_t>(), c->h_hk_off.back(), ids, cap, n);
}

int kmp_repeat_mphf(kmp_ctx* c, const kmp_mphf** out) {
    KMP_TRY(c, repeat_prologue(c, out));
    KMP_TRY(c, ensure_repeat_index(c));
    *out = c->rep_mphf;
    return KMP_OK;
}

int kmp_mphf_build(kmp_ctx* c, const uint32_t* keys, uint64_t n, double gamma, kmp_mphf** out) {
    if (!c || !out) return KMP_EINVAL;
    c->err.clear();
    *out = nullptr;
    if (n && !keys) return fail(c, KMP_EINVAL, "keys is NULL");
    KMP_TRY(c, use_device(c));
    DevBuf d;
    KMP_HIP(c, d.reserve(n * 4));
    if (n) KMP_HIP(c, hipMemcpyAsync(d.p, keys, n * 4, hipMemcpyHostToDevice, c->stream));
    const int rc = mphf_build_device(d.as<uint32_t>(), n, gamma, c->stream, out);
    if (rc == KMP_EINVAL) return fail(c, rc, "MPHF build: gamma must be in [1, 100] and keys distinct");
    if (rc != KMP_OK) return fail(c, rc, "MPHF build: %s", kmp_status_string(rc));
    return KMP_OK;
}

// Bounded-memory passes over the rows (Σ C(df,2) runs to 10^10-10^11
// (k-mer, pair) incidences, far more than one pass of pair keys can hold).  A pair belongs to
// its smaller protein, so row p carries about (N - 1 - p) units of the pair mass; the planner
// measures incidences per unit on each pass (the first pass is a probe of N/256 rows) and sizes
// the next pass to 3/4 of the key budget with the densest rate seen so far.
struct PassPlan {
    uint32_t n;
    double budget;
    double density = -1.0;
    uint32_t max_rows = 0xFFFFFFFFu;  // rows one call may cover (scored: kmp_dev_rows_max)
    uint32_t end = 0xFFFFFFFFu;       // the last row + 1 (a rank's share; default n)
    double mass(uint32_t a, uint32_t b) const {  // Σ_{p in [a, b)} (n - 1 - p)
        const double A = a, B = b, N = n;
        return (B - A) * (N - 1) - (B * (B - 1) - A * (A - 1)) / 2;
    }
    // the end of the pass starting at a: always > a while a < end (a zero max_rows is rejected
    // by the callers before planning: a batch too large for the scored key)
    uint32_t next(uint32_t a) const {
        const uint32_t e = std::min(end, n);
        if (a >= e) return e;
        if (max_rows == 0) return a;
        const uint32_t lim = (uint32_t)std::min<uint64_t>(e, (uint64_t)a + max_rows);
        if (density < 0) return std::min<uint32_t>(lim, a + std::max<uint32_t>(1, n / 256));
        const double target = 0.75 * budget / std::max(density, 1e-12);
        if (mass(a, e) <= target) return lim;
        uint32_t lo = a + 1, hi = e;
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            if (mass(a, mid) >= target) hi = mid;
            else lo = mid + 1;
        }
        return std::min(lo, lim);
    }
    void seen(uint32_t a, uint32_t b, uint64_t inc) {
        const double m = mass(a, b);
        if (m > 0) density = std::max(density, inc / m);
    }
};

constexpr uint64_t kPassSlots = 1ull << 26;  // batches above ~67M windows run in passes by default

uint64_t pass_budget_free(kmp_ctx* c, bool fused);
uint64_t pass_budget(kmp_ctx* c, bool fused = false) {
    if (c->pass_keys) return c->pass_keys;
    std::lock_guard<std::mutex> lk(c->budget_mu);
    uint64_t& b = c->budget[fused ? 1 : 0];
    // (a budget re-read per call planned 378 passes on the second stream of config 5, whose free
    // memory the first stream's cached buffers hold: 6.44 s against 5.82 s for the first call's 58)
    if (!b) b = pass_budget_free(c, fused);
    return b;
}
uint64_t pass_budget_free(kmp_ctx* c, bool fused) {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) fr = 16ull << 30;
    // device memory per pair key of a pass: ~96 B when dense row blocks take the tagged-key sort
    // (shard regions 8, row-block keys 8, staged runs 12, the sort's keys 48 and run arrays 12,
    // slack; half the free memory kept back); the fused tail, whose dense blocks are cut into LDS
    // sub-blocks, sizes its buffers once per stream (kmp_postings_set_shard_floor): shard regions
    // of the smaller k with a 2x fullest-region allowance 20, row-block and sub-block keys 8,
    // staged runs 20, the pass's edges 17 (edges / incidences ~0.63), +25 % growth headroom:
    // ~86 B per key of the 3/4-budget pass, so 3/4 of the free memory over 90 B leaves ~40 % free;
    // the in-place reduce (kmp_ctx_set_direct_tail, default) stages nothing: ~56 B, budget 66 B
    if (fused)
        return std::max<uint64_t>(1u << 20, std::min<uint64_t>(fr / 4 * 3 / (c->direct_tail ? 66 : 90), 3ull << 30));
    return std::max<uint64_t>(1u << 20, std::min<uint64_t>(fr / 2 / 96, 3ull << 30));
}

// the batch and stream a pass runs on: the context's (nullptr) or a rank's copy
struct Lane {
    const uint8_t* res;
    const uint64_t* off;
    const uint16_t* cls;
    hipStream_t stream;
};

// three (scored: four) u32 edge arrays of cap entries, grown to want entries keeping their first
// keep entries
int grow_edges(kmp_ctx* c, DevBuf& ep, DevBuf& eq, DevBuf& ew, uint64_t& cap, uint64_t want, uint64_t keep,
               DevBuf* es = nullptr, hipStream_t stream = nullptr) {
    if (!stream) stream = c->stream;
    uint64_t have = ep.p && eq.p && ew.p ? std::min({ep.bytes, eq.bytes, ew.bytes}) / 4 : 0;
    if (es) have = es->p ? std::min<uint64_t>(have, es->bytes / 4) : 0;
    if (have >= want) {
        cap = have;
        return KMP_OK;
    }
    for (DevBuf* b : {&ep, &eq, &ew, es}) {
        if (!b) continue;
        DevBuf nb;
        KMP_HIP(c, nb.reserve(want * sizeof(uint32_t)));
        if (keep) KMP_HIP(c, hipMemcpyAsync(nb.p, b->p, keep * 4, hipMemcpyDeviceToDevice, stream));
        KMP_HIP(c, hipStreamSynchronize(stream));
        b->swap(nb);
    }
    cap = want;
    return KMP_OK;
}

// rows [a, b) with workspace ws (front reuse on) into (ep, eq, ew[, es]) from entry off on; the
// buffers grow, keeping [0, off), when the call reports an overflow.  es: the scored reduction
// (BLOSUM), its u32 scores into es
int rows_into(kmp_ctx* c, kmp_postings* ws, int k, const kmp_pair_opts& o, uint32_t a, uint32_t b, DevBuf& ep,
              DevBuf& eq, DevBuf& ew, uint64_t& cap, uint64_t off, uint64_t* ne, kmp_postings_stats* st,
              DevBuf* es = nullptr, const Lane* lane = nullptr) {
    const uint64_t slots = kmp_set_capacity(c->n, c->total_res);
    const Lane L = lane ? *lane : Lane{c->res.as<uint8_t>(), c->off.as<uint64_t>(), c->cls.as<uint16_t>(), c->stream};
    KMP_TRY(c, grow_edges(c, ep, eq, ew, cap, std::max<uint64_t>(cap, off + (1u << 16)), off, es, L.stream));
    for (int attempt = 0; attempt < 3; ++attempt) {
        uint64_t m = 0;
        const int rc =
            es ? kmp_dev_pairs_rows_scored(ws, L.res, L.off, L.cls, c->n, k, slots, 0xFFFFFFFFu, o.min_shared,
                                           o.require_class_diff, a, b, ep.as<uint32_t>() + off, eq.as<uint32_t>() + off,
                                           ew.as<uint32_t>() + off, es->as<uint32_t>() + off, cap - off, &m, st,
                                           L.stream)
               : kmp_dev_pairs_rows(ws, L.res, L.off, L.cls, c->n, k, slots, 0xFFFFFFFFu, o.min_shared,
                                    o.require_class_diff, a, b, ep.as<uint32_t>() + off, eq.as<uint32_t>() + off,
                                    ew.as<uint32_t>() + off, cap - off, &m, st, L.stream);
        if (rc == KMP_EOVERFLOW) {
            KMP_TRY(c, grow_edges(c, ep, eq, ew, cap, off + m + m / 8 + 1024, off, es, L.stream));
            continue;
        }
        if (rc != KMP_OK) return fail(c, rc, "rows [%u, %u): %s", a, b, kmp_status_string(rc));
        *ne = m;
        return KMP_OK;
    }
    return fail(c, KMP_EDEVICE, "rows [%u, %u): edge count unstable across reruns", a, b);
}

// single GPU, residue path, in passes: the pass edges land behind each other in the context's
// buffers (already canonical: passes are consecutive row ranges)
int pass_pairs(kmp_ctx* c, const kmp_pair_opts& o, uint64_t* count, bool scored) {
    KMP_TRY(c, kmp_postings_set_reuse(c->postings, 1));
    PassPlan plan{c->n, (double)pass_budget(c)};
    if (scored) plan.max_rows = kmp_dev_rows_max(c->n, 1);
    uint64_t off = 0;
    uint32_t passes = 0;
    int rc = KMP_OK;
    for (uint32_t a = 0; a < c->n && rc == KMP_OK;) {
        const uint32_t b = plan.next(a);
        if (b <= a) return fail(c, KMP_EINVAL, "pass planner: no row fits one pass at N = %u", c->n);
        kmp_postings_stats st{};
        uint64_t ne = 0;
        rc = rows_into(c, c->postings, c->k_sets, o, a, b, c->ep, c->eq, c->ew, c->edge_cap, off, &ne, &st,
                       scored ? &c->escore : nullptr);
        plan.seen(a, b, st.incidences);
        if (rc == KMP_OK && getenv("KMP_DEBUG_PASSES")) {  // each pass's edges: rows in [a, b), p < q
            std::vector<uint32_t> hp(ne), hq(ne);
            (void)hipMemcpy(hp.data(), c->ep.as<uint32_t>() + off, ne * 4, hipMemcpyDeviceToHost);
            (void)hipMemcpy(hq.data(), c->eq.as<uint32_t>() + off, ne * 4, hipMemcpyDeviceToHost);
            uint64_t bad = 0, first = ~0ull;
            for (uint64_t i = 0; i < ne; ++i)
                if (hp[i] < a || hp[i] >= b || hp[i] >= hq[i] || (i && hp[i] < hp[i - 1])) {
                    if (!bad++) first = i;
                }
            fprintf(stderr, "kmp: pass %u rows [%u, %u) edges %llu at %llu, incidences %llu, bad %llu first %lld\n",
                    passes, a, b, (unsigned long long)ne, (unsigned long long)off,
                    (unsigned long long)st.incidences, (unsigned long long)bad, (long long)first);
            if (bad)
                for (uint64_t i = first > 3 ? first - 3 : 0; i < std::min<uint64_t>(ne, first + 4); ++i)
                    fprintf(stderr, "kmp:   %llu: (%u, %u)\n", (unsigned long long)i, hp[i], hq[i]);
        }
        off += ne;
        a = b;
        ++passes;
    }
    (void)kmp_postings_set_reuse(c->postings, 0);
    c->last_passes = passes;
    *count = off;
    return rc;
}

// Multi-GPU: every rank's edges of its rows (kmp_row_split) into its own (ep, eq, ew), then the
// transport gathers them into the context's buffers in rank order (the canonical list).
//   k-mer split (default): phase 1 on every rank (kmp_dev_split_expand, enqueued from this
//     thread), the all-to-all of the routed pair keys, the flags reduced on the host (a rerun grows
//     the capacities identically on every rank), phase 2 on every rank (kmp_dev_split_edges, one
//     host thread per rank: it synchronises);
//   row split: every rank groups every k-mer and expands its rows (kmp_dev_pairs_rows, one host
//     thread per rank), for batches whose frequent k-mers spill.
constexpr int kSplitFallback = -1;

static int split_rank_edges(kmp_ctx* c, const kmp_pair_opts& o, const std::vector<uint32_t>& start,
                            std::vector<uint64_t>& cnt) {
    const uint32_t G = (uint32_t)c->ranks.size();
    const uint64_t slots = kmp_set_capacity(c->n, c->total_res);
    uint64_t cap = c->split_cap ? c->split_cap : std::max<uint64_t>(4096, c->total_res / 4 / ((uint64_t)G * G));
    std::vector<uint32_t> learn(KMP_SPLIT_FLAGS, 0), fl(KMP_SPLIT_FLAGS, 0);
    bool have_learn = false;
    auto rank_buf = [&](uint32_t g) -> const uint8_t* { return (g ? c->ranks[g]->res : c->res).as<uint8_t>(); };
    for (int attempt = 0; attempt < 6; ++attempt) {
        std::vector<const char*> sendp(G);
        std::vector<char*> recvp(G);
        std::vector<hipStream_t> streams(G);
        for (uint32_t g = 0; g < G; ++g) {
            kmp_rank& r = *c->ranks[g];
            KMP_HIP(c, hipSetDevice(r.device));
            KMP_HIP(c, r.send.reserve((uint64_t)G * cap * 8));
            KMP_HIP(c, r.recv.reserve((uint64_t)G * cap * 8));
            KMP_HIP(c, r.sflags.reserve(KMP_SPLIT_FLAGS * sizeof(uint32_t)));
            KMP_HIP(c, r.sstats.reserve(8 * sizeof(unsigned long long)));
            const uint64_t* off = (g ? r.off : c->off).as<uint64_t>();
            const uint16_t* cls = (g ? r.cls : c->cls).as<uint16_t>();
            const int rc = kmp_dev_split_expand(r.ws, rank_buf(g), off, cls, c->n, c->k_sets, slots, 0xFFFFFFFFu,
                                                o.require_class_diff, g, G, cap, have_learn ? learn.data() : nullptr,
                                                r.send.as<unsigned long long>(), r.sflags.as<uint32_t>(),
                                                r.sstats.as<unsigned long long>(), r.stream);
            if (rc == KMP_ESTATE) return kSplitFallback;
            if (rc != KMP_OK) return fail(c, rc, "rank %u: k-mer split expand: %s", g, kmp_status_string(rc));
            sendp[g] = static_cast<const char*>(r.send.p);
            recvp[g] = static_cast<char*>(r.recv.p);
            streams[g] = r.stream;
        }
        std::string err;
        const int rc = c->transport->alltoall(sendp, recvp, cap * 8, streams, &err);
        if (rc != KMP_OK) return fail(c, rc, "%s", err.c_str());
        std::fill(fl.begin(), fl.end(), 0u);
        for (uint32_t g = 0; g < G; ++g) {  // the flags, reduced (max) over the ranks
            kmp_rank& r = *c->ranks[g];
            uint32_t h[KMP_SPLIT_FLAGS];
            KMP_HIP(c, hipSetDevice(r.device));
            KMP_HIP(c, hipMemcpyAsync(h, r.sflags.p, sizeof h, hipMemcpyDeviceToHost, r.stream));
            KMP_HIP(c, hipStreamSynchronize(r.stream));
            for (int i = 0; i < KMP_SPLIT_FLAGS; ++i) fl[i] = std::max(fl[i], h[i]);
        }
        if (fl[KMP_SPLIT_CLASS]) return kSplitFallback;
        if (fl[KMP_SPLIT_RERUN] || fl[KMP_SPLIT_HEAVY]) {  // HEAVY: a rank spilled; every rank's heavy path on
            learn = fl;
            have_learn = true;
            if (fl[KMP_SPLIT_MAX_PART] > cap) cap = fl[KMP_SPLIT_MAX_PART] + fl[KMP_SPLIT_MAX_PART] / 16 + 1024;
            continue;
        }
        c->split_cap = cap;
        std::vector<int> status(G, KMP_OK);
        auto work = [&](uint32_t g) {
            kmp_rank& r = *c->ranks[g];
            if (hipSetDevice(r.device) != hipSuccess) {
                status[g] = KMP_EDEVICE;
                return;
            }
            if (r.cap == 0) r.cap = std::max<uint64_t>(1u << 16, 4ull * c->n / G);
            for (int a = 0; a < 3; ++a) {
                if (r.ep.reserve(r.cap * 4) != hipSuccess || r.eq.reserve(r.cap * 4) != hipSuccess ||
                    r.ew.reserve(r.cap * 4) != hipSuccess) {
                    status[g] = KMP_ENOMEM;
                    return;
                }
                uint64_t ne = 0;
                status[g] = kmp_dev_split_edges(r.ws, r.recv.as<unsigned long long>(), (uint64_t)G * cap, c->n,
                                                start[g], start[g + 1], o.min_shared, r.ep.as<uint32_t>(),
                                                r.eq.as<uint32_t>(), r.ew.as<uint32_t>(), r.cap, &ne, r.stream);
                cnt[g] = ne;
                if (status[g] != KMP_EOVERFLOW) break;
                r.cap = ne + ne / 8 + 1024;
            }
        };
        run_parts((int)G, [&](int g) { work((uint32_t)g); });
        KMP_TRY(c, use_device(c));
        for (uint32_t g = 0; g < G; ++g)
            if (status[g] != KMP_OK)
                return fail(c, status[g], "rank %u (device %d, rows [%u, %u)): k-mer split edges: %s", g,
                            c->ranks[g]->device, start[g], start[g + 1], kmp_status_string(status[g]));
        return KMP_OK;
    }
    return fail(c, KMP_EDEVICE, "k-mer split: capacities unstable across reruns");
}

static int rows_rank_edges(kmp_ctx* c, const kmp_pair_opts& o, const std::vector<uint32_t>& start,
                           std::vector<uint64_t>& cnt) {
    const uint32_t G = (uint32_t)c->ranks.size();
    const uint64_t slots = kmp_set_capacity(c->n, c->total_res);
    std::vector<int> status(G, KMP_OK);
    auto work = [&](uint32_t g) {
        kmp_rank& r = *c->ranks[g];
        if (hipSetDevice(r.device) != hipSuccess) {
            status[g] = KMP_EDEVICE;
            return;
        }
        const uint8_t* res = (g ? r.res : c->res).as<uint8_t>();
        const uint64_t* off = (g ? r.off : c->off).as<uint64_t>();
        const uint16_t* cls = (g ? r.cls : c->cls).as<uint16_t>();
        if (r.cap == 0) r.cap = std::max<uint64_t>(1u << 16, 4ull * c->n / G);
        for (int attempt = 0; attempt < 3; ++attempt) {
            if (r.ep.reserve(r.cap * 4) != hipSuccess || r.eq.reserve(r.cap * 4) != hipSuccess ||
                r.ew.reserve(r.cap * 4) != hipSuccess) {
                status[g] = KMP_ENOMEM;
                return;
            }
            uint64_t ne = 0;
            status[g] = kmp_dev_pairs_rows(r.ws, res, off, cls, c->n, c->k_sets, slots, 0xFFFFFFFFu, o.min_shared,
                                           o.require_class_diff, start[g], start[g + 1], r.ep.as<uint32_t>(),
                                           r.eq.as<uint32_t>(), r.ew.as<uint32_t>(), r.cap, &ne, nullptr, r.stream);
            cnt[g] = ne;
            if (status[g] != KMP_EOVERFLOW) break;
            r.cap = ne + ne / 8 + 1024;
        }
        if (status[g] == KMP_OK && cnt[g] > r.cap) status[g] = KMP_EDEVICE;
    };
    run_parts((int)G, [&](int g) { work((uint32_t)g); });
    KMP_TRY(c, use_device(c));
    for (uint32_t g = 0; g < G; ++g)
        if (status[g] != KMP_OK)
            return fail(c, status[g], "rank %u (device %d, rows [%u, %u)): %s", g, c->ranks[g]->device, start[g],
                        start[g + 1], kmp_status_string(status[g]));
    return KMP_OK;
}

static int multi_pairs(kmp_ctx* c, const kmp_pair_opts& o, uint64_t* count) {
    const uint32_t G = (uint32_t)c->ranks.size();
    std::vector<uint32_t> start(G + 1);
    kmp_row_split(c->n, G, start.data());
    std::vector<uint64_t> cnt(G, 0);
    int rc = kSplitFallback;
    if (!c->split_rows) rc = split_rank_edges(c, o, start, cnt);
    if (rc == kSplitFallback) {
        c->split_rows = true;  // for this batch
        std::fill(cnt.begin(), cnt.end(), 0ull);
        rc = rows_rank_edges(c, o, start, cnt);
    }
    if (rc != KMP_OK) return rc;
    c->last_split = c->split_rows ? "rows" : "kmer";
    uint64_t total = 0;
    for (uint64_t x : cnt) total += x;
    if (total > c->edge_cap) c->edge_cap = total + total / 8 + 1024;
    KMP_HIP(c, c->ep.reserve(c->edge_cap * sizeof(uint32_t)));
    KMP_HIP(c, c->eq.reserve(c->edge_cap * sizeof(uint32_t)));
    KMP_HIP(c, c->ew.reserve(c->edge_cap * sizeof(uint32_t)));
    std::vector<kmp::EdgeArrays> src(G);
    std::vector<hipStream_t> streams(G);
    for (uint32_t g = 0; g < G; ++g) {
        kmp_rank& r = *c->ranks[g];
        src[g] = {r.ep.as<uint32_t>(), r.eq.as<uint32_t>(), r.ew.as<uint32_t>()};
        streams[g] = r.stream;
    }
    std::string err;
    rc = c->transport->gather(src, {c->ep.as<uint32_t>(), c->eq.as<uint32_t>(), c->ew.as<uint32_t>()}, cnt, streams,
                              &err);
    KMP_TRY(c, use_device(c));
    if (rc != KMP_OK) return fail(c, rc, "%s", err.c_str());
    *count = total;
    return KMP_OK;
}

int kmp_pairs(kmp_ctx* c, const kmp_pair_opts* opts, kmp_edges** out) {
    if (!c || !out) return KMP_EINVAL;
    *out = nullptr;
    c->err.clear();
    if (!c->k_sets) return fail(c, KMP_ESTATE, "kmp_build_sets first");
    kmp_pair_opts o;
    kmp_pair_opts_default(&o);
    if (opts) o = *opts;
    if (o.score != KMP_SCORE_COUNT && o.score != KMP_SCORE_JACCARD && o.score != KMP_SCORE_BLOSUM)
        return fail(c, KMP_EINVAL, "unknown score %d", o.score);
    if (o.engine < KMP_ENGINE_AUTO || o.engine > KMP_ENGINE_RESIDUES) return fail(c, KMP_EINVAL, "unknown engine %d", o.engine);
    KMP_TRY(c, use_device(c));
    if (c->edge_cap == 0) c->edge_cap = std::max<uint64_t>(1u << 20, 4ull * c->n);
    unsigned long long count = 0;
    if (c->ranks.size() > 1 && (o.engine == KMP_ENGINE_AUTO || o.engine == KMP_ENGINE_RESIDUES)) {
        uint64_t total = 0;
        KMP_TRY(c, multi_pairs(c, o, &total));
        return finish_edges(c, o, total, false, out);
    }
    c->last_passes = 1;
    if (o.engine != KMP_ENGINE_TILES) {
        if (!c->postings) KMP_TRY(c, kmp_postings_create(&c->postings));
        const uint64_t slots = kmp_set_capacity(c->n, c->total_res);
        const bool residues = o.engine == KMP_ENGINE_AUTO || o.engine == KMP_ENGINE_RESIDUES;
        // the score summed in the reduction; a batch too large for the scored key (N >= 2^24:
        // kmp_dev_rows_max 0) takes the unscored reduction and the per-edge BLOSUM pass of finish_edges
        const bool scored = residues && o.score == KMP_SCORE_BLOSUM && kmp_dev_rows_max(c->n, 1) > 0;
        if (residues && (c->pass_keys || slots > kPassSlots || (scored && kmp_dev_rows_max(c->n, 1) < c->n))) {
            uint64_t total = 0;
            KMP_TRY(c, pass_pairs(c, o, &total, scored));
            return finish_edges(c, o, total, false, out, scored);
        }
        if (scored) {
            uint64_t total = 0;
            KMP_TRY(c, kmp_postings_set_reuse(c->postings, 0));
            KMP_TRY(c, rows_into(c, c->postings, c->k_sets, o, 0, c->n, c->ep, c->eq, c->ew, c->edge_cap, 0, &total,
                                 nullptr, &c->escore));
            return finish_edges(c, o, total, false, out, true);
        }
        bool ok = false;
        for (int attempt = 0; attempt < 3 && !ok; ++attempt) {
            KMP_HIP(c, c->ep.reserve(c->edge_cap * sizeof(uint32_t)));
            KMP_HIP(c, c->eq.reserve(c->edge_cap * sizeof(uint32_t)));
            KMP_HIP(c, c->ew.reserve(c->edge_cap * sizeof(uint32_t)));
            uint64_t ne = 0;
            const int st =
                (o.engine == KMP_ENGINE_RESIDUES || o.engine == KMP_ENGINE_AUTO)
                    ? kmp_dev_pairs_residues(c->postings, c->res.as<uint8_t>(), c->off.as<uint64_t>(),
                                             c->cls.as<uint16_t>(), c->n, c->k_sets, slots, 0xFFFFFFFFu,
                                             o.min_shared, o.require_class_diff, c->ep.as<uint32_t>(),
                                             c->eq.as<uint32_t>(), c->ew.as<uint32_t>(), c->edge_cap, &ne, nullptr,
                                             c->stream)
                    : kmp_dev_pairs_postings(c->postings, c->set.as<uint32_t>(), c->set_len.as<uint32_t>(),
                                             c->off.as<uint64_t>(), c->cls.as<uint16_t>(), c->n, c->k_sets, slots,
                                             0xFFFFFFFFu, o.min_shared, o.require_class_diff, c->ep.as<uint32_t>(),
                                             c->eq.as<uint32_t>(), c->ew.as<uint32_t>(), c->edge_cap, &ne, nullptr,
                                             c->stream);
            count = ne;
            if (st == KMP_EOVERFLOW) {  // the buffers were too small: grow them and rerun
                c->edge_cap = ne + ne / 8 + 1024;
                continue;
            }
            if (st != KMP_OK) return fail(c, st, "postings engine: %s", kmp_status_string(st));
            ok = count <= c->edge_cap;
        }
        if (!ok) return fail(c, KMP_EDEVICE, "edge count unstable across reruns");
        return finish_edges(c, o, count, false, out);
    }

    // plan (host): dense CSR offsets, row tiles x column chunks, XCD-aware launch order
    // sets longer than a row tile take the long-protein kernel; they are planned with length 0
    std::vector<uint32_t> plan_len(c->h_rep_len);
    std::vector<uint32_t> long_ids;
    for (uint32_t p = 0; p < c->n; ++p)
        if (plan_len[p] > kTileCap) {
            long_ids.push_back(p);
            plan_len[p] = 0;
        }
    std::vector<uint64_t> dense_off(c->n + 1);
    uint64_t n_plan = 0, n_items = 0;
    int st = kmp_plan_pairs(plan_len.data(), c->n, 0, dense_off.data(), nullptr, 0, &n_plan);
    if (st != KMP_OK && st != KMP_EOVERFLOW)
        return fail(c, st, "planner: a repeat-filtered set exceeds %u k-mers", kTileCap);
    std::vector<kmp_work_item> plan(n_plan);
    KMP_TRY(c, kmp_plan_pairs(plan_len.data(), c->n, 0, dense_off.data(), plan.data(), n_plan, &n_plan));
    kmp_order_items_xcd(plan.data(), n_plan, nullptr, 0, &n_items);
    std::vector<kmp_work_item> items(n_items);
    KMP_TRY(c, kmp_order_items_xcd(plan.data(), n_plan, items.data(), n_items, &n_items));
    KMP_HIP(c, c->items.reserve(std::max<uint64_t>(1, n_items) * sizeof(kmp_work_item)));
    KMP_HIP(c, c->dense_off.reserve((c->n + 1) * sizeof(uint64_t)));
    KMP_HIP(c, c->dense.reserve(std::max<uint64_t>(1, dense_off[c->n]) * sizeof(uint32_t)));
    KMP_HIP(c, hipMemcpyAsync(c->dense_off.p, dense_off.data(), (c->n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice,
                              c->stream));
    if (n_items)
        KMP_HIP(c, hipMemcpyAsync(c->items.p, items.data(), n_items * sizeof(kmp_work_item), hipMemcpyHostToDevice,
                                  c->stream));
    KMP_HIP(c, c->long_ids.reserve(std::max<size_t>(1, long_ids.size()) * sizeof(uint32_t)));
    if (!long_ids.empty())
        KMP_HIP(c, hipMemcpyAsync(c->long_ids.p, long_ids.data(), long_ids.size() * sizeof(uint32_t),
                                  hipMemcpyHostToDevice, c->stream));
    KMP_TRY(c, kmp_dev_pack_dense(c->rep.as<uint32_t>(), c->off.as<uint64_t>(), c->dense_off.as<uint64_t>(), c->n,
                                  c->dense.as<uint32_t>(), c->stream));
    KMP_HIP(c, c->ecount.reserve(sizeof(unsigned long long)));
    bool ok = false;
    for (int attempt = 0; attempt < 3 && !ok; ++attempt) {
        KMP_HIP(c, c->ep.reserve(c->edge_cap * sizeof(uint32_t)));
        KMP_HIP(c, c->eq.reserve(c->edge_cap * sizeof(uint32_t)));
        KMP_HIP(c, c->ew.reserve(c->edge_cap * sizeof(uint32_t)));
        KMP_HIP(c, hipMemsetAsync(c->ecount.p, 0, sizeof(unsigned long long), c->stream));
        KMP_TRY(c, kmp_dev_pairs(c->dense.as<uint32_t>(), c->dense_off.as<uint64_t>(), c->cls.as<uint16_t>(), c->n,
                                 c->items.as<kmp_work_item>(), n_items, kmp_pair_col_window(plan_len.data(), c->n),
                                 o.min_shared, o.require_class_diff, c->ep.as<uint32_t>(), c->eq.as<uint32_t>(),
                                 c->ew.as<uint32_t>(), c->edge_cap, c->ecount.as<unsigned long long>(), c->stream));
        KMP_TRY(c, kmp_dev_pairs_long(c->rep.as<uint32_t>(), c->rep_len.as<uint32_t>(), c->off.as<uint64_t>(),
                                      c->cls.as<uint16_t>(), c->n, c->long_ids.as<uint32_t>(),
                                      (uint32_t)long_ids.size(), o.min_shared, o.require_class_diff,
                                      c->ep.as<uint32_t>(), c->eq.as<uint32_t>(), c->ew.as<uint32_t>(), c->edge_cap,
                                      c->ecount.as<unsigned long long>(), c->stream));
        KMP_HIP(c, hipMemcpyAsync(&count, c->ecount.p, sizeof count, hipMemcpyDeviceToHost, c->stream));
        KMP_HIP(c, hipStreamSynchronize(c->stream));
        ok = count <= c->edge_cap;  // else the buffers grow and the kernels rerun
        if (!ok) c->edge_cap = count + count / 8 + 1024;
    }
    if (!ok) return fail(c, KMP_EDEVICE, "edge count unstable across reruns");
    return finish_edges(c, o, count, true, out);
}

int kmp_edges_count(const kmp_edges* e, uint64_t* n) {
    if (!e || !n) return KMP_EINVAL;
    *n = e->p.size();
    return KMP_OK;
}

int kmp_edges_get(const kmp_edges* e, uint32_t* p, uint32_t* q, uint32_t* w, float* score, uint64_t cap,
                  uint64_t* n) {
    if (!e || !n) return KMP_EINVAL;
    const uint64_t m = e->p.size();
    *n = m;
    if (cap < m) return KMP_EOVERFLOW;
    if (p) std::copy(e->p.begin(), e->p.end(), p);
    if (q) std::copy(e->q.begin(), e->q.end(), q);
    if (w) std::copy(e->w.begin(), e->w.end(), w);
    if (score) std::copy(e->score.begin(), e->score.end(), score);
    return KMP_OK;
}

}  // extern "C" (templates below)

// ---- streamed passes (kmp_pairs_stream) and the config-5 union (kmp_pairs_multi_k) ----
// Config 5 of SURVEY.md §8d: w_k computed independently for each k; an edge is emitted when any
// w_k >= min_shared (and, with require_class_diff, the classes differ).  Each k's sets are built
// and kept, each k gets its own workspace whose front (keys, grouping, heavy compaction) is kept
// across the passes, and the rows run in passes (one when the batch is small): per pass, every
// k's edges of the pass's rows (kmp_dev_pairs_rows[_scored]: BLOSUM summed inside the reduction)
// and, for nk > 1, the device union (kmp_merge.hip): w = Σ_k w_k, score = Σ_k score_k.  The pass's
// chunk is summarised on the device (kmp_stream.hip) and handed to the sink; the buffers are then
// reused, so the whole list is never resident.  The context's sets are left at the last k.

static int opts_multi(kmp_ctx* c, const kmp_pair_opts* opts, const int* ks, uint32_t nk, kmp_pair_opts* o) {
    if (!ks || nk < 1 || nk > KMP_MULTI_K_MAX) return fail(c, KMP_EINVAL, "need 1 to %d values of k", KMP_MULTI_K_MAX);
    kmp_pair_opts_default(o);
    if (opts) *o = *opts;
    if (o->score == KMP_SCORE_JACCARD) return fail(c, KMP_EINVAL, "JACCARD does not sum over k");
    if (o->score != KMP_SCORE_COUNT && o->score != KMP_SCORE_BLOSUM) return fail(c, KMP_EINVAL, "unknown score %d", o->score);
    if (o->engine != KMP_ENGINE_AUTO && o->engine != KMP_ENGINE_RESIDUES)
        return fail(c, KMP_EINVAL, "streamed pairs run the residues engine (engine %d)", o->engine);
    for (uint32_t j = 0; j < nk; ++j) {
        if (ks[j] < 1 || ks[j] > kMaxK) return fail(c, KMP_EINVAL, "k = %d", ks[j]);
        for (uint32_t i = 0; i < j; ++i)
            if (ks[i] == ks[j]) return fail(c, KMP_EINVAL, "k = %d twice", ks[j]);
    }
    if (!c->loaded) return fail(c, KMP_ESTATE, "kmp_load_proteins first");
    return KMP_OK;
}

// every k's sets, stashed in its KSet (the caller swaps the last k's back: restore_ksets)
static int prepare_ksets(kmp_ctx* c, const int* ks, uint32_t nk) {
    while (c->ksets.size() < nk) c->ksets.emplace_back(new kmp_ctx::KSet);
    for (uint32_t j = 0; j < nk; ++j) {
        KMP_TRY(c, kmp_build_sets(c, ks[j]));
        kmp_ctx::KSet& s = *c->ksets[j];
        s.k = ks[j];
        s.set.swap(c->set);
        s.set_len.swap(c->set_len);
        s.rep.swap(c->rep);
        s.rep_len.swap(c->rep_len);
        s.h_set_len.swap(c->h_set_len);
        s.h_rep_len.swap(c->h_rep_len);
        if (!s.ws) KMP_TRY(c, kmp_postings_create(&s.ws));
        KMP_TRY(c, kmp_postings_set_reuse(s.ws, 1));
    }
    return KMP_OK;
}

static void restore_ksets(kmp_ctx* c, uint32_t nk) {  // the context keeps the last k's sets
    kmp_ctx::KSet& s = *c->ksets[nk - 1];
    s.set.swap(c->set);
    s.set_len.swap(c->set_len);
    s.rep.swap(c->rep);
    s.rep_len.swap(c->rep_len);
    s.h_set_len.swap(c->h_set_len);
    s.h_rep_len.swap(c->h_rep_len);
    for (uint32_t j = 0; j < nk; ++j) (void)kmp_postings_set_reuse(c->ksets[j]->ws, 0);
}

// pinned host staging of a chunk (a host sink)
struct HostChunk {
    void* p = nullptr;
    size_t bytes = 0;
    ~HostChunk() {
        if (p) (void)hipHostFree(p);
    }
    hipError_t reserve(size_t b) {
        if (b <= bytes && p) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        bytes = 0;
        hipError_t e = hipHostMalloc(&p, b ? b : 16, hipHostMallocDefault);
        if (e == hipSuccess) bytes = b ? b : 16;
        return e;
    }
};

// One lane of the streamed passes: a device, its copy of the batch and stream, the rows it owns,
// per-k workspaces and pass edges, the merged arrays (nk > 1) and its summary accumulators.
struct StreamLane {
    Lane L;
    int device = 0;
    uint32_t rank = 0, row_lo = 0, row_hi = 0;
    uint32_t share = 1;  // lanes streaming on this lane's device at once: they split its memory budget
    std::vector<std::unique_ptr<kmp_kset>>* ks = nullptr;
    DevBuf *ep = nullptr, *eq = nullptr, *ew = nullptr, *mscore = nullptr, *mwk = nullptr, *mscratch = nullptr;
    kmp::DigestAcc* acc = nullptr;
    uint64_t incidences = 0;
    uint32_t passes = 0;
    float stage_ms[4] = {0, 0, 0, 0};  // kmp_stream_summary.stage_ms
    uint64_t windows = 0;              // sub-blocks the in-place reduce took in windows
};

// two HIP events around the summary kernel of a pass (lane-local, created on first use)
struct EventPair {
    hipEvent_t a = nullptr, b = nullptr;
    ~EventPair() {
        if (a) (void)hipEventDestroy(a);
        if (b) (void)hipEventDestroy(b);
    }
    bool ready() { return (a || hipEventCreate(&a) == hipSuccess) && (b || hipEventCreate(&b) == hipSuccess); }
    float ms() {
        float t = 0.f;
        const bool ok = hipEventElapsedTime(&t, a, b) == hipSuccess;
        if (!ok) (void)hipGetLastError();
        return ok ? t : 0.f;
    }
};

// The passes of the lane's rows: for each, the chunk on the lane's device, its summary into
// lane.acc (device), then on_chunk(chunk).  The lane's workspaces keep their front across passes.
template <class OnChunk>
static int stream_passes(kmp_ctx* c, const kmp_pair_opts& o, const int* ks, uint32_t nk, StreamLane& ln,
                         OnChunk on_chunk) {
    auto& kv = *ln.ks;
    while (kv.size() < nk) kv.emplace_back(new kmp_kset);
    for (uint32_t j = 0; j < nk; ++j) {
        kv[j]->k = ks[j];
        if (!kv[j]->ws) KMP_TRY(c, kmp_postings_create(&kv[j]->ws));
        KMP_TRY(c, kmp_postings_set_reuse(kv[j]->ws, 1));
        KMP_TRY(c, kmp_postings_set_timing(kv[j]->ws, 1));  // stage times of the summary
        KMP_TRY(c, kmp_postings_set_direct(kv[j]->ws, c->direct_tail));
        KMP_TRY(c, kmp_postings_set_flat_heavy(kv[j]->ws, c->flat_heavy));
        // every pass lies in the lane's rows: the flat index covers only them (a rank's share)
        KMP_TRY(c, kmp_postings_set_row_span(kv[j]->ws, ln.row_lo, ln.row_hi));
    }
    EventPair dev;
    if (!dev.ready()) return fail(c, KMP_EDEVICE, "events");
    const bool blosum = o.score == KMP_SCORE_BLOSUM;
    const uint64_t slots = kmp_set_capacity(c->n, c->total_res);
    // the budget comes from the device's free memory unless set (kmp_ctx_set_pass_keys): virtual
    // ranks on one device (devices = [0, 0, ...]) take an equal part of it each
    PassPlan plan{c->n, (double)(c->pass_keys ? pass_budget(c, nk == 2) : pass_budget(c, nk == 2) / std::max(1u, ln.share))};
    plan.end = ln.row_hi;
    const bool fused = nk == 2;  // both k reduced together (kmp_dev_pairs_rows_multi): no merge
    if (fused) plan.max_rows = kmp_dev_rows_max(c->n, 2);
    else if (blosum) plan.max_rows = kmp_dev_rows_max(c->n, 1);
    if (plan.max_rows == 0)
        return fail(c, KMP_EINVAL, "%s at N = %u: the %s key needs more than 31 bits (N < 2^%u)",
                    fused ? "combined k" : "BLOSUM stream", c->n, fused ? "fused k-bit + score" : "scored",
                    fused ? 23u : 24u);
    if (!c->pass_keys && slots <= kPassSlots && plan.max_rows >= ln.row_hi - ln.row_lo)
        plan.density = 0;  // small batch: one pass
    const hipStream_t st = ln.L.stream;
    if (fused && plan.density != 0) {
        // the smaller k carries most of a pass's incidences: its regions (and the fused tail's
        // staging) sized for the planned pass, 3/4 of the budget
        const uint32_t big = ks[0] <= ks[1] ? 0 : 1;
        KMP_TRY(c, kmp_postings_set_shard_floor(kv[big]->ws, (uint64_t)(0.75 * plan.budget)));
        KMP_TRY(c, kmp_postings_set_shard_floor(kv[1 - big]->ws, 0));
    }
    uint64_t mcap = 0;
    double edge_ratio = 1.0;  // the largest edges / incidences of a pass so far (after the first)
    bool ratio_seen = false;
    int rc = KMP_OK;
    for (uint32_t a = ln.row_lo; a < ln.row_hi && rc == KMP_OK;) {
        const uint32_t b = plan.density == 0 ? ln.row_hi : plan.next(a);
        if (b <= a) return fail(c, KMP_EINVAL, "pass planner: no row fits one pass at N = %u", c->n);
        MergeIn in{};
        in.nk = nk;
        uint64_t total = 0, inc = 0;
        kmp_edge_chunk ch{};
        if (fused) {
            // p q w (ln.ep/eq/ew), score (ln.mscore), w0 | w1 (ln.mwk), grown on overflow
            kmp_postings* wsp[2] = {kv[0]->ws, kv[1]->ws};
            // edges <= incidences: size the arrays from the densest incidence rate seen times the
            // largest edges-per-incidence ratio seen (+10 %; an overflow reruns the pass)
            // a growth takes a quarter of headroom: reallocating six multi-GB arrays (a synchronous
            // free and a fresh allocation each) stalled the device for seconds per growth
            double est = plan.density > 0 ? plan.density * plan.mass(a, b) * std::min(1.0, edge_ratio * 1.1) : 0.0;
            // once a pass has measured the edge ratio: the largest pass the planner aims for (3/4 of
            // the key budget), so the arrays are allocated once instead of growing pass by pass
            if (ratio_seen && plan.density > 0) est = std::max(est, 0.75 * plan.budget * std::min(1.0, edge_ratio * 1.1) * 1.1);
            if (est + 4096 > (double)mcap) mcap = std::max<uint64_t>((uint64_t)est + 4096, mcap + mcap / 4);
            for (int attempt = 0; attempt < 3; ++attempt) {
                if (!mcap || !ln.mwk->p) mcap = std::max<uint64_t>(mcap, 1u << 20);
                uint64_t cap3 = 0;
                if ((rc = grow_edges(c, *ln.ep, *ln.eq, *ln.ew, cap3, mcap, 0, ln.mscore, st)) != KMP_OK) break;
                if (ln.mwk->reserve(2 * mcap * 4) != hipSuccess) {
                    rc = fail(c, KMP_ENOMEM, "pass weights (%llu)", (unsigned long long)mcap);
                    break;
                }
                kmp_postings_stats pst{};
                rc = kmp_dev_pairs_rows_multi(wsp, ks, 2, ln.L.res, ln.L.off, ln.L.cls, c->n, slots, o.min_shared,
                                              o.require_class_diff, a, b, ln.ep->as<uint32_t>(), ln.eq->as<uint32_t>(),
                                              ln.ew->as<uint32_t>(), ln.mscore->as<uint32_t>(), ln.mwk->as<uint32_t>(),
                                              ln.mwk->as<uint32_t>() + mcap, mcap, &total, &pst, st);
                if (pst.incidences) inc = pst.incidences;  // (a re-emit after an overflow expands nothing)
                for (int i = 0; i < 3; ++i) ln.stage_ms[i] += std::max(0.f, pst.stage_ms[i]);
                if (rc == KMP_EOVERFLOW) {
                    mcap = total + total / 8 + 1024;
                    rc = KMP_OK;
                    continue;
                }
                if (rc != KMP_OK) rc = fail(c, rc, "rows [%u, %u) of k = %d + %d: %s", a, b, ks[0], ks[1],
                                            kmp_status_string(rc));
                break;
            }
            if (rc == KMP_OK && total > mcap) rc = fail(c, KMP_EDEVICE, "rows [%u, %u): edge count unstable", a, b);
            if (rc != KMP_OK) break;
            ln.windows += kmp_postings_last_overflow_blocks(kv[0]->ws);
            ch.n = total;
            ch.p = ln.ep->as<uint32_t>();
            ch.q = ln.eq->as<uint32_t>();
            ch.w = ln.ew->as<uint32_t>();
            ch.score = blosum ? ln.mscore->as<uint32_t>() : ch.w;
            ch.wk[0] = ln.mwk->as<uint32_t>();
            ch.wk[1] = ln.mwk->as<uint32_t>() + mcap;
        }
        for (uint32_t j = 0; j < nk && rc == KMP_OK && !fused; ++j) {
            kmp_kset& s = *kv[j];
            kmp_postings_stats pst{};
            uint64_t ne = 0;
            // nk > 1: every w_j >= 1 (the true w_j of each kept pair), min_shared applied by the merge
            kmp_pair_opts oj = o;
            if (nk > 1) oj.min_shared = 1;
            rc = rows_into(c, s.ws, s.k, oj, a, b, s.ep, s.eq, s.ew, s.cap, 0, &ne, &pst, blosum ? &s.score : nullptr,
                           &ln.L);
            if (rc != KMP_OK) break;
            inc += pst.incidences;
            // stages 0-2 (keys, level 2, buckets + heavy) expand; 3-5 (partition, reduce, emit) reduce
            ln.stage_ms[j ? 1 : 0] += std::max(0.f, pst.stage_ms[0]) + std::max(0.f, pst.stage_ms[1]) +
                                      std::max(0.f, pst.stage_ms[2]);
            ln.stage_ms[2] += std::max(0.f, pst.stage_ms[3]) + std::max(0.f, pst.stage_ms[4]) +
                              std::max(0.f, pst.stage_ms[5]);
            in.p[j] = s.ep.as<uint32_t>();
            in.q[j] = s.eq.as<uint32_t>();
            in.w[j] = s.ew.as<uint32_t>();
            in.s[j] = blosum ? s.score.as<uint32_t>() : s.ew.as<uint32_t>();  // COUNT: the merge sums w
            in.off[j] = total;
            total += ne;
        }
        if (rc != KMP_OK) break;
        in.off[nk] = total;
        if (plan.density != 0) plan.seen(a, b, inc);
        if (inc) {
            const double ratio = (double)total / (double)inc;
            edge_ratio = ratio_seen ? std::max(edge_ratio, ratio) : ratio;
            ratio_seen = true;
        }
        ln.incidences += inc;
        ch.rank = ln.rank;
        ch.device = ln.device;
        ch.row_lo = a;
        ch.row_hi = b;
        ch.on_device = 1;
        if (fused) {
            // the chunk was filled by the fused reduction
        } else if (nk == 1) {
            kmp_kset& s = *kv[0];
            ch.n = total;
            ch.p = s.ep.as<uint32_t>();
            ch.q = s.eq.as<uint32_t>();
            ch.w = s.ew.as<uint32_t>();
            ch.score = in.s[0];
            ch.wk[0] = ch.w;
        } else {
            if (total > mcap || !ln.mwk->p) {  // merged arrays: p q w, score, wk (nk x mcap)
                mcap = total + total / 8 + (1u << 16);
                uint64_t cap3 = 0;
                if ((rc = grow_edges(c, *ln.ep, *ln.eq, *ln.ew, cap3, mcap, 0, nullptr, st)) != KMP_OK) break;
                if (ln.mscore->reserve(mcap * 4) != hipSuccess || ln.mwk->reserve((uint64_t)nk * mcap * 4) != hipSuccess) {
                    rc = fail(c, KMP_ENOMEM, "merged edge arrays (%llu)", (unsigned long long)mcap);
                    break;
                }
            }
            const uint64_t sb = merge_scratch_bytes(total);
            if (ln.mscratch->bytes < sb && ln.mscratch->reserve(sb) != hipSuccess) {
                rc = fail(c, KMP_ENOMEM, "merge scratch");
                break;
            }
            MergeOut mo{};
            mo.p = ln.ep->as<uint32_t>();
            mo.q = ln.eq->as<uint32_t>();
            mo.w = ln.ew->as<uint32_t>();
            mo.s = ln.mscore->as<uint32_t>();
            for (uint32_t j = 0; j < nk; ++j) mo.wk[j] = ln.mwk->as<uint32_t>() + j * mcap;
            mo.cap = mcap;
            mo.min_shared = std::max(1u, o.min_shared);
            uint64_t m = 0;
            rc = merge_edges_device(in, mo, ln.mscratch->p, ln.mscratch->bytes, &m, st);
            if (rc != KMP_OK) {
                rc = fail(c, rc, "merge: %s", kmp_status_string(rc));
                break;
            }
            ch.n = m;
            ch.p = mo.p;
            ch.q = mo.q;
            ch.w = mo.w;
            ch.score = mo.s;
            for (uint32_t j = 0; j < nk; ++j) ch.wk[j] = mo.wk[j];
        }
        kmp::DigestIn di{};
        di.p = ch.p;
        di.q = ch.q;
        di.w = ch.w;
        di.s = ch.score;
        di.w0 = ch.wk[0];
        di.n = ch.n;
        di.n_prot = c->n;
        di.row_lo = a;
        di.row_hi = b;
        di.cls = o.require_class_diff ? nullptr : ln.L.cls;
        di.align_threshold = o.align_threshold;
        if (hipEventRecord(dev.a, st) != hipSuccess || kmp::edge_digest_enqueue(di, ln.acc, st) != hipSuccess ||
            hipEventRecord(dev.b, st) != hipSuccess) {
            rc = fail(c, KMP_EDEVICE, "edge digest");
            break;
        }
        if (hipStreamSynchronize(st) != hipSuccess) {
            rc = fail(c, KMP_EDEVICE, "stream synchronise");
            break;
        }
        ln.stage_ms[3] += dev.ms();
        if (getenv("KMP_DEBUG")) {
            size_t fr = 0, tot = 0;
            (void)hipMemGetInfo(&fr, &tot);
            fprintf(stderr, "kmp: rank %u pass %u rows [%u, %u): %llu incidences, %llu edges, free %.1f GB\n", ln.rank,
                    ln.passes, a, b, (unsigned long long)inc, (unsigned long long)ch.n, fr / 1e9);
        }
        ++ln.passes;
        rc = on_chunk(ch);
        a = b;
    }
    for (uint32_t j = 0; j < nk; ++j) {
        (void)kmp_postings_set_reuse(kv[j]->ws, 0);
        (void)kmp_postings_set_timing(kv[j]->ws, 0);
        (void)kmp_postings_set_shard_floor(kv[j]->ws, 0);
        (void)kmp_postings_set_row_span(kv[j]->ws, 0, 0);
    }
    return rc;
}

// the context's lane (rank 0 of a multi-GPU context too): its batch, stream and buffers
static StreamLane ctx_lane(kmp_ctx* c, uint32_t lo, uint32_t hi, DevBuf& dacc) {
    StreamLane ln;
    ln.L = Lane{c->res.as<uint8_t>(), c->off.as<uint64_t>(), c->cls.as<uint16_t>(), c->stream};
    ln.device = c->device;
    ln.row_lo = lo;
    ln.row_hi = hi;
    ln.ks = &c->ksets;
    ln.ep = &c->ep;
    ln.eq = &c->eq;
    ln.ew = &c->ew;
    ln.mscore = &c->mscore;
    ln.mwk = &c->mwk;
    ln.mscratch = &c->mscratch;
    ln.acc = dacc.as<kmp::DigestAcc>();
    return ln;
}

// summary of the lanes' device accumulators (+ the counters the context reports)
static int finish_summary(kmp_ctx* c, const kmp_pair_opts& o, const std::vector<StreamLane*>& lanes,
                          kmp_stream_summary* out) {
    kmp_stream_summary sm{};
    bool bad = false;
    uint64_t windows = 0;
    for (StreamLane* ln : lanes) {
        kmp::DigestAcc h{};
        KMP_HIP(c, hipSetDevice(ln->device));
        KMP_HIP(c, hipMemcpyAsync(&h, ln->acc, sizeof h, hipMemcpyDeviceToHost, ln->L.stream));
        KMP_HIP(c, hipStreamSynchronize(ln->L.stream));
        for (int i = 0; i < KMP_DIGEST_SEGMENTS; ++i) {
            sm.seg_edges[i] += h.seg_edges[i];
            sm.seg_digest[i] += h.seg_digest[i];
            sm.n_edges += h.seg_edges[i];
            sm.digest += h.seg_digest[i];
        }
        sm.sum_w += h.tot[0];
        sm.sum_score += h.tot[1];
        sm.n_align += h.tot[2];
        sm.sum_w_diff += h.tot[3];
        sm.incidences += ln->incidences;
        sm.passes += ln->passes;
        for (int i = 0; i < 4; ++i) sm.stage_ms[i] += ln->stage_ms[i];
        windows += ln->windows;
        bad |= h.bad != 0;
    }
    c->last_windows = windows;
    KMP_TRY(c, use_device(c));
    // Σ w over class-differing pairs: every edge when the class filter is on
    if (o.require_class_diff) sm.sum_w_diff = sm.sum_w;
    sm.ordered = bad ? 0 : 1;
    c->last_passes = sm.passes;
    c->counters.n_edges = sm.n_edges;
    c->counters.n_align = sm.n_align;
    c->counters.sum_w_diff = sm.sum_w_diff;
    if (out) *out = sm;
    if (bad) return fail(c, KMP_EDEVICE, "a streamed chunk was not in canonical order inside its rows");
    return KMP_OK;
}

// host copies of a device chunk (p q w score, and the nk weights when nk > 1) for a host sink
static int chunk_to_host(kmp_ctx* c, const kmp_edge_chunk& ch, uint32_t nk, HostChunk& host, hipStream_t st,
                         kmp_edge_chunk* hc) {
    const uint32_t na = 4 + (nk > 1 ? nk : 0);
    if (host.reserve(std::max<uint64_t>(1, ch.n) * 4 * na) != hipSuccess) return fail(c, KMP_ENOMEM, "pinned chunk");
    uint32_t* hb = static_cast<uint32_t*>(host.p);
    const uint32_t* src[4 + KMP_MULTI_K_MAX] = {ch.p, ch.q, ch.w, ch.score, ch.wk[0], ch.wk[1], ch.wk[2], ch.wk[3]};
    for (uint32_t i = 0; i < na; ++i)
        if (ch.n && hipMemcpyAsync(hb + i * ch.n, src[i], ch.n * 4, hipMemcpyDeviceToHost, st) != hipSuccess)
            return fail(c, KMP_EDEVICE, "chunk copy");
    if (hipStreamSynchronize(st) != hipSuccess) return fail(c, KMP_EDEVICE, "chunk copy");
    *hc = ch;
    hc->on_device = 0;
    hc->p = hb;
    hc->q = hb + ch.n;
    hc->w = hb + 2 * ch.n;
    hc->score = hb + 3 * ch.n;
    for (uint32_t j = 0; j < KMP_MULTI_K_MAX; ++j) hc->wk[j] = j < nk ? (nk > 1 ? hb + (4 + j) * ch.n : hc->w) : nullptr;
    return KMP_OK;
}

// rows [lo, hi) cut into parts ranges of equal pair mass (a pair belongs to its smaller protein)
static std::vector<uint32_t> mass_split(uint32_t n, uint32_t lo, uint32_t hi, uint32_t parts) {
    PassPlan pm{n, 0.0};
    std::vector<uint32_t> start(parts + 1, lo);
    const double total = pm.mass(lo, hi);
    for (uint32_t d = 1; d < parts; ++d) {
        const double want = total * d / parts;
        uint32_t a = start[d - 1], b = hi;
        while (a < b) {
            const uint32_t mid = a + (b - a) / 2;
            if (pm.mass(lo, mid) >= want) b = mid;
            else a = mid + 1;
        }
        start[d] = a;
    }
    start[parts] = hi;
    return start;
}

// every rank streams its own rows (one host thread per rank); the sink is called under a mutex
static int multi_stream(kmp_ctx* c, const kmp_pair_opts& o, const int* ks, uint32_t nk, int sink_on_device,
                        kmp_edge_sink sink, void* user, kmp_stream_summary* summary, uint32_t lo, uint32_t hi) {
    const uint32_t G = (uint32_t)c->ranks.size();
    const std::vector<uint32_t> start =
        lo == 0 && hi == c->n ? [&] {
            std::vector<uint32_t> s(G + 1);
            kmp_row_split(c->n, G, s.data());
            return s;
        }()
                              : mass_split(c->n, lo, hi, G);
    std::vector<StreamLane> lanes(G);
    std::vector<HostChunk> host(G);
    std::vector<int> status(G, KMP_OK);
    std::mutex sink_mu;
    int sink_rc = KMP_OK;
    for (uint32_t g = 0; g < G; ++g) {
        kmp_rank& r = *c->ranks[g];
        KMP_HIP(c, hipSetDevice(r.device));
        KMP_HIP(c, r.dacc.reserve(sizeof(kmp::DigestAcc)));
        KMP_HIP(c, hipMemsetAsync(r.dacc.p, 0, sizeof(kmp::DigestAcc), r.stream));
        StreamLane& ln = lanes[g];
        if (g == 0) {
            ln = ctx_lane(c, start[0], start[1], r.dacc);
        } else {
            ln.L = Lane{r.res.as<uint8_t>(), r.off.as<uint64_t>(), r.cls.as<uint16_t>(), r.stream};
            ln.device = r.device;
            ln.row_lo = start[g];
            ln.row_hi = start[g + 1];
            ln.ks = &r.ksets;
            ln.ep = &r.ep;
            ln.eq = &r.eq;
            ln.ew = &r.ew;
            ln.mscore = &r.mscore;
            ln.mwk = &r.mwk;
            ln.mscratch = &r.mscratch;
            ln.acc = r.dacc.as<kmp::DigestAcc>();
        }
        ln.rank = g;
    }
    for (uint32_t g = 0; g < G; ++g)
        for (uint32_t h = 0; h < G; ++h)
            if (h != g && lanes[h].device == lanes[g].device) ++lanes[g].share;
    run_parts((int)G, [&](int gi) {
        const uint32_t g = (uint32_t)gi;
        StreamLane& ln = lanes[g];
        if (hipSetDevice(ln.device) != hipSuccess) {
            status[g] = KMP_EDEVICE;
            return;
        }
        status[g] = stream_passes(c, o, ks, nk, ln, [&](const kmp_edge_chunk& ch) -> int {
            if (!sink) return KMP_OK;
            kmp_edge_chunk hc = ch;
            if (!sink_on_device) {
                const int rc = chunk_to_host(c, ch, nk, host[g], ln.L.stream, &hc);
                if (rc != KMP_OK) return rc;
            }
            std::lock_guard<std::mutex> lk(sink_mu);
            if (sink_rc != KMP_OK) return sink_rc;  // another rank's sink stopped the stream
            const int rc = sink(user, &hc);
            if (rc != KMP_OK) sink_rc = rc;
            return rc;
        });
    });
    KMP_TRY(c, use_device(c));
    for (uint32_t g = 0; g < G; ++g)
        if (status[g] != KMP_OK) {
            if (status[g] == sink_rc) return sink_rc;
            return fail(c, status[g], "rank %u (device %d, rows [%u, %u)): stream: %s (%s)", g, lanes[g].device,
                        start[g], start[g + 1], kmp_status_string(status[g]), c->err.c_str());
        }
    std::vector<StreamLane*> lp;
    for (auto& ln : lanes) lp.push_back(&ln);
    return finish_summary(c, o, lp, summary);
}

extern "C" {

int kmp_ctx_set_rows(kmp_ctx* c, uint32_t row_lo, uint32_t row_hi) {
    if (!c) return KMP_EINVAL;
    if (row_lo > row_hi) return fail(c, KMP_EINVAL, "rows [%u, %u)", row_lo, row_hi);
    c->rows_lo = row_lo;
    c->rows_hi = row_hi;
    return KMP_OK;
}

int kmp_pairs_stream(kmp_ctx* c, const kmp_pair_opts* opts, const int* ks, uint32_t nk, int sink_on_device,
                     kmp_edge_sink sink, void* user, kmp_stream_summary* summary) {
    if (!c) return KMP_EINVAL;
    c->err.clear();
    kmp_pair_opts o;
    KMP_TRY(c, opts_multi(c, opts, ks, nk, &o));
    KMP_TRY(c, use_device(c));
    uint32_t lo = 0, hi = c->n;
    if (c->rows_hi) {
        if (c->rows_hi > c->n) return fail(c, KMP_EINVAL, "rows [%u, %u) past the batch (%u)", c->rows_lo, c->rows_hi, c->n);
        lo = c->rows_lo;
        hi = c->rows_hi;
    }
    if (getenv("KMP_DEBUG")) fprintf(stderr, "kmp: stream rows [%u, %u)\n", lo, hi);
    KMP_TRY(c, prepare_ksets(c, ks, nk));  // the reference's counters per k (kmp_build_sets)
    if (getenv("KMP_DEBUG")) fprintf(stderr, "kmp: stream sets built\n");
    restore_ksets(c, nk);
    if (c->ranks.size() > 1) return multi_stream(c, o, ks, nk, sink_on_device, sink, user, summary, lo, hi);
    DevBuf dacc;
    KMP_HIP(c, dacc.reserve(sizeof(kmp::DigestAcc)));
    KMP_HIP(c, hipMemsetAsync(dacc.p, 0, sizeof(kmp::DigestAcc), c->stream));
    StreamLane ln = ctx_lane(c, lo, hi, dacc);
    HostChunk host;
    int rc = stream_passes(c, o, ks, nk, ln, [&](const kmp_edge_chunk& ch) -> int {
        if (!sink) return KMP_OK;
        if (sink_on_device) return sink(user, &ch);
        kmp_edge_chunk hc{};
        KMP_TRY(c, chunk_to_host(c, ch, nk, host, c->stream, &hc));
        return sink(user, &hc);
    });
    if (rc != KMP_OK) return rc;
    rc = finish_summary(c, o, {&ln}, summary);
    if (getenv("KMP_DEBUG")) fprintf(stderr, "kmp: stream done (%u passes)\n", ln.passes);
    return rc;
}

// kmp_pairs_multi_k: the stream, collected into one device list (D2D appends), then copied out
int kmp_pairs_multi_k(kmp_ctx* c, const kmp_pair_opts* opts, const int* ks, uint32_t nk, kmp_edges** out) {
    if (!c || !out) return KMP_EINVAL;
    *out = nullptr;
    c->err.clear();
    kmp_pair_opts o;
    KMP_TRY(c, opts_multi(c, opts, ks, nk, &o));
    KMP_TRY(c, use_device(c));
    const bool blosum = o.score == KMP_SCORE_BLOSUM;
    // collected device arrays: p q w score w_0 .. w_{nk-1}, each cap entries
    const uint32_t na = 4 + nk;
    DevBuf all;
    uint64_t cap = 0, count = 0;
    DevBuf dacc;
    KMP_HIP(c, dacc.reserve(sizeof(kmp::DigestAcc)));
    KMP_HIP(c, hipMemsetAsync(dacc.p, 0, sizeof(kmp::DigestAcc), c->stream));
    KMP_TRY(c, prepare_ksets(c, ks, nk));
    restore_ksets(c, nk);
    StreamLane ln = ctx_lane(c, 0, c->n, dacc);
    KMP_TRY(c, stream_passes(c, o, ks, nk, ln, [&](const kmp_edge_chunk& ch) -> int {
        if (count + ch.n > cap) {
            const uint64_t ncap = std::max<uint64_t>(1u << 16, (count + ch.n) + (count + ch.n) / 4);
            DevBuf nb;
            KMP_HIP(c, nb.reserve(ncap * 4 * na));
            for (uint32_t i = 0; i < na && count; ++i)
                KMP_HIP(c, hipMemcpyAsync(nb.as<uint32_t>() + i * ncap, all.as<uint32_t>() + i * cap, count * 4,
                                          hipMemcpyDeviceToDevice, c->stream));
            KMP_HIP(c, hipStreamSynchronize(c->stream));
            all.swap(nb);
            cap = ncap;
        }
        const uint32_t* src[4 + KMP_MULTI_K_MAX] = {ch.p, ch.q, ch.w, ch.score, ch.wk[0], ch.wk[1], ch.wk[2], ch.wk[3]};
        for (uint32_t i = 0; i < na && ch.n; ++i)
            KMP_HIP(c, hipMemcpyAsync(all.as<uint32_t>() + i * cap + count, src[i], ch.n * 4, hipMemcpyDeviceToDevice,
                                      c->stream));
        KMP_HIP(c, hipStreamSynchronize(c->stream));
        count += ch.n;
        return KMP_OK;
    }));
    KMP_TRY(c, finish_summary(c, o, {&ln}, nullptr));
    std::unique_ptr<kmp_edges> e(new (std::nothrow) kmp_edges);
    if (!e) return fail(c, KMP_ENOMEM, "edges");
    e->p.resize(count);
    e->q.resize(count);
    e->w.resize(count);
    e->score.resize(count);
    e->wk.resize((uint64_t)nk * count);
    hvec<uint32_t> iscore(count);
    if (count) {
        const uint32_t* d = all.as<uint32_t>();
        KMP_HIP(c, hipMemcpyAsync(e->p.data(), d, count * 4, hipMemcpyDeviceToHost, c->stream));
        KMP_HIP(c, hipMemcpyAsync(e->q.data(), d + cap, count * 4, hipMemcpyDeviceToHost, c->stream));
        KMP_HIP(c, hipMemcpyAsync(e->w.data(), d + 2 * cap, count * 4, hipMemcpyDeviceToHost, c->stream));
        KMP_HIP(c, hipMemcpyAsync(iscore.data(), d + 3 * cap, count * 4, hipMemcpyDeviceToHost, c->stream));
        for (uint32_t j = 0; j < nk; ++j)
            KMP_HIP(c, hipMemcpyAsync(e->wk.data() + j * count, d + (4 + j) * cap, count * 4, hipMemcpyDeviceToHost,
                                      c->stream));
    }
    KMP_HIP(c, hipStreamSynchronize(c->stream));
    for (uint64_t i = 0; i < count; ++i) e->score[i] = blosum ? (float)iscore[i] : (float)e->w[i];
    e->ks.assign(ks, ks + nk);
    *out = e.release();
    return KMP_OK;
}

int kmp_ctx_set_pass_keys(kmp_ctx* c, uint64_t keys) {
    if (!c) return KMP_EINVAL;
    c->pass_keys = keys;
    c->budget[0] = c->budget[1] = 0;
    return KMP_OK;
}

uint32_t kmp_ctx_last_passes(const kmp_ctx* c) { return c ? c->last_passes : 0u; }

uint64_t kmp_ctx_last_tail_windows(const kmp_ctx* c) { return c ? c->last_windows : 0u; }

int kmp_ctx_set_flat_heavy(kmp_ctx* c, int enable) {
    if (!c) return KMP_EINVAL;
    c->flat_heavy = enable ? 1 : 0;
    return KMP_OK;
}

int kmp_ctx_set_direct_tail(kmp_ctx* c, int enable) {
    if (!c) return KMP_EINVAL;
    c->direct_tail = enable ? 1 : 0;
    c->budget[1] = 0;  // the fused pass budget depends on the bytes per key of the tail
    return KMP_OK;
}

int kmp_edges_get_wk(const kmp_edges* e, uint32_t j, uint32_t* wk, uint64_t cap, uint64_t* n) {
    if (!e || !n) return KMP_EINVAL;
    const uint64_t count = e->p.size();
    *n = count;
    if (j >= e->ks.size()) return KMP_EINVAL;
    if (cap < count) return KMP_EOVERFLOW;
    if (count && !wk) return KMP_EINVAL;
    std::copy(e->wk.begin() + j * count, e->wk.begin() + (j + 1) * count, wk);
    return KMP_OK;
}

int kmp_edges_kmers(kmp_ctx* c, kmp_edges* e, int space) {
    if (!c || !e) return KMP_EINVAL;
    c->err.clear();
    if (space != KMP_KMERS_CODES && space != KMP_KMERS_IDS) return fail(c, KMP_EINVAL, "space must be CODES or IDS");
    if (e->ks.size() > 1) return fail(c, KMP_ESTATE, "k-mer lists of a multi-k edge set are per k: use one k");
    if (!c->k_sets) return fail(c, KMP_ESTATE, "kmp_build_sets first");
    KMP_TRY(c, use_device(c));
    const uint64_t count = e->p.size();
    std::vector<uint64_t> kofs(count + 1, 0);
    for (uint64_t i = 0; i < count; ++i) {
        if (e->p[i] >= c->n || e->q[i] >= c->n) return fail(c, KMP_EINVAL, "edge %llu names a protein out of range",
                                                             (unsigned long long)i);
        kofs[i + 1] = kofs[i] + e->w[i];
    }
    const uint64_t total = kofs[count];
    if (space == KMP_KMERS_IDS) KMP_TRY(c, ensure_repeat_index(c));
    DevBuf dp, dq, dk, dout, dref;
    KMP_HIP(c, dp.reserve(count * 4));
    KMP_HIP(c, dq.reserve(count * 4));
    KMP_HIP(c, dk.reserve((count + 1) * 8));
    KMP_HIP(c, dout.reserve(total * 4));
    if (space == KMP_KMERS_IDS) KMP_HIP(c, dref.reserve(count * 8));
    if (count) {
        KMP_HIP(c, hipMemcpyAsync(dp.p, e->p.data(), count * 4, hipMemcpyHostToDevice, c->stream));
        KMP_HIP(c, hipMemcpyAsync(dq.p, e->q.data(), count * 4, hipMemcpyHostToDevice, c->stream));
    }
    KMP_HIP(c, hipMemcpyAsync(dk.p, kofs.data(), (count + 1) * 8, hipMemcpyHostToDevice, c->stream));
    int rc = edge_kmers_device(c->rep.as<uint32_t>(), c->rep_len.as<uint32_t>(), c->off.as<uint64_t>(), dp.as<uint32_t>(),
                               dq.as<uint32_t>(), dk.as<uint64_t>(), count, dout.as<uint32_t>(), c->stream);
    if (rc == KMP_EINVAL) return fail(c, rc, "edge weights do not match the context's sets (edges of another build?)");
    if (rc != KMP_OK) return fail(c, rc, "edge k-mers: %s", kmp_status_string(rc));
    if (space == KMP_KMERS_IDS) {
        rc = edge_kmers_to_ids(c->rep_mphf, dk.as<uint64_t>(), count, total, dout.as<uint32_t>(), dref.as<uint64_t>(),
                               c->stream);
        if (rc != KMP_OK) return fail(c, rc, "edge k-mer ids: %s", kmp_status_string(rc));
    }
    std::vector<uint32_t> kmers(total);
    std::vector<uint64_t> ref(space == KMP_KMERS_IDS ? count : 0);
    if (total) KMP_HIP(c, hipMemcpyAsync(kmers.data(), dout.p, total * 4, hipMemcpyDeviceToHost, c->stream));
    if (!ref.empty()) KMP_HIP(c, hipMemcpyAsync(ref.data(), dref.p, count * 8, hipMemcpyDeviceToHost, c->stream));
    KMP_HIP(c, hipStreamSynchronize(c->stream));
    e->kofs.swap(kofs);
    e->kmers.swap(kmers);
    e->ref_key.swap(ref);
    e->kspace = space;
    return KMP_OK;
}

int kmp_edges_get_kmers(const kmp_edges* e, uint64_t* offsets, uint32_t* kmers, uint64_t cap, uint64_t* n) {
    if (!e || !n) return KMP_EINVAL;
    if (e->kspace < 0) return KMP_ESTATE;
    *n = e->kmers.size();
    if (offsets) std::copy(e->kofs.begin(), e->kofs.end(), offsets);
    if (cap < e->kmers.size()) return KMP_EOVERFLOW;
    if (!e->kmers.empty()) {
        if (!kmers) return KMP_EINVAL;
        std::copy(e->kmers.begin(), e->kmers.end(), kmers);
    }
    return KMP_OK;
}

int kmp_edges_reference_keys(const kmp_edges* e, uint64_t* keys, uint64_t cap, uint64_t* n) {
    if (!e || !n) return KMP_EINVAL;
    if (e->kspace != KMP_KMERS_IDS) return KMP_ESTATE;
    *n = e->ref_key.size();
    if (cap < e->ref_key.size()) return KMP_EOVERFLOW;
    if (!e->ref_key.empty()) {
        if (!keys) return KMP_EINVAL;
        std::copy(e->ref_key.begin(), e->ref_key.end(), keys);
    }
    return KMP_OK;
}

void kmp_edges_free(kmp_edges* e) { delete e; }

uint64_t kmp_edge_digest_term(uint32_t p, uint32_t q, uint32_t w, uint32_t score, uint32_t w0) {
    auto m = [](uint64_t z) {
        z += 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    };
    const uint64_t a = (uint64_t)p << 32 | q, b = (uint64_t)w << 32 | score;
    return m(a ^ m(b ^ m((uint64_t)w0)));
}

}  // extern "C"

