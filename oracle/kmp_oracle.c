/*
 * kmp_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's k-mer pair path
 * (Isabella136/uniprot_kmer_based_clustering, snapshot 2025-05-23).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and
 * only as the checker / the timed CPU baseline; the product path never calls it.
 *
 * PARITY UNPINNED.  The reference is a Rust crate that cannot be built in this image
 * (no rustc/cargo, crates not vendored, nightly-only) and it ships no
 * tests, known-answer vectors or golden outputs.  This restatement is therefore pinned
 * only by (1) hand-derived known-answer tests of the reference semantics
 * (tests/golden/), (2) an independent NumPy restatement in tests/ (sparse A·Aᵀ), and
 * (3) the dataset counters SURVEY.md §8c lists for uniprot_arg.fasta.
 *
 * Algorithm, phase for phase (file:line into /root/reference):
 *   windows + radix-21 codes ......... src/protein.rs:9-54 (codec), :107-132 (windows)
 *   per-protein sort+dedup ........... src/main.rs:99-101,187-189
 *   global df, df>=2 "repeat" split .. src/main.rs:77-122 (merge_sort :23-48), :127-149
 *   dense repeat ids (boomphf stand-in; ids differ from boomphf, unobservable in the
 *     edge list) ...................... src/main.rs:139-147, src/protein.rs:151-174
 *   Σ C(df,2) incidence expansion .... src/graph/mod.rs:39-193, src/graph/vertex.rs:59-140
 *   AMR-class edge filter ............ src/graph/mod.rs:549-697 (test at :580-587)
 *   per-pair collapse, w = #kmers .... src/graph/mod.rs:322-546, src/graph/edge.rs:56-85
 *   alignment candidates w > 10 ...... src/graph/mod.rs:242
 * The incidence expansion is executed row-wise (Gustavson): protein p walks the posting
 * list of each of its repeat k-mers and counts the later visitors q; every (k-mer, p, q)
 * incidence of the reference's multigraph is visited exactly once, the same-class ones
 * are dropped as mod.rs:584 does, and the per-pair count is the collapsed Group length.
 * Threading mirrors the reference's model (src/main.rs:84-121): `threads` workers pull
 * protein indices from one atomic cursor.
 */
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_OK 0
#define ORC_EINVAL 1
#define ORC_ENOMEM 2

/* src/protein.rs:9-13 — code = position in this list, anything else -> 20 (:49-54) */
static const char AMINO_ACID_LIST[21] = {'C', 'S', 'T', 'A', 'G', 'P', 'D', 'E', 'Q', 'N', 'H',
                                         'R', 'K', 'M', 'I', 'L', 'V', 'W', 'Y', 'F', '*'};

uint8_t orc_residue_code(uint8_t b) {
    for (int i = 0; i < 21; ++i)  /* linear search as amino_acid_to_bits does */
        if ((uint8_t)AMINO_ACID_LIST[i] == b) return (uint8_t)i;
    return 20;
}

/* src/protein.rs:114 — windows j in [0, L-k]; L < k yields none (the reference wraps
 * usize for L < 4 and panics; documented deviation in DESIGN.md). */
static inline uint64_t n_windows(uint64_t L, int k) { return L >= (uint64_t)k ? L - k + 1 : 0; }

/* src/protein.rs:29-37 generalised to k digits, big-endian base 21 */
uint32_t orc_pack(const uint8_t* s, int k) {
    uint32_t v = 0;
    for (int i = 0; i < k; ++i) v = v * 21u + orc_residue_code(s[i]);
    return v;
}

/* codes of every window of every protein; win_off[N+1] gets the CSR offsets */
int orc_extract(const uint8_t* res, const uint64_t* off, uint32_t n, int k, uint32_t* out,
                uint64_t* win_off) {
    if (k < 1 || k > 7) return ORC_EINVAL;
    uint8_t lut[256];
    for (int b = 0; b < 256; ++b) lut[b] = orc_residue_code((uint8_t)b);
    uint64_t w = 0;
    for (uint32_t p = 0; p < n; ++p) {
        win_off[p] = w;
        uint64_t L = off[p + 1] - off[p];
        const uint8_t* s = res + off[p];
        uint64_t nw = n_windows(L, k);
        for (uint64_t j = 0; j < nw; ++j) {
            uint32_t v = 0;
            for (int i = 0; i < k; ++i) v = v * 21u + lut[s[j + i]];
            out[w++] = v;
        }
    }
    win_off[n] = w;
    return ORC_OK;
}

/* ---- LSD radix sort of u32 (8-bit digits); tmp has n slots ---- */
static void radix_u32(uint32_t* a, uint32_t* tmp, uint64_t n) {
    uint64_t cnt[256];
    uint32_t *src = a, *dst = tmp;
    for (int shift = 0; shift < 32; shift += 8) {
        memset(cnt, 0, sizeof cnt);
        for (uint64_t i = 0; i < n; ++i) cnt[(src[i] >> shift) & 255]++;
        if (n == 0 || cnt[(src[0] >> shift) & 255] == n) continue; /* digit constant: skip pass */
        uint64_t s = 0;
        for (int d = 0; d < 256; ++d) { uint64_t c = cnt[d]; cnt[d] = s; s += c; }
        for (uint64_t i = 0; i < n; ++i) dst[cnt[(src[i] >> shift) & 255]++] = src[i];
        uint32_t* t = src; src = dst; dst = t;
    }
    if (src != a) memcpy(a, src, n * sizeof(uint32_t));
}

static void insertion_u32(uint32_t* a, uint64_t n) {
    for (uint64_t i = 1; i < n; ++i) {
        uint32_t v = a[i];
        uint64_t j = i;
        while (j > 0 && a[j - 1] > v) { a[j] = a[j - 1]; --j; }
        a[j] = v;
    }
}

static void sort_u32(uint32_t* a, uint32_t* tmp, uint64_t n) {
    if (n < 48) insertion_u32(a, n);
    else radix_u32(a, tmp, n);
}

static uint64_t dedup_sorted(uint32_t* a, uint64_t n) {
    if (n == 0) return 0;
    uint64_t m = 1;
    for (uint64_t i = 1; i < n; ++i)
        if (a[i] != a[m - 1]) a[m++] = a[i];
    return m;
}

typedef struct {
    uint64_t n_windows;   /* Σ (L-k+1) */
    uint64_t sum_S;       /* Σ |K(p)| */
    uint64_t distinct;    /* D: distinct k-mers over all proteins */
    uint64_t repeat;      /* R: k-mers with df >= 2 (graph/mod.rs:50) */
    uint64_t sum_cdf2;    /* Σ C(df,2): "Number of total edges" (graph/mod.rs:51) */
    uint64_t sum_w_diff;  /* Σ w over class-differing pairs = edges after AMR filter (:695) */
    uint64_t n_edges;     /* collapsed pairs emitted (:545 when min_shared == 1) */
    uint64_t n_align;     /* emitted pairs with w > align_threshold (mod.rs:242) */
    uint64_t pairs_any;   /* pairs with w >= 1 regardless of class */
    uint64_t max_df;
} orc_counters;

typedef struct {
    uint32_t n;
    int k;
    uint16_t* cls;
    uint64_t* win_off;     /* [n+1] */
    uint32_t* codes;       /* all windows, position order (Protein.five_mers) */
    uint64_t* set_off;     /* [n+1] CSR of K(p), sorted distinct codes */
    uint32_t* set_val;
    uint32_t* distinct;    /* sorted distinct codes [D] */
    uint32_t* df;          /* df per distinct code [D] */
    uint64_t n_distinct;
    uint32_t* rep_codes;   /* sorted repeat codes [R]; dense id = index (boomphf stand-in) */
    uint64_t n_repeat;
    uint32_t* rep_df;      /* five_mer_hash_freq (main.rs:154,192) */
    uint64_t* hid_off;     /* [n+1] CSR of the protein's repeat ids, ascending */
    uint32_t* hid_val;
    uint32_t* hid_pos;     /* position of p inside posting(h) for each hid entry */
    uint64_t* post_off;    /* [R+1] posting lists, protein index order */
    uint32_t* post_val;
    orc_counters c;
    int threads;
} orc_ctx;

typedef struct {
    orc_ctx* x;
    _Atomic uint32_t cursor;
} set_job;

static void* set_worker(void* arg) {
    set_job* j = (set_job*)arg;
    orc_ctx* x = j->x;
    uint32_t* tmp = NULL;
    uint64_t tmp_cap = 0;
    for (;;) {
        uint32_t p = atomic_fetch_add(&j->cursor, 1);
        if (p >= x->n) break;
        uint64_t b = x->win_off[p], e = x->win_off[p + 1], m = e - b;
        if (m > tmp_cap) {
            free(tmp);
            tmp_cap = m;
            tmp = (uint32_t*)malloc(m * sizeof(uint32_t));
        }
        uint32_t* a = x->set_val + b;   /* sets stored at window offsets, compacted below */
        memcpy(a, x->codes + b, m * sizeof(uint32_t));
        sort_u32(a, tmp, m);
        x->set_off[p] = dedup_sorted(a, m); /* temporarily: |K(p)| */
    }
    free(tmp);
    return NULL;
}

static void run_pool(int threads, void* (*fn)(void*), void* arg) {
    if (threads <= 1) { fn(arg); return; }
    pthread_t* t = (pthread_t*)malloc(sizeof(pthread_t) * threads);
    for (int i = 0; i < threads; ++i) pthread_create(&t[i], NULL, fn, arg);
    for (int i = 0; i < threads; ++i) pthread_join(t[i], NULL);
    free(t);
}

void orc_free_ctx(orc_ctx* x);

/* ---- the build's phases on the `threads` pool (main.rs:84-121 runs every phase on its pool) ---- */
typedef struct {
    orc_ctx* x;
    const uint8_t* res;
    const uint64_t* off;
    const uint8_t* lut;
    _Atomic uint32_t cursor;
} extract_job;

static void* extract_worker(void* arg) {  /* Protein::new for blocks of 64 proteins */
    extract_job* j = (extract_job*)arg;
    orc_ctx* x = j->x;
    for (;;) {
        uint32_t p0 = atomic_fetch_add(&j->cursor, 64);
        if (p0 >= x->n) break;
        uint32_t p1 = p0 + 64 < x->n ? p0 + 64 : x->n;
        for (uint32_t p = p0; p < p1; ++p) {
            const uint8_t* s = j->res + j->off[p];
            uint64_t w = x->win_off[p], nw = x->win_off[p + 1] - w;
            for (uint64_t t = 0; t < nw; ++t) {
                uint32_t v = 0;
                for (int i = 0; i < x->k; ++i) v = v * 21u + j->lut[s[t + i]];
                x->codes[w + t] = v;
            }
        }
    }
    return NULL;
}

/* stable LSD radix sort of u64 keys on bits [lo, hi), each pass split over the pool: per-chunk
 * digit counts, an exclusive scan over (digit, chunk), chunk-ordered scatter */
enum { RX_BITS = 11, RX_BINS = 1 << RX_BITS };
typedef struct {
    uint64_t *src, *dst;
    uint64_t n;
    int shift, T;
    uint64_t* cnt;  /* T x RX_BINS */
    _Atomic int next;
} rx_pass;

static void* rx_hist(void* arg) {
    rx_pass* r = (rx_pass*)arg;
    int t = atomic_fetch_add(&r->next, 1);
    uint64_t* c = r->cnt + (uint64_t)t * RX_BINS;
    memset(c, 0, sizeof(uint64_t) * RX_BINS);
    for (uint64_t i = r->n * t / r->T, e = r->n * (t + 1) / r->T; i < e; ++i) c[(r->src[i] >> r->shift) & (RX_BINS - 1)]++;
    return NULL;
}

static void* rx_scatter(void* arg) {
    rx_pass* r = (rx_pass*)arg;
    int t = atomic_fetch_add(&r->next, 1);
    uint64_t* c = r->cnt + (uint64_t)t * RX_BINS;
    for (uint64_t i = r->n * t / r->T, e = r->n * (t + 1) / r->T; i < e; ++i)
        r->dst[c[(r->src[i] >> r->shift) & (RX_BINS - 1)]++] = r->src[i];
    return NULL;
}

static void radix_u64_par(uint64_t* a, uint64_t* tmp, uint64_t n, int lo, int hi, int T) {
    if (T < 1) T = 1;
    if ((uint64_t)T > n / 4096 + 1) T = (int)(n / 4096 + 1);
    rx_pass r;
    r.n = n;
    r.T = T;
    r.cnt = (uint64_t*)malloc(sizeof(uint64_t) * RX_BINS * T);
    uint64_t *src = a, *dst = tmp;
    for (int shift = lo; shift < hi; shift += RX_BITS) {
        r.src = src; r.dst = dst; r.shift = shift;
        atomic_init(&r.next, 0);
        run_pool(T, rx_hist, &r);
        uint64_t s = 0, tot0 = 0;
        for (int t = 0; t < T; ++t) tot0 += r.cnt[(uint64_t)t * RX_BINS + ((n ? src[0] >> shift : 0) & (RX_BINS - 1))];
        if (n == 0 || tot0 == n) continue;  /* digit constant: skip the pass */
        for (int d = 0; d < RX_BINS; ++d)
            for (int t = 0; t < T; ++t) {
                uint64_t* c = &r.cnt[(uint64_t)t * RX_BINS + d];
                uint64_t v = *c;
                *c = s;
                s += v;
            }
        atomic_init(&r.next, 0);
        run_pool(T, rx_scatter, &r);
        uint64_t* t = src; src = dst; dst = t;
    }
    if (src != a) memcpy(a, src, n * sizeof(uint64_t));
    free(r.cnt);
}

/* keys (code << 32 | p) of K(p) in protein order, and the compacted set array */
typedef struct {
    orc_ctx* x;
    uint64_t* key;
    uint32_t* dst;        /* compacted K(p) values */
    const uint64_t* nset; /* |K(p)| (set_off before the prefix) */
    _Atomic uint32_t cursor;
} key_job;

static void* key_worker(void* arg) {
    key_job* j = (key_job*)arg;
    orc_ctx* x = j->x;
    for (;;) {
        uint32_t p0 = atomic_fetch_add(&j->cursor, 64);
        if (p0 >= x->n) break;
        uint32_t p1 = p0 + 64 < x->n ? p0 + 64 : x->n;
        for (uint32_t p = p0; p < p1; ++p) {
            const uint32_t* src = x->set_val + x->win_off[p];
            for (uint64_t i = x->set_off[p], t = 0; i < x->set_off[p + 1]; ++i, ++t) {
                j->dst[i] = src[t];
                j->key[i] = ((uint64_t)src[t] << 32) | p;
            }
        }
    }
    return NULL;
}

/* the sorted keys cut into T chunks at k-mer boundaries; pass 0 counts each chunk's distinct and
 * repeat k-mers and posting entries, pass 1 fills the arrays at the chunks' prefix offsets */
typedef struct {
    orc_ctx* x;
    const uint64_t* key;
    uint64_t s;
    int T, pass;
    uint64_t* cut;   /* [T+1] */
    uint64_t* cd;    /* per chunk: distinct, repeat, posting entries, Σ C(df,2), max df */
    _Atomic int next;
} run_job;

static void* run_worker(void* arg) {
    run_job* j = (run_job*)arg;
    orc_ctx* x = j->x;
    int t = atomic_fetch_add(&j->next, 1);
    const uint64_t* key = j->key;
    uint64_t* c = j->cd + 5 * (uint64_t)t;
    uint64_t d = j->pass ? c[0] : 0, r = j->pass ? c[1] : 0, tot = j->pass ? c[2] : 0, cdf2 = 0, maxdf = 0;
    for (uint64_t i = j->cut[t], e = j->cut[t + 1]; i < e;) {
        uint64_t k = i;
        while (k < e && (key[k] >> 32) == (key[i] >> 32)) ++k;
        uint32_t f = (uint32_t)(k - i);
        if (j->pass) {
            x->distinct[d] = (uint32_t)(key[i] >> 32);
            x->df[d] = f;
            if (f >= 2) {   /* repeat split (main.rs:127-149); dense id = rank among repeats */
                x->rep_codes[r] = (uint32_t)(key[i] >> 32);
                x->rep_df[r] = f;
                x->post_off[r] = tot;
                for (uint64_t q = i; q < k; ++q) x->post_val[tot++] = (uint32_t)key[q];
                ++r;
            }
        } else if (f >= 2) {
            ++r;
            tot += f;
            cdf2 += (uint64_t)f * (f - 1) / 2;
            if (f > maxdf) maxdf = f;
        }
        ++d;
        i = k;
    }
    if (!j->pass) {
        c[0] = d; c[1] = r; c[2] = tot; c[3] = cdf2; c[4] = maxdf;
    }
    return NULL;
}

/* each protein's repeat ids, ascending, with the position inside the id's posting list: the pool's
 * workers own consecutive id ranges, count per protein, then fill at per-(protein, worker) offsets */
typedef struct {
    orc_ctx* x;
    int T, pass;
    uint64_t* hcut;   /* [T+1] id ranges */
    uint32_t* cnt;    /* T x n: entries per (worker, protein), then the worker's cursor */
    _Atomic int next;
} hid_job;

static void* hid_worker(void* arg) {
    hid_job* j = (hid_job*)arg;
    orc_ctx* x = j->x;
    int t = atomic_fetch_add(&j->next, 1);
    uint32_t* c = j->cnt + (uint64_t)t * x->n;
    for (uint64_t h = j->hcut[t]; h < j->hcut[t + 1]; ++h)
        for (uint64_t q = x->post_off[h]; q < x->post_off[h + 1]; ++q) {
            uint32_t p = x->post_val[q];
            if (!j->pass) {
                c[p]++;
            } else {
                uint64_t o = x->hid_off[p] + c[p]++;
                x->hid_val[o] = (uint32_t)h;
                x->hid_pos[o] = (uint32_t)(q - x->post_off[h]);
            }
        }
    return NULL;
}

/* Builds windows, K(p), df, repeat ids and posting lists, every phase on the `threads` pool. */
orc_ctx* orc_build(const uint8_t* res, const uint64_t* off, uint32_t n, const uint16_t* cls, int k,
                   int threads) {
    if (k < 1 || k > 7) return NULL;
    orc_ctx* x = (orc_ctx*)calloc(1, sizeof(orc_ctx));
    x->n = n; x->k = k; x->threads = threads < 1 ? 1 : threads;
    x->cls = (uint16_t*)malloc(sizeof(uint16_t) * (n ? n : 1));
    if (cls) memcpy(x->cls, cls, sizeof(uint16_t) * n); else memset(x->cls, 0, sizeof(uint16_t) * n);
    x->win_off = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
    uint64_t nw = 0;
    for (uint32_t p = 0; p < n; ++p) nw += n_windows(off[p + 1] - off[p], k);
    x->codes = (uint32_t*)malloc(sizeof(uint32_t) * (nw ? nw : 1));
    {
        uint8_t lut[256];
        for (int b = 0; b < 256; ++b) lut[b] = orc_residue_code((uint8_t)b);
        uint64_t w = 0;
        for (uint32_t p = 0; p < n; ++p) {
            x->win_off[p] = w;
            w += n_windows(off[p + 1] - off[p], k);
        }
        x->win_off[n] = w;
        extract_job ej = {x, res, off, lut, 0};
        run_pool(x->threads, extract_worker, &ej);
    }
    x->c.n_windows = nw;

    /* per-protein sort + dedup (main.rs:99-101,187-189) */
    x->set_val = (uint32_t*)malloc(sizeof(uint32_t) * (nw ? nw : 1));
    x->set_off = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
    set_job sj = {x, 0};
    run_pool(x->threads, set_worker, &sj);
    uint64_t s = 0;
    for (uint32_t p = 0; p < n; ++p) {  /* |K(p)| -> offsets of the compacted sets */
        uint64_t m = x->set_off[p];
        x->set_off[p] = s;
        s += m;
    }
    x->set_off[n] = s;
    x->c.sum_S = s;

    /* global df over distinct per-protein k-mers (main.rs:77-122): one radix sort of
     * (code << 32 | protein) keys; each run of equal codes is one distinct k-mer, its
     * length the df, its low halves the posting list in protein-index order (the
     * visitor order of vertex.rs:100 with threads == 1).  The keys are built in protein
     * order, so a stable sort on the code bits alone keeps each run's proteins ascending. */
    uint64_t* key = (uint64_t*)malloc(sizeof(uint64_t) * (s ? s : 1));
    uint64_t* ktmp = (uint64_t*)malloc(sizeof(uint64_t) * (s ? s : 1));
    {
        uint32_t* sv = (uint32_t*)malloc(sizeof(uint32_t) * (s ? s : 1));
        key_job kj = {x, key, sv, NULL, 0};
        run_pool(x->threads, key_worker, &kj);
        free(x->set_val);
        x->set_val = sv;
    }
    int cbits = 1;
    { uint64_t top = 1; for (int i = 0; i < k; ++i) top *= 21; while ((1ull << cbits) < top) ++cbits; }
    radix_u64_par(key, ktmp, s, 32, 32 + cbits, x->threads);
    free(ktmp);
    /* k-mer runs: chunks cut at run starts, counted, scanned, filled */
    int T = x->threads;
    if ((uint64_t)T > s / 4096 + 1) T = (int)(s / 4096 + 1);
    run_job rj;
    rj.x = x; rj.key = key; rj.s = s; rj.T = T;
    rj.cut = (uint64_t*)malloc(sizeof(uint64_t) * (T + 1));
    rj.cd = (uint64_t*)calloc(5 * (uint64_t)T, sizeof(uint64_t));
    for (int t = 0; t <= T; ++t) {
        uint64_t c = s * t / T;
        while (c > 0 && c < s && (key[c] >> 32) == (key[c - 1] >> 32)) ++c;
        rj.cut[t] = t == T ? s : c;
    }
    for (int t = 1; t <= T; ++t) if (rj.cut[t] < rj.cut[t - 1]) rj.cut[t] = rj.cut[t - 1];
    rj.pass = 0;
    atomic_init(&rj.next, 0);
    run_pool(T, run_worker, &rj);
    uint64_t d = 0, r = 0, cdf2 = 0, maxdf = 0, tot = 0;
    for (int t = 0; t < T; ++t) {  /* chunk totals -> chunk offsets (kept in cd[0..2]) */
        uint64_t* c = rj.cd + 5 * (uint64_t)t;
        uint64_t cd0 = c[0], cr = c[1], ct = c[2];
        c[0] = d; c[1] = r; c[2] = tot;
        d += cd0; r += cr; tot += ct;
        cdf2 += c[3];
        if (c[4] > maxdf) maxdf = c[4];
    }
    x->distinct = (uint32_t*)malloc(sizeof(uint32_t) * (d ? d : 1));
    x->df = (uint32_t*)malloc(sizeof(uint32_t) * (d ? d : 1));
    x->rep_codes = (uint32_t*)malloc(sizeof(uint32_t) * (r ? r : 1));
    x->rep_df = (uint32_t*)malloc(sizeof(uint32_t) * (r ? r : 1));
    x->post_off = (uint64_t*)malloc(sizeof(uint64_t) * (r + 1));
    x->post_val = (uint32_t*)malloc(sizeof(uint32_t) * (tot ? tot : 1));
    rj.pass = 1;
    atomic_init(&rj.next, 0);
    run_pool(T, run_worker, &rj);
    x->post_off[r] = tot;
    free(rj.cut);
    free(rj.cd);
    free(key);
    x->n_distinct = d;
    x->n_repeat = r;
    x->c.distinct = d;
    x->c.repeat = r;
    x->c.sum_cdf2 = cdf2;
    x->c.max_df = maxdf;

    /* remove_unique_five_mers + modify_hash_five_mer (protein.rs:151-174): each protein's
     * repeat ids, ascending, with its position inside the id's posting list */
    x->hid_off = (uint64_t*)calloc(n + 1, sizeof(uint64_t));
    x->hid_val = (uint32_t*)malloc(sizeof(uint32_t) * (tot ? tot : 1));
    x->hid_pos = (uint32_t*)malloc(sizeof(uint32_t) * (tot ? tot : 1));
    {
        int H = x->threads;
        if ((uint64_t)H > tot / 65536 + 1) H = (int)(tot / 65536 + 1);
        hid_job hj;
        hj.x = x; hj.T = H;
        hj.hcut = (uint64_t*)malloc(sizeof(uint64_t) * (H + 1));
        hj.cnt = (uint32_t*)calloc((uint64_t)H * (n ? n : 1), sizeof(uint32_t));
        uint64_t h = 0;  /* id ranges of about equal posting entries */
        for (int t = 0; t <= H; ++t) {
            uint64_t want = tot * t / H;
            while (h < r && x->post_off[h] < want) ++h;
            hj.hcut[t] = t == H ? r : h;
        }
        hj.pass = 0;
        atomic_init(&hj.next, 0);
        run_pool(H, hid_worker, &hj);
        uint64_t o = 0;  /* protein-major offsets; inside a protein the workers in id order */
        for (uint32_t p = 0; p < n; ++p) {
            x->hid_off[p] = o;
            for (int t = 0; t < H; ++t) {
                uint32_t* c = &hj.cnt[(uint64_t)t * n + p];
                uint32_t v = *c;
                *c = (uint32_t)(o - x->hid_off[p]);
                o += v;
            }
        }
        x->hid_off[n] = o;
        hj.pass = 1;
        atomic_init(&hj.next, 0);
        run_pool(H, hid_worker, &hj);
        free(hj.hcut);
        free(hj.cnt);
    }
    return x;
}

/* ---- pair expansion + class filter + collapse ---- */
typedef struct {
    uint32_t* q;
    uint32_t* w;
    uint64_t n, cap;
} edge_buf;

typedef struct {
    orc_ctx* x;
    _Atomic uint32_t cursor;
    uint32_t min_shared;
    int require_class_diff;
    uint32_t align_threshold;
    edge_buf* rows;          /* one per protein p */
    _Atomic uint64_t pairs_any, sum_w_diff, n_align;
} pair_job;

static void* pair_worker(void* arg) {
    pair_job* j = (pair_job*)arg;
    orc_ctx* x = j->x;
    uint32_t n = x->n;
    uint32_t* cnt = (uint32_t*)calloc(n ? n : 1, sizeof(uint32_t));
    uint32_t* touched = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    uint32_t* tmp = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    uint64_t any = 0, wdiff = 0, nal = 0;
    for (;;) {
        uint32_t p = atomic_fetch_add(&j->cursor, 1);
        if (p >= n) break;
        uint64_t nt = 0;
        /* every (k-mer h, p, q>p) incidence of the multigraph (vertex.rs:103-137) */
        for (uint64_t i = x->hid_off[p]; i < x->hid_off[p + 1]; ++i) {
            uint32_t h = x->hid_val[i];
            uint64_t b = x->post_off[h] + x->hid_pos[i] + 1, e = x->post_off[h + 1];
            for (uint64_t t = b; t < e; ++t) {
                uint32_t q = x->post_val[t];
                if (cnt[q]++ == 0) touched[nt++] = q;
            }
        }
        sort_u32(touched, tmp, nt);
        edge_buf* row = &j->rows[p];
        for (uint64_t t = 0; t < nt; ++t) {
            uint32_t q = touched[t], w = cnt[q];
            cnt[q] = 0;
            ++any;
            int differ = x->cls[p] != x->cls[q];   /* mod.rs:580-587 */
            if (differ) wdiff += w;
            if ((differ || !j->require_class_diff) && w >= j->min_shared) {
                if (row->n == row->cap) {
                    row->cap = row->cap ? row->cap * 2 : 16;
                    row->q = (uint32_t*)realloc(row->q, row->cap * sizeof(uint32_t));
                    row->w = (uint32_t*)realloc(row->w, row->cap * sizeof(uint32_t));
                }
                row->q[row->n] = q;
                row->w[row->n] = w;
                row->n++;
                if (w > j->align_threshold) ++nal;
            }
        }
    }
    atomic_fetch_add(&j->pairs_any, any);
    atomic_fetch_add(&j->sum_w_diff, wdiff);
    atomic_fetch_add(&j->n_align, nal);
    free(cnt); free(touched); free(tmp);
    return NULL;
}

/* Canonical edge list: (p,q,w), p<q, sorted by (p,q).  Arrays malloc'd; free with orc_free. */
int orc_pairs(orc_ctx* x, uint32_t min_shared, int require_class_diff, uint32_t align_threshold,
              uint32_t** P, uint32_t** Q, uint32_t** W, uint64_t* n_edges) {
    if (!x) return ORC_EINVAL;
    pair_job j;
    j.x = x;
    atomic_init(&j.cursor, 0);
    j.min_shared = min_shared < 1 ? 1 : min_shared;
    j.require_class_diff = require_class_diff;
    j.align_threshold = align_threshold;
    j.rows = (edge_buf*)calloc(x->n ? x->n : 1, sizeof(edge_buf));
    atomic_init(&j.pairs_any, 0);
    atomic_init(&j.sum_w_diff, 0);
    atomic_init(&j.n_align, 0);
    run_pool(x->threads, pair_worker, &j);
    uint64_t tot = 0;
    for (uint32_t p = 0; p < x->n; ++p) tot += j.rows[p].n;
    uint32_t* pp = (uint32_t*)malloc(sizeof(uint32_t) * (tot ? tot : 1));
    uint32_t* qq = (uint32_t*)malloc(sizeof(uint32_t) * (tot ? tot : 1));
    uint32_t* ww = (uint32_t*)malloc(sizeof(uint32_t) * (tot ? tot : 1));
    uint64_t o = 0;
    for (uint32_t p = 0; p < x->n; ++p) {
        edge_buf* r = &j.rows[p];
        for (uint64_t t = 0; t < r->n; ++t) { pp[o] = p; qq[o] = r->q[t]; ww[o] = r->w[t]; ++o; }
        free(r->q); free(r->w);
    }
    free(j.rows);
    x->c.pairs_any = atomic_load(&j.pairs_any);
    x->c.sum_w_diff = atomic_load(&j.sum_w_diff);
    x->c.n_edges = tot;
    x->c.n_align = atomic_load(&j.n_align);
    *P = pp; *Q = qq; *W = ww; *n_edges = tot;
    return ORC_OK;
}

void orc_get_counters(const orc_ctx* x, orc_counters* c) { *c = x->c; }
uint64_t orc_n_windows(const orc_ctx* x) { return x->c.n_windows; }
const uint32_t* orc_codes(const orc_ctx* x) { return x->codes; }
const uint64_t* orc_win_off(const orc_ctx* x) { return x->win_off; }
const uint32_t* orc_set_val(const orc_ctx* x) { return x->set_val; }
const uint64_t* orc_set_off(const orc_ctx* x) { return x->set_off; }
const uint32_t* orc_rep_codes(const orc_ctx* x) { return x->rep_codes; }
const uint32_t* orc_rep_df(const orc_ctx* x) { return x->rep_df; }
uint64_t orc_n_repeat(const orc_ctx* x) { return x->n_repeat; }
const uint32_t* orc_distinct(const orc_ctx* x) { return x->distinct; }
const uint32_t* orc_distinct_df(const orc_ctx* x) { return x->df; }
uint64_t orc_n_distinct(const orc_ctx* x) { return x->n_distinct; }

/* shared codes of (p,q), ascending (KmerEdgeGroup.kmers by code, edge.rs:56-85) */
uint64_t orc_shared(const orc_ctx* x, uint32_t p, uint32_t q, uint32_t* out, uint64_t cap) {
    const uint32_t* a = x->set_val + x->set_off[p];
    const uint32_t* b = x->set_val + x->set_off[q];
    uint64_t na = x->set_off[p + 1] - x->set_off[p], nb = x->set_off[q + 1] - x->set_off[q];
    uint64_t i = 0, k = 0, m = 0;
    while (i < na && k < nb) {
        if (a[i] < b[k]) ++i;
        else if (a[i] > b[k]) ++k;
        else { if (m < cap) out[m] = a[i]; ++m; ++i; ++k; }
    }
    return m;
}

void orc_free(void* p) { free(p); }

void orc_free_ctx(orc_ctx* x) {
    if (!x) return;
    free(x->cls); free(x->win_off); free(x->codes); free(x->set_off); free(x->set_val);
    free(x->distinct); free(x->df); free(x->rep_codes); free(x->rep_df); free(x->hid_off);
    free(x->hid_val); free(x->hid_pos); free(x->post_off); free(x->post_val);
    free(x);
}

/* ======================================================================================
 * Config 5 restated for streamed checking: the union over nk contexts (the
 * same batch at distinct k) of the edges of rows [row_lo, row_hi), an edge (p, q) emitted when
 * the classes differ (when required) and any w_j >= min_shared, with w = Σ_j w_j and
 * score = Σ_j score_j (BLOSUM: Σ over the shared k-mers x of Σ_i B62[x_i][x_i], the diagonal of
 * blosum.rs:8-30 in residue-code order, code 20 scored 0; COUNT: score = w).  Row p walks, per
 * k, the posting list of each of its repeat k-mers past its own position (vertex.rs:103-137),
 * exactly as orc_pairs does, and counts w_j and the score per later protein q.  Either the
 * edges are collected (canonical order) or only summarised: the counters and the digest that
 * kmp_pairs_stream reports (Σ of kmp_edge_digest_term over the edges, also per row segment
 * p * 64 / N).  The digest term is restated here from its definition in kmerpair.h.
 * ====================================================================================== */
#define ORC_SEGMENTS 64

static const uint8_t B62_DIAG[21] = {9, 4, 5, 4, 6, 7, 6, 5, 5, 6, 8, 5, 5, 5, 4, 4, 4, 11, 7, 6, 0};

static uint32_t code_self_score(uint32_t code, int k) {
    uint32_t s = 0;
    for (int i = 0; i < k; ++i) {
        s += B62_DIAG[code % 21u];
        code /= 21u;
    }
    return s;
}

static inline uint64_t orc_mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint64_t orc_digest_term(uint32_t p, uint32_t q, uint32_t w, uint32_t s, uint32_t w0) {
    uint64_t a = ((uint64_t)p << 32) | q, b = ((uint64_t)w << 32) | s;
    return orc_mix(a ^ orc_mix(b ^ orc_mix((uint64_t)w0)));
}

typedef struct {
    uint64_t n_edges, sum_w, sum_score, n_align, sum_w_diff, incidences, digest;
    uint64_t seg_edges[ORC_SEGMENTS], seg_digest[ORC_SEGMENTS];
} orc_digest;

#define ORC_MAXK 4
typedef struct {
    orc_ctx* xs[ORC_MAXK];
    uint32_t* hscore[ORC_MAXK];  /* self-score of each repeat id, per k */
    int nk;
    uint32_t row_lo, row_hi, min_shared, align_threshold;
    int require_class_diff, blosum, collect;
    _Atomic uint32_t cursor;
    edge_buf* rows;              /* collect: one per row (q, w of the union) */
    uint32_t** rs;               /* collect: per row, score and w_j arrays (1 + nk per edge) */
    pthread_mutex_t lock;
    orc_digest dg;
} stream_job;

static void* stream_worker(void* arg) {
    stream_job* j = (stream_job*)arg;
    orc_ctx* x0 = j->xs[0];
    const uint32_t n = x0->n, nk = (uint32_t)j->nk;
    uint32_t* cnt = (uint32_t*)calloc((size_t)nk * (n ? n : 1), sizeof(uint32_t));
    uint32_t* sc = (uint32_t*)calloc(n ? n : 1, sizeof(uint32_t));
    uint8_t* mark = (uint8_t*)calloc(n + 8, 1);
    uint32_t* touched = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    uint32_t* tmp = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    orc_digest d;
    memset(&d, 0, sizeof d);
    for (;;) {
        uint32_t r0 = atomic_fetch_add(&j->cursor, 16u);
        if (r0 >= j->row_hi - j->row_lo) break;
        uint32_t r1 = r0 + 16 < j->row_hi - j->row_lo ? r0 + 16 : j->row_hi - j->row_lo;
        for (uint32_t pr = j->row_lo + r0; pr < j->row_lo + r1; ++pr) {
            const uint32_t p = pr;
            uint64_t nt = 0;
            for (uint32_t k = 0; k < nk; ++k) {
                orc_ctx* x = j->xs[k];
                uint32_t* ck = cnt + (size_t)k * n;
                for (uint64_t i = x->hid_off[p]; i < x->hid_off[p + 1]; ++i) {
                    const uint32_t h = x->hid_val[i];
                    const uint32_t s = j->blosum ? j->hscore[k][h] : 0u;
                    const uint64_t b = x->post_off[h] + x->hid_pos[i] + 1, e = x->post_off[h + 1];
                    for (uint64_t t = b; t < e; ++t) {
                        const uint32_t q = x->post_val[t];
                        ck[q]++;
                        sc[q] += s;
                        if (!mark[q]) {
                            mark[q] = 1;
                            touched[nt++] = q;
                        }
                        if (!j->require_class_diff || x->cls[p] != x->cls[q]) d.incidences++;
                    }
                }
            }
            /* ascending q: sort the touched list, or scan the marks when they are dense */
            const uint64_t span = n - p;
            int scan = nt * 16 > span / 8;
            if (!scan) sort_u32(touched, tmp, nt);
            uint64_t it = 0;
            uint64_t qi = p + 1;
            edge_buf* row = j->collect ? &j->rows[p - j->row_lo] : NULL;
            for (;;) {
                uint32_t q;
                if (scan) {
                    while (qi < n && !mark[qi]) {
                        if ((qi & 7) == 0 && qi + 8 <= n) {
                            uint64_t wd;
                            memcpy(&wd, mark + qi, 8);
                            if (!wd) { qi += 8; continue; }
                        }
                        ++qi;
                    }
                    if (qi >= n) break;
                    q = (uint32_t)qi++;
                } else {
                    if (it >= nt) break;
                    q = touched[it++];
                }
                mark[q] = 0;
                uint32_t w = 0, any = 0, wj[ORC_MAXK];
                for (uint32_t k = 0; k < nk; ++k) {
                    wj[k] = cnt[(size_t)k * n + q];
                    cnt[(size_t)k * n + q] = 0;
                    w += wj[k];
                    any |= wj[k] >= j->min_shared;
                }
                const uint32_t s = j->blosum ? sc[q] : w;
                sc[q] = 0;
                const int differ = x0->cls[p] != x0->cls[q]; /* mod.rs:580-587 */
                if (!any || (j->require_class_diff && !differ)) continue;
                d.n_edges++;
                d.sum_w += w;
                d.sum_score += s;
                d.n_align += w > j->align_threshold;
                if (differ) d.sum_w_diff += w;
                const uint64_t term = orc_digest_term(p, q, w, s, wj[0]);
                d.digest += term;
                const uint32_t g = (uint32_t)((uint64_t)p * ORC_SEGMENTS / n);
                d.seg_edges[g]++;
                d.seg_digest[g] += term;
                if (row) {
                    if (row->n == row->cap) {
                        row->cap = row->cap ? row->cap * 2 : 16;
                        row->q = (uint32_t*)realloc(row->q, row->cap * sizeof(uint32_t));
                        row->w = (uint32_t*)realloc(row->w, row->cap * sizeof(uint32_t));
                        j->rs[p - j->row_lo] =
                            (uint32_t*)realloc(j->rs[p - j->row_lo], row->cap * (1 + nk) * sizeof(uint32_t));
                    }
                    uint32_t* ex = j->rs[p - j->row_lo] + row->n * (1 + nk);
                    ex[0] = s;
                    for (uint32_t k = 0; k < nk; ++k) ex[1 + k] = wj[k];
                    row->q[row->n] = q;
                    row->w[row->n] = w;
                    row->n++;
                }
            }
        }
    }
    pthread_mutex_lock(&j->lock);
    j->dg.n_edges += d.n_edges;
    j->dg.sum_w += d.sum_w;
    j->dg.sum_score += d.sum_score;
    j->dg.n_align += d.n_align;
    j->dg.sum_w_diff += d.sum_w_diff;
    j->dg.incidences += d.incidences;
    j->dg.digest += d.digest;
    for (int g = 0; g < ORC_SEGMENTS; ++g) {
        j->dg.seg_edges[g] += d.seg_edges[g];
        j->dg.seg_digest[g] += d.seg_digest[g];
    }
    pthread_mutex_unlock(&j->lock);
    free(cnt); free(sc); free(mark); free(touched); free(tmp);
    return NULL;
}

/* collect != 0: the arrays P, Q, W, S (score) and WK (nk x n_edges, k-major) are malloc'd, canonical order. */
int orc_stream(orc_ctx** xs, int nk, uint32_t row_lo, uint32_t row_hi, uint32_t min_shared,
               int require_class_diff, uint32_t align_threshold, int blosum, int threads, int collect,
               orc_digest* dg, uint32_t** P, uint32_t** Q, uint32_t** W, uint32_t** S, uint32_t** WK,
               uint64_t* n_edges) {
    if (nk < 1 || nk > ORC_MAXK || !xs || !xs[0] || row_lo > row_hi || row_hi > xs[0]->n) return ORC_EINVAL;
    for (int k = 1; k < nk; ++k)
        if (!xs[k] || xs[k]->n != xs[0]->n) return ORC_EINVAL;
    stream_job j;
    memset(&j, 0, sizeof j);
    j.nk = nk;
    for (int k = 0; k < nk; ++k) {
        j.xs[k] = xs[k];
        j.hscore[k] = (uint32_t*)malloc(sizeof(uint32_t) * (xs[k]->n_repeat ? xs[k]->n_repeat : 1));
        for (uint64_t h = 0; h < xs[k]->n_repeat; ++h) j.hscore[k][h] = code_self_score(xs[k]->rep_codes[h], xs[k]->k);
    }
    j.row_lo = row_lo;
    j.row_hi = row_hi;
    j.min_shared = min_shared < 1 ? 1 : min_shared;
    j.align_threshold = align_threshold;
    j.require_class_diff = require_class_diff;
    j.blosum = blosum;
    j.collect = collect;
    atomic_init(&j.cursor, 0);
    pthread_mutex_init(&j.lock, NULL);
    const uint32_t nr = row_hi - row_lo;
    if (collect) {
        j.rows = (edge_buf*)calloc(nr ? nr : 1, sizeof(edge_buf));
        j.rs = (uint32_t**)calloc(nr ? nr : 1, sizeof(uint32_t*));
    }
    run_pool(threads < 1 ? 1 : threads, stream_worker, &j);
    pthread_mutex_destroy(&j.lock);
    for (int k = 0; k < nk; ++k) free(j.hscore[k]);
    if (dg) *dg = j.dg;
    if (n_edges) *n_edges = j.dg.n_edges;
    if (collect) {
        const uint64_t tot = j.dg.n_edges;
        uint32_t* pp = (uint32_t*)malloc(sizeof(uint32_t) * (tot ? tot : 1));
        uint32_t* qq = (uint32_t*)malloc(sizeof(uint32_t) * (tot ? tot : 1));
        uint32_t* ww = (uint32_t*)malloc(sizeof(uint32_t) * (tot ? tot : 1));
        uint32_t* ss = (uint32_t*)malloc(sizeof(uint32_t) * (tot ? tot : 1));
        uint32_t* wk = (uint32_t*)malloc(sizeof(uint32_t) * (tot ? tot : 1) * nk);
        uint64_t o = 0;
        for (uint32_t r = 0; r < nr; ++r) {
            edge_buf* b = &j.rows[r];
            for (uint64_t t = 0; t < b->n; ++t) {
                pp[o] = row_lo + r;
                qq[o] = b->q[t];
                ww[o] = b->w[t];
                ss[o] = j.rs[r][t * (1 + nk)];
                for (int k = 0; k < nk; ++k) wk[(uint64_t)k * tot + o] = j.rs[r][t * (1 + nk) + 1 + k];
                ++o;
            }
            free(b->q); free(b->w); free(j.rs[r]);
        }
        free(j.rows); free(j.rs);
        *P = pp; *Q = qq; *W = ww; *S = ss; *WK = wk;
    }
    return ORC_OK;
}

/* BLOSUM score of each pair (p[i], q[i]): Σ over the shared codes of their self-scores */
typedef struct {
    const orc_ctx* x;
    const uint32_t *p, *q;
    uint64_t n;
    uint32_t* out;
    _Atomic uint64_t cursor;
} score_job;

static void* score_worker(void* arg) {
    score_job* j = (score_job*)arg;
    const orc_ctx* x = j->x;
    for (;;) {
        uint64_t i0 = atomic_fetch_add(&j->cursor, 4096);
        if (i0 >= j->n) break;
        uint64_t i1 = i0 + 4096 < j->n ? i0 + 4096 : j->n;
        for (uint64_t i = i0; i < i1; ++i) {
            const uint32_t* a = x->set_val + x->set_off[j->p[i]];
            const uint32_t* b = x->set_val + x->set_off[j->q[i]];
            uint64_t na = x->set_off[j->p[i] + 1] - x->set_off[j->p[i]], nb = x->set_off[j->q[i] + 1] - x->set_off[j->q[i]];
            uint64_t u = 0, v = 0;
            uint32_t s = 0;
            while (u < na && v < nb) {
                if (a[u] < b[v]) ++u;
                else if (a[u] > b[v]) ++v;
                else { s += code_self_score(a[u], x->k); ++u; ++v; }
            }
            j->out[i] = s;
        }
    }
    return NULL;
}

int orc_pair_scores(const orc_ctx* x, const uint32_t* p, const uint32_t* q, uint64_t n, uint32_t* out, int threads) {
    if (!x) return ORC_EINVAL;
    for (uint64_t i = 0; i < n; ++i)
        if (p[i] >= x->n || q[i] >= x->n) return ORC_EINVAL;
    score_job j = {x, p, q, n, out, 0};
    atomic_init(&j.cursor, 0);
    run_pool(threads < 1 ? 1 : threads, score_worker, &j);
    return ORC_OK;
}

/* ======================================================================================
 * Direct restatement for sampled rows (an independent check of orc_stream and of the library
 * at sizes where the posting-list oracle is too slow to run live): for the few proteins p in
 * [row_lo, row_hi) and every q > p of the batch, w_k(p, q) = |K_k(p) ∩ K_k(q)| straight from the
 * definition (SURVEY.md §8 "Canonical result definition"; K(p) = the distinct window codes,
 * protein.rs:107-132 + main.rs:99-101), the BLOSUM score Σ over the shared codes of their
 * self-scores, the class filter of mod.rs:580-587 and the config-5 union rule.  Each q's windows
 * are extracted, sorted and deduplicated, and each distinct code is looked up in the sorted
 * (code, sample row) table of the sample's codes.  Edges in canonical order.
 * ====================================================================================== */
typedef struct {
    const uint8_t* res;
    const uint64_t* off;
    const uint16_t* cls;
    uint32_t n, lo, hi, nr;
    int nk;
    int ks[ORC_MAXK];
    uint64_t* tab[ORC_MAXK];    /* sorted (code << 32 | sample row index) */
    uint64_t ntab[ORC_MAXK];
    uint32_t min_shared;
    int require_class_diff, blosum;
    _Atomic uint32_t cursor;
    pthread_mutex_t lock;
    uint64_t* out;              /* (p << 32 | q) keys, then per edge: w, s, w_k ... (2 + nk words) */
    uint32_t* val;
    uint64_t nout, capout;
} direct_job;

static int cmp_u64(const void* a, const void* b) {
    uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : x > y;
}

static uint64_t distinct_codes(const uint8_t* s, uint64_t L, int k, const uint8_t* lut, uint32_t* buf,
                               uint32_t* tmp) {
    uint64_t nw = n_windows(L, k);
    for (uint64_t j = 0; j < nw; ++j) {
        uint32_t v = 0;
        for (int i = 0; i < k; ++i) v = v * 21u + lut[s[j + i]];
        buf[j] = v;
    }
    sort_u32(buf, tmp, nw);
    return dedup_sorted(buf, nw);
}

static void* direct_worker(void* arg) {
    direct_job* j = (direct_job*)arg;
    uint8_t lut[256];
    for (int b = 0; b < 256; ++b) lut[b] = orc_residue_code((uint8_t)b);
    uint64_t maxl = 0;
    for (uint32_t p = 0; p < j->n; ++p)
        if (j->off[p + 1] - j->off[p] > maxl) maxl = j->off[p + 1] - j->off[p];
    uint32_t* buf = (uint32_t*)malloc(sizeof(uint32_t) * (maxl + 1));
    uint32_t* tmp = (uint32_t*)malloc(sizeof(uint32_t) * (maxl + 1));
    uint32_t* w = (uint32_t*)calloc((size_t)j->nr * ORC_MAXK, sizeof(uint32_t));
    uint32_t* sc = (uint32_t*)calloc(j->nr, sizeof(uint32_t));
    uint32_t* touched = (uint32_t*)malloc(sizeof(uint32_t) * (j->nr ? j->nr : 1));
    uint8_t* mk = (uint8_t*)calloc(j->nr ? j->nr : 1, 1);
    uint64_t lcap = 1024, ln = 0;
    uint64_t* lkey = (uint64_t*)malloc(sizeof(uint64_t) * lcap);
    uint32_t* lval = (uint32_t*)malloc(sizeof(uint32_t) * lcap * (2 + j->nk));
    const uint32_t first = j->lo + 1;
    for (;;) {
        uint32_t q0 = atomic_fetch_add(&j->cursor, 256u);
        if ((uint64_t)first + q0 >= j->n) break;
        uint32_t q1 = first + q0 + 256 < j->n ? first + q0 + 256 : j->n;
        for (uint32_t q = first + q0; q < q1; ++q) {
            uint32_t nt = 0;
            for (int k = 0; k < j->nk; ++k) {
                uint64_t m = distinct_codes(j->res + j->off[q], j->off[q + 1] - j->off[q], j->ks[k], lut, buf, tmp);
                const uint64_t* T = j->tab[k];
                const uint64_t nT = j->ntab[k];
                for (uint64_t i = 0; i < m; ++i) {
                    const uint64_t key = (uint64_t)buf[i] << 32;
                    uint64_t a = 0, b = nT;  /* first entry >= key */
                    while (a < b) {
                        uint64_t mid = (a + b) >> 1;
                        if (T[mid] < key) a = mid + 1; else b = mid;
                    }
                    for (; a < nT && (T[a] >> 32) == buf[i]; ++a) {
                        const uint32_t r = (uint32_t)T[a];
                        if (j->lo + r >= q) continue;  /* pairs p < q only */
                        w[(size_t)r * ORC_MAXK + k]++;
                        if (j->blosum) sc[r] += code_self_score(buf[i], j->ks[k]);
                        if (!mk[r]) { mk[r] = 1; touched[nt++] = r; }
                    }
                }
            }
            for (uint32_t t = 0; t < nt; ++t) {
                const uint32_t r = touched[t], p = j->lo + r;
                mk[r] = 0;
                uint32_t tot = 0, any = 0;
                for (int k = 0; k < j->nk; ++k) {
                    tot += w[(size_t)r * ORC_MAXK + k];
                    any |= w[(size_t)r * ORC_MAXK + k] >= j->min_shared;
                }
                const int keep = any && (!j->require_class_diff || j->cls[p] != j->cls[q]);
                if (keep) {
                    if (ln == lcap) {
                        lcap *= 2;
                        lkey = (uint64_t*)realloc(lkey, sizeof(uint64_t) * lcap);
                        lval = (uint32_t*)realloc(lval, sizeof(uint32_t) * lcap * (2 + j->nk));
                    }
                    lkey[ln] = ((uint64_t)p << 32) | q;
                    uint32_t* v = lval + ln * (2 + j->nk);
                    v[0] = tot;
                    v[1] = j->blosum ? sc[r] : tot;
                    for (int k = 0; k < j->nk; ++k) v[2 + k] = w[(size_t)r * ORC_MAXK + k];
                    ++ln;
                }
                for (int k = 0; k < j->nk; ++k) w[(size_t)r * ORC_MAXK + k] = 0;
                sc[r] = 0;
            }
        }
    }
    pthread_mutex_lock(&j->lock);
    if (j->nout + ln > j->capout) {
        j->capout = (j->nout + ln) * 2 + 1024;
        j->out = (uint64_t*)realloc(j->out, sizeof(uint64_t) * j->capout);
        j->val = (uint32_t*)realloc(j->val, sizeof(uint32_t) * j->capout * (2 + j->nk));
    }
    memcpy(j->out + j->nout, lkey, sizeof(uint64_t) * ln);
    memcpy(j->val + j->nout * (2 + j->nk), lval, sizeof(uint32_t) * ln * (2 + j->nk));
    j->nout += ln;
    pthread_mutex_unlock(&j->lock);
    free(buf); free(tmp); free(w); free(sc); free(touched); free(mk); free(lkey); free(lval);
    return NULL;
}

/* Edges (p, q) of rows [row_lo, row_hi) (at most 65,536 rows) over ks[0..nk): P, Q, W, S and WK
 * (nk x n, k-major) malloc'd, canonical order. */
int orc_rows_direct(const uint8_t* res, const uint64_t* off, uint32_t n, const uint16_t* cls, const int* ks, int nk,
                    uint32_t row_lo, uint32_t row_hi, uint32_t min_shared, int require_class_diff, int blosum,
                    int threads, uint32_t** P, uint32_t** Q, uint32_t** W, uint32_t** S, uint32_t** WK,
                    uint64_t* n_edges) {
    if (nk < 1 || nk > ORC_MAXK || row_lo > row_hi || row_hi > n || row_hi - row_lo > 65536) return ORC_EINVAL;
    direct_job j;
    memset(&j, 0, sizeof j);
    j.res = res; j.off = off; j.n = n; j.lo = row_lo; j.hi = row_hi; j.nr = row_hi - row_lo; j.nk = nk;
    uint16_t* zero = NULL;
    if (!cls) { zero = (uint16_t*)calloc(n ? n : 1, sizeof(uint16_t)); cls = zero; }
    j.cls = cls;
    j.min_shared = min_shared < 1 ? 1 : min_shared;
    j.require_class_diff = require_class_diff;
    j.blosum = blosum;
    uint8_t lut[256];
    for (int b = 0; b < 256; ++b) lut[b] = orc_residue_code((uint8_t)b);
    uint64_t maxl = 0;
    for (uint32_t p = row_lo; p < row_hi; ++p)
        if (off[p + 1] - off[p] > maxl) maxl = off[p + 1] - off[p];
    uint32_t* buf = (uint32_t*)malloc(sizeof(uint32_t) * (maxl + 1));
    uint32_t* tmp = (uint32_t*)malloc(sizeof(uint32_t) * (maxl + 1));
    for (int k = 0; k < nk; ++k) {
        if (ks[k] < 1 || ks[k] > 7) return ORC_EINVAL;
        j.ks[k] = ks[k];
        uint64_t tot = 0, cap = 1024;
        uint64_t* t = (uint64_t*)malloc(sizeof(uint64_t) * cap);
        for (uint32_t p = row_lo; p < row_hi; ++p) {
            uint64_t m = distinct_codes(res + off[p], off[p + 1] - off[p], ks[k], lut, buf, tmp);
            if (tot + m > cap) { cap = (tot + m) * 2; t = (uint64_t*)realloc(t, sizeof(uint64_t) * cap); }
            for (uint64_t i = 0; i < m; ++i) t[tot++] = ((uint64_t)buf[i] << 32) | (p - row_lo);
        }
        qsort(t, tot, sizeof(uint64_t), cmp_u64);
        j.tab[k] = t;
        j.ntab[k] = tot;
    }
    free(buf); free(tmp);
    atomic_init(&j.cursor, 0);
    pthread_mutex_init(&j.lock, NULL);
    run_pool(threads < 1 ? 1 : threads, direct_worker, &j);
    pthread_mutex_destroy(&j.lock);
    /* canonical order: sort the keys with their value rows */
    const uint64_t m = j.nout, vw = 2 + nk;
    uint64_t* idx = (uint64_t*)malloc(sizeof(uint64_t) * (m ? m : 1));
    for (uint64_t i = 0; i < m; ++i) idx[i] = i;
    /* sort (key, index) pairs: keys are distinct, so sort 128-bit by key via an index array */
    uint64_t* kk = j.out;
    {   /* simple: pack to (key, idx) records and qsort */
        typedef struct { uint64_t key, i; } rec;
        rec* r = (rec*)malloc(sizeof(rec) * (m ? m : 1));
        for (uint64_t i = 0; i < m; ++i) { r[i].key = kk[i]; r[i].i = i; }
        qsort(r, m, sizeof(rec), cmp_u64);  /* key is the first field */
        for (uint64_t i = 0; i < m; ++i) idx[i] = r[i].i;
        free(r);
    }
    uint32_t* pp = (uint32_t*)malloc(sizeof(uint32_t) * (m ? m : 1));
    uint32_t* qq = (uint32_t*)malloc(sizeof(uint32_t) * (m ? m : 1));
    uint32_t* ww = (uint32_t*)malloc(sizeof(uint32_t) * (m ? m : 1));
    uint32_t* ss = (uint32_t*)malloc(sizeof(uint32_t) * (m ? m : 1));
    uint32_t* wk = (uint32_t*)malloc(sizeof(uint32_t) * (m ? m : 1) * nk);
    for (uint64_t o = 0; o < m; ++o) {
        const uint64_t i = idx[o];
        pp[o] = (uint32_t)(kk[i] >> 32);
        qq[o] = (uint32_t)kk[i];
        const uint32_t* v = j.val + i * vw;
        ww[o] = v[0];
        ss[o] = v[1];
        for (int k = 0; k < nk; ++k) wk[(uint64_t)k * m + o] = v[2 + k];
    }
    free(idx); free(j.out); free(j.val); free(zero);
    for (int k = 0; k < nk; ++k) free(j.tab[k]);
    *P = pp; *Q = qq; *W = ww; *S = ss; *WK = wk; *n_edges = m;
    return ORC_OK;
}
