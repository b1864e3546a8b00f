/*
 * kmerpair.h — C ABI of the MI355X-native k-mer pair engine (libkmerpair.so).
 *
 * Drop-in boundary for the hot path of Isabella136/uniprot_kmer_based_clustering:
 * the Rust module surface that src/main.rs calls in src/protein.rs and the src/graph/ modules.
 * The reference has no FFI of its own; each entry point below names the
 * reference interface it replaces (file:line in the reference tree).  INTEGRATION.md
 * shows the Rust `extern "C"` block a maintainer would add to bind it.
 *
 * Conventions
 *  - Plain C: integer status returns (kmp_status), no exceptions or aborts cross the ABI.
 *  - Host-buffer API (kmp_load_proteins … kmp_edges_get): caller-owned inputs are copied
 *    before return; results are library-owned objects the caller frees.
 *  - Calls are synchronous, like the reference's graph methods (each spawns and joins
 *    its own pool before returning, mod.rs:81-124).  One host thread per kmp_ctx.
 *  - Device-stage API (kmp_dev_*): plain device pointers + an optional hipStream_t passed
 *    as void*, so a multi-GPU host (one process per GPU, RCCL between stages) can drive the
 *    stages on its own streams.  The set/tile stages allocate nothing and do not
 *    synchronise; the postings stages own their scratch in a kmp_postings workspace and
 *    synchronise the stream where they read device counts back (documented per call).
 *  - Proteins are indexed 0..N-1 in input (file) order; edges are (p, q, w) with p < q,
 *    sorted by (p, q) — the reference's post-combine_edges graph with orientation [p, q]
 *    (single-thread visitor order, vertex.rs:100).
 */
#ifndef KMERPAIR_H
#define KMERPAIR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KMP_ABI_VERSION 1

typedef enum {
    KMP_OK = 0,
    KMP_EINVAL = 1,     /* bad argument (reference: panic / expect) */
    KMP_ENOMEM = 2,     /* host or device allocation failed */
    KMP_EDEVICE = 3,    /* HIP runtime error or no usable gfx950 device */
    KMP_ERCCL = 4,      /* RCCL unavailable or a collective failed (multi-GPU context) */
    KMP_EOVERFLOW = 5,  /* caller buffer too small; *n holds the size needed */
    KMP_ESTATE = 6,     /* call out of order (e.g. kmp_pairs before kmp_load_proteins) */
    KMP_EIO = 7         /* file could not be read / written */
} kmp_status;

/* length laws of the synthetic generator */
enum { KMP_LEN_NORMAL300 = 0, KMP_LEN_LOGUNIFORM = 1 };

/* pair scores (kmp_pair_opts.score), build extensions (the reference computes neither, so their
 * parity is unpinned):
 *   COUNT    score = w
 *   JACCARD  score = w / (|K(p)| + |K(q)| - w), one correctly rounded f32 divide
 *   BLOSUM   score = Σ over the shared k-mers x of Σ_i B62[x_i][x_i] (the BLOSUM62 diagonal of
 *            blosum.rs:8-30 in residue-code order; code 20 scores 0), an exact integer in f32 */
enum { KMP_SCORE_COUNT = 0, KMP_SCORE_JACCARD = 1, KMP_SCORE_BLOSUM = 2 };

/* pair engines (kmp_pair_opts.engine); every engine returns the same edges */
enum {
    KMP_ENGINE_AUTO = 0,      /* the fastest engine for the batch: currently RESIDUES */
    KMP_ENGINE_POSTINGS = 1,  /* sort / expand Σ C(df,2) incidences / reduce (the reference's algorithm) */
    KMP_ENGINE_TILES = 2,     /* LDS-tiled all-pairs intersection over the N x N upper triangle */
    KMP_ENGINE_RESIDUES = 3   /* postings fed by the k-mer windows of the residues (kmp_dev_pairs_residues) */
};

typedef struct kmp_ctx kmp_ctx;
typedef struct kmp_edges kmp_edges;
typedef struct kmp_mphf kmp_mphf;

/* The reference's stderr counters (graph/mod.rs:50,51,545,695) plus set statistics. */
typedef struct {
    uint64_t n_proteins;
    uint64_t n_windows;   /* Σ (L-k+1): Protein.five_mers total (protein.rs:114) */
    uint64_t sum_S;       /* Σ |K(p)|, distinct k-mers per protein */
    uint64_t distinct;    /* distinct k-mers over all proteins (main.rs:137-140: five_mer_all) */
    uint64_t repeat;      /* df >= 2 k-mers: "Number of 5mers found in at least two proteins" (mod.rs:50) */
    uint64_t sum_cdf2;    /* Σ C(df,2): "Number of total edges" (mod.rs:51) */
    uint64_t sum_w_diff;  /* Σ w over class-differing pairs: edges after AMR filter (mod.rs:695) */
    uint64_t n_edges;     /* emitted pairs: "Number of edges now" after collapse (mod.rs:545) */
    uint64_t n_align;     /* emitted pairs with w > align_threshold (mod.rs:242) */
    uint64_t max_df;
} kmp_counters;

typedef struct {
    uint32_t min_shared;         /* emit iff w >= min_shared (reference: 1) */
    int32_t require_class_diff;  /* 1: drop same-AMR-class pairs (mod.rs:549-697); 0: keep */
    uint32_t align_threshold;    /* alignment candidates: w > threshold (mod.rs:242: 10) */
    int32_t score;               /* KMP_SCORE_COUNT | KMP_SCORE_JACCARD | KMP_SCORE_BLOSUM (build extensions) */
    int32_t engine;              /* KMP_ENGINE_* */
} kmp_pair_opts;

/* defaults: min_shared 1, require_class_diff 1, align_threshold 10, score COUNT, engine AUTO */
void kmp_pair_opts_default(kmp_pair_opts* opts);

/* ------------------------------------------------------------------ context -------- */
int kmp_version(void);                         /* KMP_ABI_VERSION */
const char* kmp_status_string(int status);
/* device: HIP ordinal; cpu_threads: host threads for ingest / planning (reference: `threads`, main.rs:57-60) */
int kmp_ctx_create(kmp_ctx** ctx, int device, int cpu_threads);
/* Multi-GPU context (the reference's `threads` split of the same work, main.rs:57-60,
 * graph/mod.rs:81-124): n_gpus ranks on the HIP devices devices[0..n_gpus) (NULL: 0..n_gpus-1),
 * rank 0 on devices[0] doing everything a single-GPU context does.  kmp_load_proteins copies the
 * batch to every rank; kmp_pairs (engine AUTO / RESIDUES) leaves rank g with the canonical edges of
 * its rows (kmp_row_split: the pairs whose smaller protein is in them) — by the k-mer split (rank g
 * expands its share of the k-mers, an all-to-all routes each pair key to its row owner, which
 * reduces it; kmp_dev_split_expand / kmp_dev_split_edges; frequent k-mers through each rank's
 * heavy path) or, when the class ids overflow the key or the split cannot run, by the row split
 * (every rank groups every k-mer and expands its rows) — and gathers the
 * ranks' edges to device 0 in rank order, which is the canonical list.  The library owns the
 * collectives: distinct devices get RCCL communicators created
 * in-process (ncclCommInitAll; KMP_ERCCL if RCCL is unavailable or a collective fails); a device
 * listed more than once runs several ranks on one GPU and the gather uses device copies (for
 * testing the split where RCCL admits one rank per device).  Other engines run on rank 0. */
int kmp_ctx_create_multi(kmp_ctx** ctx, int n_gpus, const int* devices, int cpu_threads);
int kmp_ctx_gpus(const kmp_ctx* ctx);               /* ranks (1 for kmp_ctx_create) */
const char* kmp_ctx_transport(const kmp_ctx* ctx);  /* "local", "copy" or "rccl" */
/* the flow of the last multi-GPU kmp_pairs: "kmer" (the k-mer split: each rank expands its share of
 * the k-mers, an all-to-all routes the pair keys to their row owners; kmp_dev_split_expand) or
 * "rows" (the row split: class ids wider than the key's field, or a batch the split cannot
 * take); "" before one */
const char* kmp_ctx_last_split(const kmp_ctx* ctx);
void kmp_ctx_destroy(kmp_ctx* ctx);
const char* kmp_last_error(const kmp_ctx* ctx);

/* ------------------------------------------------------------------ ingest --------- */
/* Replaces the Protein::new batch (protein.rs:107-132 via main.rs:65-72).  residues: the
 * packed sequence bytes of all proteins; offsets[N+1]: byte offsets; class_id[N]: AMR
 * class per protein, equal ids <=> equal get_amr_class() strings (protein.rs:135-138).
 * class_id may be NULL (all one class).  Copies to the device before return. */
int kmp_load_proteins(kmp_ctx* ctx, const uint8_t* residues, const uint64_t* offsets, uint32_t n,
                      const uint16_t* class_id);

/* ------------------------------------------------------------------ k-mers --------- */
/* Protein.five_mers generalised to k in {1..7} (protein.rs:29-37,107-132): all L-k+1 windows
 * in position order, duplicates kept; radix-21 big-endian codes.  Replaces get_five_mers
 * (protein.rs:141-143). */
int kmp_extract(kmp_ctx* ctx, int k);
int kmp_get_kmers(kmp_ctx* ctx, uint32_t protein, uint32_t* out, uint64_t cap, uint64_t* n);

/* ------------------------------------------------------------------ sets ----------- */
/* K(p): sorted distinct codes per protein (main.rs:99-101,187-189), plus the global repeat
 * (df >= 2) filter of remove_unique_five_mers (protein.rs:151-162). */
int kmp_build_sets(kmp_ctx* ctx, int k);
int kmp_get_set(kmp_ctx* ctx, uint32_t protein, uint32_t* out, uint64_t cap, uint64_t* n);
int kmp_counters_get(kmp_ctx* ctx, kmp_counters* out);

/* ------------------------------------------------------------------ repeat index --- */
/* The repeat k-mers (df >= 2) of the last kmp_build_sets, indexed by a device minimal perfect
 * hash (main.rs:127-149: Mphf::new(3.0, &five_mer_repeat)); built on first use, kept until the
 * next kmp_load_proteins / kmp_build_sets.  Ids are dense, 0 .. repeat-1, but not boomphf's
 * (SURVEY.md §8c): they are internal indices, and code_by_id / df_by_id give their meaning.
 *   kmp_get_df: df_by_id[repeat] = five_mer_hash_freq (main.rs:154,187-193);
 *   kmp_get_repeat_codes: code_by_id[repeat], the inverse of the hash;
 *   kmp_get_hash_kmers: hash_five_mers of protein p (remove_unique_five_mers +
 *     modify_hash_five_mer, protein.rs:151-174; get_five_hash, :146): the ids of p's repeat
 *     windows in first-occurrence order, duplicates dropped;
 *   kmp_get_hash_kmers_all: the same for every protein, CSR: ids[offsets[p] .. offsets[p+1]),
 *     offsets has n+1 entries (may be NULL to query the total in *n);
 *   kmp_repeat_mphf: the context-owned MPHF (valid until the index is rebuilt) for lookups.
 * All copy up to cap entries, set *n to the total and return KMP_EOVERFLOW if cap < total. */
int kmp_get_df(kmp_ctx* ctx, uint32_t* df_by_id, uint64_t cap, uint64_t* n);
int kmp_get_repeat_codes(kmp_ctx* ctx, uint32_t* code_by_id, uint64_t cap, uint64_t* n);
int kmp_get_hash_kmers(kmp_ctx* ctx, uint32_t protein, uint32_t* ids, uint64_t cap, uint64_t* n);
int kmp_get_hash_kmers_all(kmp_ctx* ctx, uint32_t* ids, uint64_t cap, uint64_t* offsets, uint64_t* n);
int kmp_repeat_mphf(kmp_ctx* ctx, const kmp_mphf** out);

/* ------------------------------------------------------------------ MPHF ----------- */
/* boomphf's Mphf<u32> surface (Mphf::new(gamma, &keys) / hash(&key), main.rs:139-140,145,192;
 * protein.rs:154,168) on the device: a BBHash of levelled bit vectors, about gamma bits per key
 * per level, ranks by popcount prefix.  keys must be distinct (KMP_EINVAL otherwise, where
 * boomphf would not terminate); ids of the n keys are a permutation of 0 .. n-1.  A key outside
 * the set gets an arbitrary id or UINT64_MAX, as with boomphf.  Host buffers; the build and
 * lookups run on the context's device.  kmp_mphf_dev_lookup takes device buffers and a
 * hipStream_t (NULL: default stream).  gamma in [1, 100]. */
int kmp_mphf_build(kmp_ctx* ctx, const uint32_t* keys, uint64_t n, double gamma, kmp_mphf** out);
int kmp_mphf_lookup(const kmp_mphf* m, const uint32_t* keys, uint64_t n, uint64_t* ids);
int kmp_mphf_dev_lookup(const kmp_mphf* m, const uint32_t* d_keys, uint64_t n, uint64_t* d_ids, void* stream);
/* n keys, levels used, total level bits, keys in the fallback table; any pointer may be NULL */
int kmp_mphf_info(const kmp_mphf* m, uint64_t* n, uint32_t* levels, uint64_t* bits, uint64_t* n_fallback);
void kmp_mphf_free(kmp_mphf* m);

/* ------------------------------------------------------------------ pairs ---------- */
/* Fused Graph::new (mod.rs:39-193) + remove_uninteresting_edges (mod.rs:549-697) +
 * combine_edges (mod.rs:322-546): every pair p<q with w = |K(p) ∩ K(q)| >= min_shared
 * (and differing classes when required), w = the collapsed KmerEdge::Group length.
 * Requires kmp_build_sets for the same k.  Result is library-owned. */
int kmp_pairs(kmp_ctx* ctx, const kmp_pair_opts* opts, kmp_edges** out);
int kmp_edges_count(const kmp_edges* e, uint64_t* n);
/* copies up to cap edges; *n = total; KMP_EOVERFLOW if cap < total.  Any output pointer
 * may be NULL.  score[] is w for KMP_SCORE_COUNT, Jaccard w/(S_p+S_q-w) otherwise. */
int kmp_edges_get(const kmp_edges* e, uint32_t* p, uint32_t* q, uint32_t* w, float* score,
                  uint64_t cap, uint64_t* n);

/* Config 5 of SURVEY.md §8d (k = 5 and k = 7 combined): w_k is computed independently for each k
 * in ks[0..nk) (nk <= KMP_MULTI_K_MAX, distinct k in 1..7), and an edge is emitted when any w_k
 * >= min_shared (classes differing as opts asks).  The per-k canonical lists are merged by
 * (p, q): w = Σ_k w_k, score = Σ_k score_k (COUNT or BLOSUM; JACCARD -> KMP_EINVAL).  Runs
 * kmp_build_sets for every k in turn: the context's sets are those of ks[nk-1] afterwards.
 * kmp_edges_get_wk: the weights w_{ks[j]} of every merged edge (0 where that k shares none).
 * A build extension: the reference has one k per run (main.rs), so parity is unpinned. */
/* Bounded memory (config 5: 10^10-10^11 (k-mer, pair) incidences).  kmp_pairs (engine AUTO /
 * RESIDUES on one GPU) and kmp_pairs_multi_k run the rows in passes of consecutive row ranges
 * when the batch is large (more than 2^26 windows) or a pass budget is set: each pass expands
 * only the pairs whose smaller protein lies in its rows, keeping the batch's keys, grouping and
 * heavy-path compaction from the first pass (kmp_postings_set_reuse), and appends its edges
 * (canonical: the ranges are consecutive).  The planner sizes each pass to 3/4 of `keys` pair
 * keys from the densest incidence rate measured so far (the first pass is a probe of N/256
 * rows).  keys = 0 (default): from the free device memory.  kmp_ctx_last_passes: passes of the
 * last call. */
int kmp_ctx_set_pass_keys(kmp_ctx* ctx, uint64_t keys);
/* kmp_ctx_set_direct_tail: kmp_pairs_stream's fused multi-k reduction writes each pass's edges in
 * place (default 1; kmp_postings_set_direct) or (0) stages them and emits after a scan. */
int kmp_ctx_set_direct_tail(kmp_ctx* ctx, int enable);
/* kmp_ctx_set_flat_heavy: kmp_pairs_stream's passes expand frequent k-mers by rows (default 1;
 * kmp_postings_set_flat_heavy) or by per-k-mer tiles (0). */
int kmp_ctx_set_flat_heavy(kmp_ctx* ctx, int enable);
/* Sub-blocks of the last kmp_pairs_stream that the in-place reduce took in windows of pair positions
 * (above its LDS sort capacity: a row pairing many times with few partners); staged: the ones the
 * overflow sort finished. */
uint64_t kmp_ctx_last_tail_windows(const kmp_ctx* ctx);
uint32_t kmp_ctx_last_passes(const kmp_ctx* ctx);
#define KMP_MULTI_K_MAX 4
int kmp_pairs_multi_k(kmp_ctx* ctx, const kmp_pair_opts* opts, const int* ks, uint32_t nk, kmp_edges** out);
int kmp_edges_get_wk(const kmp_edges* e, uint32_t j, uint32_t* wk, uint64_t cap, uint64_t* n);
void kmp_edges_free(kmp_edges* e);

/* ------------------------------------------------------------------ streamed pairs - */
/* Edges streamed per row pass instead of returned whole (config 5, SURVEY.md §8d: at k = 5 the
 * 10^6-protein batch has ~10^11 edges, more than one GPU's HBM or the host can hold).  The rows run
 * in bounded-memory passes (kmp_ctx_set_pass_keys) as in kmp_pairs_multi_k; each pass's edges — the
 * canonical list's consecutive block of the pairs whose smaller protein is in [row_lo, row_hi) —
 * are handed to `sink` as one chunk, then the buffers are reused.  ks[0..nk): one k (nk = 1, the
 * reference's kmp_pairs) or the config-5 union (w = Σ_k w_k, score = Σ_k score_k, w_k in wk[]).
 * score: KMP_SCORE_COUNT (score = w) or KMP_SCORE_BLOSUM (the integer BLOSUM score, summed inside
 * the pair reduction).  sink_on_device: 1 — the chunk's arrays are device pointers on
 * chunk->device, valid during the call (the stream is synchronised before and after); 0 — host
 * copies.  sink may be NULL (the summary only); a nonzero return from it stops the stream and is
 * returned.  summary (may be NULL): the reference's counters over the whole list and a digest
 * computed on the device (below).  Multi-GPU contexts: each rank streams its own rows (the row
 * split, kmp_row_split), chunks arrive from one host thread per rank one at a time (the sink is
 * never called concurrently) with chunk->rank set; per rank the chunks ascend. */
#define KMP_DIGEST_SEGMENTS 64
typedef struct {
    uint32_t rank;            /* multi-GPU: the rank (0 on one GPU) */
    int device;               /* HIP device of the arrays when on_device */
    uint32_t row_lo, row_hi;  /* every edge (p, q) with row_lo <= p < row_hi, and only those */
    uint64_t n;               /* edges in the chunk, canonical (p, q) order */
    int on_device;
    const uint32_t *p, *q, *w;
    const uint32_t* score;    /* COUNT: w; BLOSUM: the integer score */
    const uint32_t* wk[KMP_MULTI_K_MAX];  /* w of ks[j] (0 where that k shares none); NULL past nk */
} kmp_edge_chunk;
typedef int (*kmp_edge_sink)(void* user, const kmp_edge_chunk* chunk);
/* Counters over the streamed list (mod.rs:545 n_edges, :695 sum_w_diff, :242 n_align) and its
 * digest: Σ over the edges of kmp_edge_digest_term(p, q, w, score, w_{ks[0]}) mod 2^64, in total
 * and per row segment (segment of p = p * KMP_DIGEST_SEGMENTS / N).  ordered = 1 when every chunk
 * was strictly (p, q)-ascending inside its rows (then equal digests mean equal lists up to 64-bit
 * collisions: an ascending list is determined by its set). */
typedef struct {
    uint64_t n_edges, sum_w, sum_score, n_align, sum_w_diff, incidences;
    uint64_t digest;
    uint64_t seg_edges[KMP_DIGEST_SEGMENTS];
    uint64_t seg_digest[KMP_DIGEST_SEGMENTS];
    uint32_t passes;
    int32_t ordered;
    /* device time summed over the passes (and ranks), HIP events on each lane's stream: the
     * grouping + expansion of ks[0] (front, buckets, heavy path), of the other k, the pair
     * reduction (row-block tail, overflow sort, emit; nk > 2: + merge), the summary kernel */
    float stage_ms[4];
} kmp_stream_summary;
int kmp_pairs_stream(kmp_ctx* ctx, const kmp_pair_opts* opts, const int* ks, uint32_t nk, int sink_on_device,
                     kmp_edge_sink sink, void* user, kmp_stream_summary* summary);
/* The rows kmp_pairs_stream covers: [row_lo, row_hi) (row_hi 0: every row, the default).  The unit
 * of a multi-process split — one process per GPU, each streaming its kmp_row_split share of the
 * pair space with no exchange (a multi-GPU context splits [row_lo, row_hi) over its ranks by
 * equal pair mass instead). */
int kmp_ctx_set_rows(kmp_ctx* ctx, uint32_t row_lo, uint32_t row_hi);
/* The digest term of one edge: with a = p << 32 | q, b = w << 32 | score, m(z) = splitmix64's
 * finaliser (z += 0x9E3779B97F4A7C15; z = (z ^ z >> 30) * 0xBF58476D1CE4E5B9;
 * z = (z ^ z >> 27) * 0x94D049BB133111EB; z ^ z >> 31): m(a ^ m(b ^ m(w0))). */
uint64_t kmp_edge_digest_term(uint32_t p, uint32_t q, uint32_t w, uint32_t score, uint32_t w0);

/* ------------------------------------------------------------------ edge k-mers ---- */
/* The shared k-mers behind each edge's w: KmerEdge::get_kmers (edge.rs:119-124), i.e. the
 * KmerEdgeGroup.kmers that combine_edges concatenates (mod.rs:415-417; edge.rs:67-81).
 * kmp_edges_kmers computes them on the device from the context's current sets (the
 * kmp_build_sets the edges came from; KMP_EINVAL if an edge's intersection is not w long) and
 * attaches them to e:
 *   KMP_KMERS_CODES: radix-21 codes, ascending;
 *   KMP_KMERS_IDS: repeat-MPHF ids (kmp_get_df's id space), ascending as in the reference; also
 *     sets each edge's reference key, its index in the reference's final edge list, ordered by
 *     (min shared id, p, q) (combine_edges with one thread).
 * kmp_edges_get_kmers: CSR, edge i owns kmers[offsets[i] .. offsets[i+1]) (offsets: count+1,
 * may be NULL); kmp_edges_reference_keys: count keys (IDS lists only, else KMP_ESTATE). */
enum { KMP_KMERS_CODES = 0, KMP_KMERS_IDS = 1 };
int kmp_edges_kmers(kmp_ctx* ctx, kmp_edges* e, int space);
int kmp_edges_get_kmers(const kmp_edges* e, uint64_t* offsets, uint32_t* kmers, uint64_t cap, uint64_t* n);
int kmp_edges_reference_keys(const kmp_edges* e, uint64_t* keys, uint64_t cap, uint64_t* n);

/* ------------------------------------------------------------------ outputs -------- */
/* align_and_output_pairs' files (mod.rs:195-319, the diamond runs out of scope): for every edge
 * with w > threshold (mod.rs:242; reference 10), out_dir/fasta_files/{edge_key}_{prefix}.fasta
 * for p then q, each ">{id}\n{seq}" with no trailing newline (mod.rs:253-261,273-280), where
 * prefix = id.split_once('|').0 and edge_key is the reference key with IDS lists, the edge index
 * otherwise; out_dir/db_files/ (empty, for diamond makedb) and out_dir/blastp_output.tsv holding
 * the header line of mod.rs:304.  out_dir NULL: ".".  fasta_files/ and db_files/ are removed and
 * recreated first, as the reference's `rm -r` + `mkdir` (mod.rs:202-220).  residues/offsets[n+1]:
 * the loaded batch (residues NULL with candidates: KMP_EINVAL); ids: NUL-separated record ids
 * (kmp_read_fasta).  An id without '|' is KMP_EINVAL (the reference panics).  threads: writer
 * threads.  *n_written: candidate edges. */
int kmp_write_candidates(const kmp_edges* e, const uint8_t* residues, const uint64_t* offsets, uint32_t n,
                         const char* ids, uint64_t ids_bytes, uint32_t threshold, const char* out_dir, int threads,
                         uint64_t* n_written);
/* `println!("Graph right now:\n{graph:#?}")` (main.rs:234; Debug of Graph, KmerEdge, ProteinVertex:
 * mod.rs:700-708, edge.rs:158-174, vertex.rs:159-165): edges in reference order as "Single Kmer"
 * (w == 1) / "Kmer Group" with their MPHF ids, then n "Protein { key, size = degree }".  Needs
 * IDS lists.  path NULL or "-": stdout. */
int kmp_write_graph_debug(const kmp_edges* e, uint32_t n, const char* path, int threads);

/* ------------------------------------------------------------------ device stages -- */
/* Device layout.  Every per-protein u32 array (window codes, K(p), repeat-filtered K(p))
 * lives in one buffer of kmp_set_capacity(N, ΣL) elements; protein p owns the 16-B
 * aligned slot range starting at kmp_set_base(res_off[p], p) = round_up(res_off[p]+4p, 4),
 * L_p + 4 slots long (>= its window count).  No offset scan is needed on the device. */
uint64_t kmp_set_capacity(uint32_t n, uint64_t total_residues);
uint64_t kmp_set_base(uint64_t res_off, uint32_t p);

/* All windows' codes in position order (Protein.five_mers, protein.rs:107-132). */
int kmp_dev_extract(const uint8_t* d_res, const uint64_t* d_res_off, uint32_t n, int k,
                    uint32_t* d_codes, void* stream);
/* Fused extract + per-protein sort + dedup: K(p) ascending in p's slot of d_set, |K(p)| in
 * d_set_len[p].  max_len: longest protein in residues (0 = unknown).  Proteins with more
 * than KMP_LDS_SORT_MAX windows are sorted in global memory in d_scratch (same capacity as
 * d_set; may be NULL when max_len shows none is that long). */
#define KMP_LDS_SORT_MAX 4096
int kmp_dev_build_sets(const uint8_t* d_res, const uint64_t* d_res_off, uint32_t n, int k,
                       uint32_t max_len, uint32_t* d_set, uint32_t* d_set_len, uint32_t* d_scratch,
                       void* stream);
/* 32-bit words of ONE repeat bitmap for k (21^k bits rounded up). */
uint64_t kmp_dev_repeat_bitmap_words(int k);
/* remove_unique_five_mers (protein.rs:151-162): zeroes then fills two bitmaps over the
 * code space (seen once / seen in >= 2 proteins), then compacts every set to its repeat
 * k-mers (order kept) into d_rep / d_rep_len.  d_bits: 2 * kmp_dev_repeat_bitmap_words(k). */
int kmp_dev_filter_repeats(const uint32_t* d_set, const uint32_t* d_set_len, const uint64_t* d_res_off,
                           uint32_t n, int k, uint32_t* d_bits, uint32_t* d_rep, uint32_t* d_rep_len,
                           void* stream);

/* Pair-kernel plan.  The repeat-filtered sets are packed into one dense CSR (dense_off[N+1],
 * ascending within each set).  Proteins are packed greedily in index order into row tiles
 * (Σ len <= tile_cap, count <= rows_max); the column axis [0, N) is cut into chunks of about
 * chunk_cost set entries (chunk_col[c] .. chunk_col[c+1]).  A work item is one row tile
 * against one chunk, restricted to columns after the tile's first row; items are emitted
 * chunk-major (all tiles of chunk 0, then chunk 1, ...) and together cover every pair p < q
 * exactly once. */
typedef struct {
    uint32_t row_beg, row_end;  /* row proteins [row_beg, row_end): one LDS-resident tile */
    uint32_t col_beg, col_end;  /* column proteins [col_beg, col_end): streamed */
} kmp_work_item;

/* Row-tile geometry of the pair kernel (fixed at build time). */
typedef struct {
    uint32_t tile_slots;  /* exact-table entries per row tile */
    uint32_t tile_cap;    /* max set entries per row tile */
    uint32_t rows_max;    /* max proteins per row tile */
    uint32_t threads;     /* workgroup size */
} kmp_pair_geometry;
void kmp_pair_geometry_get(kmp_pair_geometry* g);

/* Host-side planner.  set_len[N]: repeat-filtered set sizes.  Fills dense_off[N+1] and up to
 * cap items (*n_items = items needed; KMP_EOVERFLOW if cap is smaller; call with cap 0 to
 * size).  chunk_cost = 0 picks the default.  A set longer than tile_cap is KMP_EINVAL. */
int kmp_plan_pairs(const uint32_t* set_len, uint32_t n, uint64_t chunk_cost, uint64_t* dense_off,
                   kmp_work_item* items, uint64_t cap, uint64_t* n_items);

/* XCD-aware launch order for an 8-XCD device: the n chunk-major items are dealt to 8 lists
 * (chunk g -> list g % 8) and written as slot 8*s + x = list x's item s, so the workgroups
 * the dispatcher places on one XCD stream the same column chunk through that XCD's L2.
 * Short lists are padded with empty items (row_beg == row_end, a no-op in the kernel).
 * *n_out = slots needed (<= n + 7 * items of one chunk); KMP_EOVERFLOW if cap is smaller.
 * A speed hint only: any order of the items gives the same edges. */
int kmp_order_items_xcd(const kmp_work_item* items, uint64_t n, kmp_work_item* out, uint64_t cap,
                        uint64_t* n_out);

/* Packs the repeat-filtered sets (slot layout) into the dense CSR: d_dense[d_dense_off[p] ...]. */
int kmp_dev_pack_dense(const uint32_t* d_rep, const uint64_t* d_res_off, const uint64_t* d_dense_off,
                       uint32_t n, uint32_t* d_dense, void* stream);

/* The pair kernel over work items [0, n_items): appends (p, q, w) with p < q,
 * w = |K(p) ∩ K(q)| >= min_shared and (if required) class[p] != class[q] to d_p/d_q/d_w in
 * arbitrary order at positions d_count[0]++ (< cap; the counter keeps counting past cap so
 * the caller can resize and rerun).  d_count (one u64) must be zeroed by the caller.
 * col_window: a column length (set entries) that almost every column fits, e.g. the 99.5th
 * percentile (kmp_pair_col_window); it sizes the kernel's register window only — longer
 * columns are handled too, more slowly. */
int kmp_dev_pairs(const uint32_t* d_dense, const uint64_t* d_dense_off, const uint16_t* d_class, uint32_t n,
                  const kmp_work_item* d_items, uint64_t n_items, uint32_t col_window, uint32_t min_shared,
                  int require_class_diff, uint32_t* d_p, uint32_t* d_q, uint32_t* d_w, uint64_t cap,
                  unsigned long long* d_count, void* stream);
/* The column window kmp_dev_pairs should be given for these (planned) set sizes. */
uint32_t kmp_pair_col_window(const uint32_t* set_len, uint32_t n);

/* Pairs of the proteins whose repeat-filtered set is longer than the tile capacity
 * (kmp_pair_geometry.tile_cap): those are planned with length 0 (kmp_plan_pairs never sees
 * them) and counted here against every other protein, from the slot layout of d_rep.  Same
 * output contract as kmp_dev_pairs (shares d_count).  d_long_ids: the long proteins' indices. */
int kmp_dev_pairs_long(const uint32_t* d_rep, const uint32_t* d_rep_len, const uint64_t* d_res_off,
                       const uint16_t* d_class, uint32_t n, const uint32_t* d_long_ids, uint32_t n_long,
                       uint32_t min_shared, int require_class_diff, uint32_t* d_p, uint32_t* d_q, uint32_t* d_w,
                       uint64_t cap, unsigned long long* d_count, void* stream);

/* The postings engine (kmp_postings.hip): one radix sort of (k-mer, protein) keys over all
 * K(p) slots (runs = distinct k-mers, run length = df), expansion of the Σ C(df,2) incidences
 * of every run with df <= heavy_df (class test fused, graph/mod.rs:39-193 + :549-697), radix
 * sort + run-length encoding of the pair keys (combine_edges, mod.rs:322-546).  Writes the
 * edges (p, q, w), w >= min_shared, ALREADY in canonical (p, q) order; *n_edges = count
 * (KMP_EOVERFLOW if cap is smaller: resize and rerun).  Reads the unfiltered K(p) slots
 * (d_set, slots = buffer capacity in elements).  Synchronises `stream` (device counts are
 * read back between phases).  The workspace grows on first use and is reused afterwards.
 * Pairs that share k-mers with df > heavy_df get only their light share here (see
 * kmp_pairs, engine AUTO). */
typedef struct kmp_postings kmp_postings;
#define KMP_POSTINGS_STAGES 6
typedef struct {
    uint64_t sum_S;           /* Σ |K(p)| */
    uint64_t distinct;        /* distinct k-mers (runs) */
    uint64_t repeat;          /* runs with df >= 2 */
    uint64_t sum_cdf2_light;  /* Σ C(df,2) over runs with df <= heavy_df */
    uint64_t max_df;
    uint64_t heavy_entries;   /* Σ df over runs with df > heavy_df */
    uint64_t incidences;      /* class-filtered incidences expanded */
    uint64_t pairs;           /* distinct pairs among them (before min_shared) */
    float stage_ms[KMP_POSTINGS_STAGES]; /* per-stage device time (kmp_postings_set_timing), else 0:
                                            keys, code sort, count + offsets, write, pair sort,
                                            run-length encode + emit */
} kmp_postings_stats;
int kmp_postings_create(kmp_postings** ws);
void kmp_postings_destroy(kmp_postings* ws);
/* Records HIP events between the stages on the call's stream (stats->stage_ms). */
int kmp_postings_set_timing(kmp_postings* ws, int enable);
/* Key layout.  bucketed (default 1): keys grouped by a 2^b-bucket hash of the k-mer (a two-level
 * counting partition from the residues), then one workgroup per bucket groups, deduplicates and
 * expands its k-mers in LDS; a frequent k-mer (more than 128 keys) is spilled whole to the heavy
 * path (sorted, split into tiles of its C(df,2) pairs across workgroups), so no df is too large.
 * 0: always flat (full code sort, scan-based expansion; also the fallback for class ids wider
 * than the bucketed key's class field, 31 - bits(N) bits).
 * kmp_postings_last_layout: KMP_LAYOUT_FLAT, KMP_LAYOUT_BUCKETED (single-synchronisation step,
 * graph-captured from the second call of a shape) or KMP_LAYOUT_BUCKETED_HEAVY (the batch spilled
 * frequent k-mers: the split step with the heavy path).  kmp_postings_last_overflow_blocks: row
 * blocks of the pair tail above the LDS capacity (a protein pairing with thousands of later
 * proteins) that the last call finished with the segmented sort. */
enum { KMP_LAYOUT_FLAT = 0, KMP_LAYOUT_BUCKETED = 1, KMP_LAYOUT_BUCKETED_HEAVY = 2 };
int kmp_postings_set_layout(kmp_postings* ws, int bucketed);
int kmp_postings_last_layout(const kmp_postings* ws);
uint32_t kmp_postings_last_overflow_blocks(const kmp_postings* ws);
/* The row-block tail the last call reduced its pair keys with (combine_edges, graph/mod.rs:322-546):
 * KMP_TAIL_FAST (unscored calls: pair keys into fixed row-block regions, one LDS hash-aggregate +
 * rank per block writing the edges in canonical order at offsets from a decoupled look-back),
 * KMP_TAIL_COUNT (histogram, scan, scatter, block sort, emit: scored / multi-k calls, and a shape
 * whose row-block regions overflowed), or -1 (the flat layout's global sort). */
enum { KMP_TAIL_COUNT = 0, KMP_TAIL_FAST = 1 };
int kmp_postings_last_tail(const kmp_postings* ws);
/* kmp_postings_set_tail: KMP_TAIL_FAST (default: the fast tail where it applies) or KMP_TAIL_COUNT
 * (the counting tail only).  Same edges either way. */
int kmp_postings_set_tail(kmp_postings* ws, int mode);
/* kmp_postings_set_direct: the fused multi-k tail (kmp_dev_pairs_rows_multi, kmp_pairs_stream)
 * writes its edges in place from the sub-block reduce, at offsets from a count launch and a scan
 * (default 1), or (0) stages its runs and emits them after a scan.  Same edges either way. */
int kmp_postings_set_direct(kmp_postings* ws, int enable);
/* kmp_postings_set_flat_heavy: ranged calls with front reuse (the row passes of one batch) expand
 * the frequent k-mers by rows — a per-protein index of the compacted elements, built once, makes
 * a pass's work its own rows' pairs (default 1) — or (0) by per-k-mer tiles.  Same edges. */
int kmp_postings_set_flat_heavy(kmp_postings* ws, int enable);
/* kmp_postings_set_row_span: the rows [lo, hi) every ranged call of the current batch lies in
 * (one rank's share of a row split; default 0, 0: any row).  The per-protein index of the
 * row-driven expansion then covers only them: its count and scatter skip the other proteins'
 * elements.  A call outside the index's rows rebuilds it for every row.  Same edges. */
int kmp_postings_set_row_span(kmp_postings* ws, uint32_t lo, uint32_t hi);
/* The bucketed step as a HIP graph (default 1): captured on the second call with an unchanged
 * shape (pointers, sizes, options, workspace buffers), replayed after that.
 * kmp_postings_graph_replays: calls served by a replay so far.  kmp_postings_reruns: calls (or phases
 * of a split call) run again after a capacity grew — every learned capacity is sized from counts, so
 * the same inputs rerun the same number of times whatever the order of the device's atomics. */
int kmp_postings_set_graph(kmp_postings* ws, int enable);
uint64_t kmp_postings_graph_replays(const kmp_postings* ws);
uint64_t kmp_postings_reruns(const kmp_postings* ws);
/* Bucket partition of the residue path (level 1 is always the counting pass).  AUTO (default):
 * level 2 by cursors — every run of keys reserved with one atomic in its bucket's fixed-capacity
 * region (sized from the hash-uniform mean), no histogram / scan passes — and, for a shape where a
 * region overflows (very frequent k-mers), the counting level 2 from then on.  COUNT: the counting
 * level 2 only.  kmp_postings_last_partition: the level 2 the last call's bucketed front used
 * (KMP_PARTITION_CURSOR or KMP_PARTITION_COUNT; -1 on the flat layout). */
enum { KMP_PARTITION_AUTO = 0, KMP_PARTITION_COUNT = 1, KMP_PARTITION_CURSOR = 2 };
int kmp_postings_set_partition(kmp_postings* ws, int mode);
int kmp_postings_last_partition(const kmp_postings* ws);
/* Front reuse (default 0).  1: a call on the same batch as the last successful call (same device
 * pointers, n, k, slots, options; the caller guarantees the contents are unchanged) keeps that
 * call's keys, bucket grouping and heavy-path compaction and runs only the bucket kernels, the
 * heavy expansion and the tail of its rows — the passes of the bounded-memory mode and the
 * per-k rows of kmp_pairs_multi_k call kmp_dev_pairs_rows this way. */
int kmp_postings_set_reuse(kmp_postings* ws, int enable);
/* Shard-region floor (default 0): the pair-key regions hold at least keys / 64 (+ a quarter) keys
 * each from the next call on.  A stream whose passes are planned to ~keys pair keys sets it once,
 * so its regions are sized before the first pass instead of regrown (a multi-GB reallocation idles
 * the device) as the passes' measured sizes climb.  0: learned only. */
int kmp_postings_set_shard_floor(kmp_postings* ws, uint64_t keys);
int kmp_dev_pairs_postings(kmp_postings* ws, const uint32_t* d_set, const uint32_t* d_set_len,
                           const uint64_t* d_res_off, const uint16_t* d_class, uint32_t n, int k, uint64_t slots,
                           uint32_t heavy_df, uint32_t min_shared, int require_class_diff, uint32_t* d_p,
                           uint32_t* d_q, uint32_t* d_w, uint64_t cap, uint64_t* n_edges,
                           kmp_postings_stats* stats, void* stream);

/* The postings engine straight from the packed residues (the fused device path): one key per
 * k-mer window (Protein::new, protein.rs:82-94) in the same slot layout, so the per-protein
 * sort + dedup of K(p) (main.rs:99-101,187-189) is never materialised — duplicate windows of one
 * protein are adjacent after the stable code sort and count once.  Same output contract and
 * edges as kmp_dev_pairs_postings; stats->sum_S = Σ |K(p)|.  slots = kmp_set_capacity(N, ΣL). */
int kmp_dev_pairs_residues(kmp_postings* ws, const uint8_t* d_res, const uint64_t* d_res_off,
                           const uint16_t* d_class, uint32_t n, int k, uint64_t slots, uint32_t heavy_df,
                           uint32_t min_shared, int require_class_diff, uint32_t* d_p, uint32_t* d_q, uint32_t* d_w,
                           uint64_t cap, uint64_t* n_edges, kmp_postings_stats* stats, void* stream);

/* Pipelined form of kmp_dev_pairs_residues (the reference's main.rs:57-234 run over a stream of
 * batches: one call per batch, back to back).  submit enqueues the step on `stream` and returns a
 * ticket; once the step's HIP graph is captured (the third submission of an unchanged shape), it
 * goes out without a host wait, so the next submission is queued behind it before its read-back is
 * checked and the device does not idle between steps.  kmp_postings_wait(ticket) waits for that
 * step, checks its read-back and returns its edge count and statistics exactly as the synchronous
 * call does; a step whose read-back asks for a rerun (a capacity overflow, a fallback) is run again
 * synchronously at its wait, after the stream has drained.  At most two submissions are
 * outstanding (KMP_ESTATE otherwise); each has its own read-back and stage events.  Edge arrays of
 * two outstanding submissions must differ if the caller reads both (the later step overwrites the
 * earlier's arrays otherwise).  Waits may come in any order; every ticket is waited once. */
int kmp_dev_pairs_residues_submit(kmp_postings* ws, const uint8_t* d_res, const uint64_t* d_res_off,
                                  const uint16_t* d_class, uint32_t n, int k, uint64_t slots, uint32_t heavy_df,
                                  uint32_t min_shared, int require_class_diff, uint32_t* d_p, uint32_t* d_q,
                                  uint32_t* d_w, uint64_t cap, void* stream, uint64_t* ticket);
int kmp_postings_wait(kmp_postings* ws, uint64_t ticket, uint64_t* n_edges, kmp_postings_stats* stats);

/* The residue path restricted to rows [row_lo, row_hi): only the pairs (p, q), p < q, whose
 * smaller protein p lies in the range (every k-mer group still grouped in full, so each pair's
 * w is complete).  The edges come out in canonical order; concatenating the calls of
 * consecutive ranges gives the canonical list.  This is the unit a rank of the multi-GPU split
 * and a pass of the bounded-memory mode run.  KMP_ESTATE: the batch needs the flat layout
 * (class ids too wide), which has no row filter. */
int kmp_dev_pairs_rows(kmp_postings* ws, const uint8_t* d_res, const uint64_t* d_res_off, const uint16_t* d_class,
                       uint32_t n, int k, uint64_t slots, uint32_t heavy_df, uint32_t min_shared,
                       int require_class_diff, uint32_t row_lo, uint32_t row_hi, uint32_t* d_p, uint32_t* d_q,
                       uint32_t* d_w, uint64_t cap, uint64_t* n_edges, kmp_postings_stats* stats, void* stream);
/* The scored residue path (config 5's BLOSUM score; a build extension, parity
 * unpinned): as kmp_dev_pairs_rows, and d_score[i] = Σ over the shared k-mers x of edge i of
 * Σ_j B62[x_j][x_j] (the BLOSUM62 diagonal of blosum.rs:8-30 in residue-code order, code 20 scored
 * 0) as an exact integer.  The score is summed inside the pair reduction: every (k-mer, pair)
 * incidence carries its k-mer's self-score (at most 7 x 11 = 77) in the pair key, so no per-edge
 * set intersection runs.  row_lo = 0, row_hi = n: the whole batch (the unranged step).  A call
 * covers at most kmp_dev_rows_max(n, 1) rows (the u32 row-block key holds the score bits too;
 * 131,072 rows at n = 10^6); more is KMP_EINVAL. */
uint32_t kmp_dev_rows_max(uint32_t n, int scored);  /* scored: 0 no score, 1 score, 2 multi-k (below) */
int kmp_dev_pairs_rows_scored(kmp_postings* ws, const uint8_t* d_res, const uint64_t* d_res_off, const uint16_t* d_class,
                              uint32_t n, int k, uint64_t slots, uint32_t heavy_df, uint32_t min_shared,
                              int require_class_diff, uint32_t row_lo, uint32_t row_hi, uint32_t* d_p, uint32_t* d_q,
                              uint32_t* d_w, uint32_t* d_score, uint64_t cap, uint64_t* n_edges,
                              kmp_postings_stats* stats, void* stream);
/* Config 5's union of two k in ONE reduction ("w5, w7 computed independently per
 * pair; an edge is emitted if w5 >= 1 or w7 >= 1"): ws[j] (two distinct workspaces, kept across
 * calls for front reuse) groups and expands the windows of ks[j], every (k-mer, pair) incidence
 * keyed with its k bit and self-score, and one row-block tail reduces both sets of keys together:
 * per pair w = w0 + w1 (w_j = the shared ks[j]-mers), score = Σ_j BLOSUM score_j, emitted when
 * w0 >= min_shared or w1 >= min_shared (and the classes differ when required).  No per-k lists,
 * no merge.  Rows as kmp_dev_pairs_rows, at most kmp_dev_rows_max(n, 2) per call (65,536 rows at
 * n = 10^6). */
/* stats (may be NULL): stage_ms[0] = the first k's grouping + expansion, [1] the second k's, [2] the
 * fused reduction + emit (HIP events on `stream`); the front statistics are the first k's. */
int kmp_dev_pairs_rows_multi(kmp_postings* const* ws, const int* ks, uint32_t nk, const uint8_t* d_res,
                             const uint64_t* d_res_off, const uint16_t* d_class, uint32_t n, uint64_t slots,
                             uint32_t min_shared, int require_class_diff, uint32_t row_lo, uint32_t row_hi,
                             uint32_t* d_p, uint32_t* d_q, uint32_t* d_w, uint32_t* d_score, uint32_t* d_w0,
                             uint32_t* d_w1, uint64_t cap, uint64_t* n_edges, kmp_postings_stats* stats,
                             void* stream);
/* The multi-GPU k-mer split (the reference's `threads` share the same work through
 * one sorted k-mer list, main.rs:77-122 / mod.rs:81-124).  Rank `part` of `parts` (<= 64):
 *   kmp_dev_split_expand  every window of the batch is keyed, the rank keeps the k-mers of its
 *     share of the bucket hash range (a contiguous range of coarse bins), groups and expands them
 *     (all rows), and routes each pair key (p << bits(N) | q) to the rank owning row p
 *     (kmp_row_split): region d of d_send (cap keys, padded with kNoKey = all ones: the bucket
 *     kernels write it in 64 sub-regions of cap / 64 keys each) is rank d's.  No host
 *     synchronisation (except with the heavy path on: one read-back of the front's spill, which
 *     the rank compacts, plans and expands into its routed keys); d_flags[KMP_SPLIT_FLAGS] and
 *     d_stats[8] (Σ|K(p)|, distinct, repeat,
 *     Σ C(df,2), max df, heavy entries, incidences, 0 — this rank's k-mers) are written on `stream`.
 *     learn: the previous call's flags reduced (max) over the ranks, or NULL for a first call;
 *     every rank grows its capacities from them identically.  A rank whose spill regions kept
 *     overflowing (heavy path) sends no keys and raises RERUN, so every rank reruns in lockstep. 
 *   exchange (the caller's collective): region d of rank g's d_send -> region g of rank d's receive
 *     buffer (an all-to-all of equal splits, cap keys each).
 *   kmp_dev_split_edges   the m = parts * cap received keys -> the canonical edges of rows
 *     [row_lo, row_hi) (the row-block tail), *n_edges; KMP_EOVERFLOW when cap is smaller (grow and
 *     call again with the same keys).  Synchronises `stream` (also when there is nothing to reduce).
 * The rank-order concatenation of the ranks' edges is the canonical list.  Flags: RERUN (a send
 * region, pair-key shard or bucket region overflowed: call expand again with learn, after growing
 * cap to at least MAX_PART when that is the cause), CLASS (class ids too wide: single GPU) and
 * HEAVY (k-mers above the LDS group limit spilled while the rank's heavy path was off: call expand
 * again with learn — every rank turns its heavy path on for the batch, vertex.rs:59-140), LARGE
 * (a bucket above the small kernel's LDS capacity was listed while the rank did not launch the
 * large-bucket kernel: every rank launches it from then on; RERUN is set too). */
enum {
    KMP_SPLIT_RERUN = 0, KMP_SPLIT_CLASS = 1, KMP_SPLIT_HEAVY = 2, KMP_SPLIT_MAX_PART = 3,
    KMP_SPLIT_MAX_SHARD = 4, KMP_SPLIT_BIN_TILES = 5, KMP_SPLIT_CURSOR = 6, KMP_SPLIT_MAX_KEYS = 7,
    KMP_SPLIT_LARGE = 8, KMP_SPLIT_FLAGS = 16
};
int kmp_dev_split_expand(kmp_postings* ws, const uint8_t* d_res, const uint64_t* d_res_off, const uint16_t* d_class,
                         uint32_t n, int k, uint64_t slots, uint32_t heavy_df, int require_class_diff, uint32_t part,
                         uint32_t parts, uint64_t cap, const uint32_t* learn, unsigned long long* d_send,
                         uint32_t* d_flags, unsigned long long* d_stats, void* stream);
int kmp_dev_split_edges(kmp_postings* ws, const unsigned long long* d_keys, uint64_t m, uint32_t n, uint32_t row_lo,
                        uint32_t row_hi, uint32_t min_shared, uint32_t* d_p, uint32_t* d_q, uint32_t* d_w,
                        uint64_t cap, uint64_t* n_edges, void* stream);

/* The k-mer split with a SHARDED START (the default multi-GPU flow of bench.py --gpus N, dist.py):
 * rank `part` holds only the residues its chunks read — chunks [c_lo, c_hi) of the batch's
 * 4,096-slot chunks (kmp_split_plan; slice [res_lo, res_hi) of the packed residues, 16-byte aligned
 * start) — plus the batch's offsets and class ids.  Instead of keying every window (the replicated
 * level 1 of kmp_dev_split_expand), each rank keys its own chunks once and the keys travel:
 *   kmp_dev_split_keys   the rank's windows keyed (radix-21 codes, protein.rs:29-37,107-132) and
 *     ranked by coarse bin; region d of d_ksend (kcap u64 words) receives the keys of rank d's bins
 *     with a run table per chunk (no host synchronisation).  d_flags: RERUN when a region was too
 *     small (MAX_KEYS = the region size that fits, every rank's the same after the max-reduce).
 *   exchange (the caller's collective): an all-to-all of equal splits of kcap words.
 *   kmp_dev_split_group  the received keys (parts regions of kcap words) grouped and expanded like
 *     kmp_dev_split_expand's (its bins, all rows, routed to the row owners in d_send), merging the
 *     keys phase's flags into d_flags (same buffer, same step).
 *   then the pair-key exchange and kmp_dev_split_edges as above.
 * kmp_split_plan: the rank's chunk range, residue slice and the default region size (key_cap). */
typedef struct {
    uint64_t slots;            /* kmp_set_capacity(n, ΣL) */
    uint32_t n_chunks, c_lo, c_hi;
    uint64_t res_lo, res_hi;   /* the residue slice the rank's chunks read */
    uint64_t key_table_words;  /* run-table words at the start of every key region */
    uint64_t key_cap;          /* a default key-region size (u64 words; grown from MAX_KEYS) */
} kmp_split_span;
int kmp_split_plan(const uint64_t* offsets, uint32_t n, int k, uint32_t part, uint32_t parts, kmp_split_span* out);
int kmp_dev_split_keys(kmp_postings* ws, const uint8_t* d_res, uint64_t res_lo, uint64_t res_hi,
                       const uint64_t* d_res_off, const uint16_t* d_class, uint32_t n, int k, uint64_t slots,
                       uint32_t part, uint32_t parts, uint64_t kcap, unsigned long long* d_ksend, uint32_t* d_flags,
                       void* stream);
int kmp_dev_split_group(kmp_postings* ws, const unsigned long long* d_krecv, uint64_t kcap, uint32_t n, int k,
                        uint64_t slots, uint32_t heavy_df, int require_class_diff, uint32_t part, uint32_t parts,
                        uint64_t cap, const uint32_t* learn, unsigned long long* d_send, uint32_t* d_flags,
                        unsigned long long* d_stats, void* stream);

/* Row ranges of a split of the pair space: range d = [start[d], start[d+1]) with start[d] =
 * floor(N (1 - sqrt(1 - d/parts))): a pair belongs to its smaller protein, so the ranges hold about
 * equal pair counts.  start has parts + 1 entries. */
void kmp_row_split(uint32_t n, uint32_t parts, uint32_t* start);

/* Canonical order: sorts n edges by (p, q).  Keys/values are read from d_p/d_q/d_w and the
 * sorted result is written back to them.  d_tmp: kmp_dev_sort_edges_tmp_bytes(n, N) bytes. */
uint64_t kmp_dev_sort_edges_tmp_bytes(uint64_t n, uint32_t n_proteins);
int kmp_dev_sort_edges(uint32_t* d_p, uint32_t* d_q, uint32_t* d_w, uint64_t n, uint32_t n_proteins,
                       void* d_tmp, uint64_t tmp_bytes, void* stream);

/* ------------------------------------------------------------------ host utilities - */
/* FASTA ingest with seq_io semantics (main.rs:62-72): id = header up to the first space,
 * seq = the record's sequence bytes; AMR class = id.split_terminator('|')[3]
 * (protein.rs:135-138) interned to ids in order of first appearance.  Library-owned
 * output buffers; free each with kmp_free_host.  ids: NUL-separated id strings.
 * Multithreaded like the reference's parallel_fasta: the mapped file is cut into byte ranges,
 * each thread parses the records whose header starts in its range; kmp_read_fasta uses
 * min(16, hardware threads), kmp_read_fasta_threads the given count (0: the same default). */
int kmp_read_fasta(const char* path, uint32_t* n, uint8_t** residues, uint64_t** offsets,
                   uint16_t** class_id, char** ids, uint64_t* ids_bytes, uint32_t* n_classes);
int kmp_read_fasta_threads(const char* path, int threads, uint32_t* n, uint8_t** residues, uint64_t** offsets,
                           uint16_t** class_id, char** ids, uint64_t* ids_bytes, uint32_t* n_classes);
/* Synthetic sets of SURVEY.md §8d.  residues is malloc'd (free with kmp_free_host);
 * offsets[N+1], class_id[N], family[N] are caller buffers (class_id/family may be NULL). */
int kmp_synth_packed(uint32_t n, uint64_t seed, int length_law, uint8_t** residues,
                     uint64_t* offsets, uint16_t* class_id, uint32_t* family);
int kmp_synth_write_fasta(const char* path, uint32_t n, uint64_t seed, int length_law);
void kmp_free_host(void* p);

#ifdef __cplusplus
}
#endif

#endif /* KMERPAIR_H */
