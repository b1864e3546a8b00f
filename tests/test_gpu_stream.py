"""GPU parity of config 5's path as the library runs it at scale (log-uniform
lengths 50-2000, k = 5 and 7 combined, BLOSUM-weighted score):

  - the BLOSUM score summed inside the pair reduction (kmp_dev_pairs_rows_scored: every
    (k-mer, pair) incidence carries its k-mer's self-score), on the light and heavy paths and the
    overflow-block sort, against the oracle's restatement (oracle/kmp_oracle.c orc_stream,
    orc_pair_scores) over EVERY edge;
  - kmp_pairs_stream: edges handed over per row pass (host and device sinks), the chunks
    concatenating to the oracle's canonical union, and the device summary (counters, digest,
    per-segment digests) equal to the oracle's.

The BLOSUM score is a build extension (parity unpinned; the oracle's restatement is pinned by the
hand-checked known answers of test_oracle.py / test_gpu_parity.py::test_blosum_scores)."""
import numpy as np
import pytest

from common import uniprot
import uniprot_kmer_based_clustering_amd as K
from uniprot_kmer_based_clustering_amd import _lib

pytestmark = pytest.mark.gpu

BLOSUM = _lib.KMP_SCORE_BLOSUM


def assert_summary(got, want):
    for key in ("n_edges", "sum_w", "sum_score", "n_align", "sum_w_diff", "incidences", "digest"):
        assert got[key] == want[key], (key, got[key], want[key])
    assert got["seg_edges"] == want["seg_edges"]
    assert got["seg_digest"] == want["seg_digest"]
    assert got["ordered"] == 1


@pytest.mark.parametrize("k", [5, 7])
@pytest.mark.parametrize("keys", [0, 1 << 21])
def test_scored_reduction_every_edge(oracle_mod, k, keys):
    """kmp_pairs(BLOSUM) on the residues engine: scores from the scored reduction, in one call
    and in several passes, equal the oracle's for every edge; min_shared filters on w."""
    b = K.synth(20000, 5, 1)
    o = oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=k, threads=16)
    _, (p, q, w, s, _) = oracle_mod.stream([o], collect=True, threads=16)
    with K.KmerPairEngine(0, 4) as e:
        e.load(b)
        e.build_sets(k)
        e.set_pass_keys(keys)
        got = e.pairs(score=BLOSUM)
        assert (e.last_passes > 1) == (keys != 0)
        np.testing.assert_array_equal(got.p, p)
        np.testing.assert_array_equal(got.q, q)
        np.testing.assert_array_equal(got.w, w)
        np.testing.assert_array_equal(got.score, s.astype(np.float32))
        got2 = e.pairs(score=BLOSUM, min_shared=2)
    _, (p2, q2, w2, s2, _) = oracle_mod.stream([o], min_shared=2, collect=True, threads=16)
    np.testing.assert_array_equal(got2.q, q2)
    np.testing.assert_array_equal(got2.w, w2)
    np.testing.assert_array_equal(got2.score, s2.astype(np.float32))


def test_scored_heavy_path_uniprot_k5(oracle_mod):
    """The reference's dataset at k = 5 (frequent 5-mers: the heavy path; rows pairing with
    thousands of later proteins: the overflow-block sort): BLOSUM scores of all 4.35M edges from
    the scored reduction equal the oracle's."""
    res, off, cls, _ = uniprot()
    o = oracle_mod.Oracle(res, off, cls, k=5, threads=16)
    p, q, w = o.pairs()
    want = o.pair_scores(p, q, threads=16)
    with K.KmerPairEngine(0, 4) as e:
        e.load(K.Proteins(res, off, cls))
        e.build_sets(5)
        got = e.pairs(score=BLOSUM)
        assert len(got) == 4_350_628
        np.testing.assert_array_equal(got.p, p)
        np.testing.assert_array_equal(got.q, q)
        np.testing.assert_array_equal(got.w, w)
        np.testing.assert_array_equal(got.score, want.astype(np.float32))
        e.set_pass_keys(1 << 22)  # passes: the heavy tiles and overflow blocks of each row range
        got = e.pairs(score=BLOSUM)
        assert e.last_passes > 1
        np.testing.assert_array_equal(got.score, want.astype(np.float32))


@pytest.mark.parametrize("direct,flat", [(True, True), (False, False)])
@pytest.mark.parametrize("ks", [(5,), (5, 7)])
def test_stream_host_chunks_concatenate(oracle_mod, ks, direct, flat):
    """kmp_pairs_stream with a host sink: the chunks (consecutive row ranges, each canonical)
    concatenate to the oracle's union edge list (w, score, every w_k), and the summary equals the
    oracle's digest and counters.  direct: the fused reduction writes each pass's edges in place
    (pt_reduce_direct_kernel), else it stages them and emits after a scan; flat: the frequent k-mers
    are expanded by rows (heavy_flat_kernel), else by per-k-mer tiles."""
    b = K.synth(30000, 5, 1)
    orcs = [oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=k, threads=16) for k in ks]
    want, (p, q, w, s, wk) = oracle_mod.stream(orcs, collect=True, threads=16)
    chunks = []
    with K.KmerPairEngine(0, 8) as e:
        e.load(b)
        e.set_direct_tail(direct)
        e.set_flat_heavy(flat)
        e.set_pass_keys(1 << 21)
        sm = e.pairs_stream(ks, score=BLOSUM, sink=chunks.append)
    assert sm["passes"] == len(chunks) > 1
    assert chunks[0]["row_lo"] == 0 and chunks[-1]["row_hi"] == 30000
    assert all(a["row_hi"] == c["row_lo"] for a, c in zip(chunks, chunks[1:]))
    cat = {key: np.concatenate([c[key] for c in chunks]) for key in ("p", "q", "w", "score")}
    np.testing.assert_array_equal(cat["p"], p)
    np.testing.assert_array_equal(cat["q"], q)
    np.testing.assert_array_equal(cat["w"], w)
    np.testing.assert_array_equal(cat["score"], s)
    for j in range(len(ks)):
        np.testing.assert_array_equal(np.concatenate([c["wk"][j] for c in chunks]), wk[j])
    assert_summary(sm, want)


@pytest.mark.parametrize("direct,flat", [(True, True), (False, False), (True, False)])
def test_stream_count_and_filters(oracle_mod, direct, flat):
    """COUNT score (score = w), min_shared = 3 (kept when either k reaches it) and the class filter
    off, streamed over passes: summary equal to the oracle's (in-place and staged reduction)."""
    b = K.synth(15000, 5, 1)
    orcs = [oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=k, threads=16) for k in (5, 7)]
    with K.KmerPairEngine(0, 8) as e:
        e.load(b)
        e.set_direct_tail(direct)
        e.set_flat_heavy(flat)
        e.set_pass_keys(1 << 20)
        for kw in ({"min_shared": 3}, {"require_class_diff": False}, {}):
            want = oracle_mod.stream(orcs, blosum=False, threads=16, **kw)
            sm = e.pairs_stream((5, 7), score=_lib.KMP_SCORE_COUNT, **kw)
            assert_summary(sm, want)
            assert sm["sum_score"] == sm["sum_w"]


@pytest.mark.parametrize("direct", [True, False])
def test_stream_dense_pairs_windows(oracle_mod, direct):
    """Rows that pair many times with few partners: four copies of one 3,000-residue protein (rows
    0, 1, 9,000 and 19,000, four classes) in 20,000 synthetic ones, k = 5 + 7 — pairs of ~6,000
    shared k-mers, so the row blocks of rows 0 and 1 hold fine bins far above the reduce's LDS sort
    capacity: the in-place reduce takes them in windows of pair positions (the staged one, the
    overflow sort).  Every edge, score and w_k equal to the oracle's."""
    base = K.synth(20000, 5, 1)
    rng = np.random.default_rng(77)
    dup = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)[rng.integers(0, 20, 3000)]
    seqs = [base.residues[base.offsets[i]:base.offsets[i + 1]] for i in range(base.n)]
    cls = base.class_id.astype(np.uint16).copy()
    for j, row in enumerate((0, 1, 9000, 19000)):
        seqs[row] = dup
        cls[row] = j + 1
    lens = np.array([len(x) for x in seqs], np.int64)
    off = np.zeros(len(seqs) + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    b = K.Proteins(np.concatenate(seqs).astype(np.uint8), off, cls)
    orcs = [oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=k, threads=16) for k in (5, 7)]
    want, (p, q, w, s, wk) = oracle_mod.stream(orcs, collect=True, threads=16)
    assert w.max() > 5000
    chunks = []
    with K.KmerPairEngine(0, 8) as e:
        e.load(b)
        e.set_direct_tail(direct)
        sm = e.pairs_stream((5, 7), score=BLOSUM, sink=chunks.append)
        assert e.last_tail_windows >= 2
    cat = {key: np.concatenate([c[key] for c in chunks]) for key in ("p", "q", "w", "score")}
    np.testing.assert_array_equal(cat["p"], p)
    np.testing.assert_array_equal(cat["q"], q)
    np.testing.assert_array_equal(cat["w"], w)
    np.testing.assert_array_equal(cat["score"], s)
    for j in range(2):
        np.testing.assert_array_equal(np.concatenate([c["wk"][j] for c in chunks]), wk[j])
    assert_summary(sm, want)


def test_stream_device_sink_100k(oracle_mod):
    """Config 5's lengths at N = 100,000, k = 5 + 7, BLOSUM (8.3e8 edges, passes chosen by the
    library): device-sink chunks (device pointers, never copied) and the summary equal to the
    oracle's digest."""
    b = K.synth(100_000, 5, 1)
    orcs = [oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=k, threads=16) for k in (5, 7)]
    want = oracle_mod.stream(orcs, threads=16)
    seen = []
    with K.KmerPairEngine(0, 8) as e:
        e.load(b)
        sm = e.pairs_stream((5, 7), score=BLOSUM, on_device=True,
                            sink=lambda c: seen.append((c["row_lo"], c["row_hi"], c["n"], c["on_device"])))
    assert want["n_edges"] > 500_000_000
    assert all(x[3] for x in seen) and sum(x[2] for x in seen) == want["n_edges"]
    assert_summary(sm, want)


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0, 0]])
def test_stream_multi_rank_rows(oracle_mod, devices):
    """A multi-GPU context (G virtual ranks on the box's GPU): each rank streams its kmp_row_split
    rows in its own passes; the summary equals the oracle's and each rank's chunks tile its rows.
    kmp_ctx_set_rows restricts the stream (the multi-process split), here split again over the
    ranks by pair mass."""
    b = K.synth(20000, 5, 1)
    orcs = [oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=k, threads=16) for k in (5, 7)]
    want = oracle_mod.stream(orcs, threads=16)
    G = len(devices)
    seen = []
    with K.KmerPairEngine(cpu_threads=4, devices=devices) as e:
        e.load(b)
        e.set_pass_keys(1 << 21)
        sm = e.pairs_stream((5, 7), score=BLOSUM, sink=lambda c: seen.append((c["rank"], c["row_lo"], c["row_hi"])))
        assert_summary(sm, want)
        start = _lib.row_split(20000, G)
        for g in range(G):
            mine = sorted((lo, hi) for r, lo, hi in seen if r == g)
            assert mine[0][0] == start[g] and mine[-1][1] == start[g + 1]
            assert all(x[1] == y[0] for x, y in zip(mine, mine[1:]))
        e.set_rows(5000, 12000)
        part = oracle_mod.stream(orcs, 5000, 12000, threads=16)
        assert_summary(e.pairs_stream((5, 7), score=BLOSUM), part)
