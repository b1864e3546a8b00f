"""GPU parity: libkmerpair (HIP, gfx950) against the oracle and the golden fixtures.
Integer path => bit-exact everywhere.  All calls go through the C ABI."""
import numpy as np
import pytest

from common import (edges_sha256, load_json, make_batch, read_edges_tsv, slice_proteins, tiny,
                    uniprot)
import uniprot_kmer_based_clustering_amd as K
from uniprot_kmer_based_clustering_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = K.KmerPairEngine(0, 4)
    yield e
    e.close()


def batch(res, off, cls):
    return K.Proteins(res, off, cls)


def assert_edges(edges, p, q, w):
    np.testing.assert_array_equal(edges.p, p)
    np.testing.assert_array_equal(edges.q, q)
    np.testing.assert_array_equal(edges.w, w)


ENGINES = [_lib.KMP_ENGINE_POSTINGS, _lib.KMP_ENGINE_TILES, _lib.KMP_ENGINE_RESIDUES]
ENGINE_IDS = ["postings", "tiles", "residues"]


@pytest.fixture(scope="module")
def uni():
    res, off, cls, _ = uniprot()
    return res, off, cls


@pytest.mark.parametrize("eng", ENGINES, ids=ENGINE_IDS)
@pytest.mark.parametrize("k", [5, 7])
def test_tiny_golden(engine, k, eng):
    res, off, cls, _ = tiny()
    engine.load(batch(res, off, cls))
    engine.build_sets(k)
    e = engine.pairs(engine=eng)
    assert_edges(e, *read_edges_tsv(f"tiny_k{k}_edges.tsv"))
    c = engine.counters()
    for key, val in load_json("tiny_counters.json")[str(k)].items():
        if key in c:
            assert c[key] == val, key


@pytest.mark.parametrize("k", [5, 7])
def test_kmers_and_sets_match_oracle(engine, oracle_mod, uni, k):
    res, off, cls = uni
    o = oracle_mod.Oracle(res, off, cls, k=k, threads=8)
    engine.load(batch(res, off, cls))
    engine.extract(k)
    codes, wo = o.codes(), o.win_off()
    so, sv = o.sets()
    rng = np.random.default_rng(k)
    sample = np.concatenate([[0, 1, len(off) - 2], rng.choice(len(off) - 1, 300, replace=False)])
    for p in sample:
        np.testing.assert_array_equal(engine.get_kmers(int(p)), codes[wo[p]:wo[p + 1]])
    engine.build_sets(k)
    for p in sample:
        np.testing.assert_array_equal(engine.get_set(int(p)), sv[so[p]:so[p + 1]])
    c, oc = engine.counters(), o.counters()
    for key in ("n_windows", "sum_S", "distinct", "repeat", "sum_cdf2", "max_df"):
        assert c[key] == oc[key], key


@pytest.mark.parametrize("eng", ENGINES, ids=ENGINE_IDS)
@pytest.mark.parametrize("k", [5, 7])
def test_uniprot_edges_bit_exact(engine, uni, k, eng):
    res, off, cls = uni
    g = load_json("uniprot_counters.json")[str(k)]
    engine.load(batch(res, off, cls))
    engine.build_sets(k)
    e = engine.pairs(engine=eng)
    assert len(e) == g["n_edges"]
    assert edges_sha256(e.p, e.q, e.w) == g["edges_sha256"]
    c = engine.counters()
    for key in ("distinct", "repeat", "sum_cdf2", "sum_w_diff", "n_edges", "n_align", "sum_S", "max_df"):
        assert c[key] == g[key], key


@pytest.mark.parametrize("eng", ENGINES, ids=ENGINE_IDS)
def test_uniprot_options_match_oracle(engine, oracle_mod, uni, eng):
    res, off, cls = uni
    idx = np.arange(0, len(off) - 1, 3)
    r2, o2, c2 = slice_proteins(res, off, cls, idx)
    o = oracle_mod.Oracle(r2, o2, c2, k=5, threads=8)
    engine.load(batch(r2, o2, c2))
    engine.build_sets(5)
    for min_shared, diff in ((1, False), (4, True), (11, False)):
        e = engine.pairs(min_shared=min_shared, require_class_diff=diff, engine=eng)
        assert_edges(e, *o.pairs(min_shared=min_shared, require_class_diff=diff))


def test_jaccard_scores(engine, oracle_mod, uni):
    res, off, cls = uni
    idx = np.arange(0, len(off) - 1, 5)
    r2, o2, c2 = slice_proteins(res, off, cls, idx)
    engine.load(batch(r2, o2, c2))
    engine.build_sets(7)
    e = engine.pairs(score=_lib.KMP_SCORE_JACCARD)
    so, _ = oracle_mod.Oracle(r2, o2, c2, k=7).sets()
    S = np.diff(so).astype(np.float32)
    want = e.w.astype(np.float32) / (S[e.p] + S[e.q] - e.w.astype(np.float32))
    np.testing.assert_array_equal(e.score, want)  # one correctly rounded f32 divide, tolerance 0
    assert np.all((e.score > 0) & (e.score <= 1))


@pytest.mark.parametrize("k", [5, 7])
def test_blosum_scores(engine, oracle_mod, k):
    """KMP_SCORE_BLOSUM (SURVEY.md §8d config-5 scoring, a build extension): every edge's score
    equals the oracle's Σ over shared k-mers of the BLOSUM62 diagonal, exactly (integers in f32),
    for every engine; plus the hand-checked batch of test_oracle.py."""
    b = K.synth(3000, 5, 1)  # config-5 length law (log-uniform 50-2000)
    o = oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=k, threads=8)
    p, q, w = o.pairs()
    want = o.blosum_scores(p, q).astype(np.float32)
    engine.load(b)
    engine.build_sets(k)
    for eng in ENGINES:
        e = engine.pairs(score=_lib.KMP_SCORE_BLOSUM, engine=eng)
        assert_edges(e, p, q, w)
        np.testing.assert_array_equal(e.score, want)
    assert len(p) > 100
    seqs = [b"CCCCCAWWWWW", b"GGCCCCCGG", b"WWWWWPP", b"XCCCC*", b"XCCCC*A"]
    res, off, cls = make_batch(seqs, ["a", "b", "c", "d", "e"])
    engine.load(batch(res, off, cls))
    engine.build_sets(5)
    e = engine.pairs(score=_lib.KMP_SCORE_BLOSUM)
    got = dict(zip(zip(e.p.tolist(), e.q.tolist()), e.score.tolist()))
    assert got == {(0, 1): 45.0, (0, 2): 55.0, (3, 4): 72.0}


def test_multi_k_config5(engine, oracle_mod):
    """Config-5 shape (log-uniform lengths, k = 5 and 7 combined, BLOSUM score): the union of the
    per-k oracle edge lists with w_5, w_7 kept, w = w_5 + w_7, score = Σ_k BLOSUM score."""
    b = K.synth(4000, 5, 1)
    want = {}
    for k in (5, 7):
        o = oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=k, threads=8)
        p, q, w = o.pairs()
        s = o.blosum_scores(p, q)
        for a, c, x, y in zip(p.tolist(), q.tolist(), w.tolist(), s.tolist()):
            d = want.setdefault((a, c), {5: 0, 7: 0, "s": 0})
            d[k] = x
            d["s"] += y
    engine.load(b)
    e, wk = engine.pairs_multi_k((5, 7), score=_lib.KMP_SCORE_BLOSUM)
    keys = sorted(want)
    assert len(e) == len(keys) and len(keys) > 100
    np.testing.assert_array_equal(e.p, np.array([a for a, _ in keys], np.uint32))
    np.testing.assert_array_equal(e.q, np.array([c for _, c in keys], np.uint32))
    np.testing.assert_array_equal(wk[5], np.array([want[x][5] for x in keys], np.uint32))
    np.testing.assert_array_equal(wk[7], np.array([want[x][7] for x in keys], np.uint32))
    np.testing.assert_array_equal(e.w, wk[5] + wk[7])
    np.testing.assert_array_equal(e.score, np.array([want[x]["s"] for x in keys], np.float32))
    assert (wk[7] > 0).sum() < (wk[5] > 0).sum()  # k = 7 shares less
    with pytest.raises(_lib.KmpError):
        engine.pairs_multi_k((5, 5))


@pytest.mark.parametrize("eng", ENGINES, ids=ENGINE_IDS)
@pytest.mark.parametrize("n,seed,law,k", [(10000, 2, 0, 7), (3000, 5, 1, 5), (3000, 5, 1, 7)])
def test_synthetic_bit_exact(engine, oracle_mod, n, seed, law, k, eng):
    b = K.synth(n, seed, law)
    o = oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=k, threads=8)
    engine.load(b)
    engine.build_sets(k)
    e = engine.pairs(engine=eng)
    assert_edges(e, *o.pairs())
    assert len(e) > 0


def test_config3_full_size_bit_exact(engine, oracle_mod):
    """Config 3 (100k synthetic, len~300, k=7) against the oracle, end to end, both engines."""
    b = K.synth(100000, 3)
    o = oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=7, threads=16)
    engine.load(b)
    engine.build_sets(7)
    p, q, w = o.pairs()
    for eng in ENGINES:
        e = engine.pairs(engine=eng)
        assert len(e) == len(p) and len(e) > 1_000_000
        assert_edges(e, p, q, w)
    c, oc = engine.counters(), o.counters()
    for key in ("distinct", "repeat", "sum_cdf2", "sum_w_diff", "n_edges", "n_align"):
        assert c[key] == oc[key], key


def test_long_proteins_global_sort_path(engine, oracle_mod):
    """Windows > KMP_LDS_SORT_MAX (global-memory sort) and repeat-filtered sets > the tile
    capacity (long-protein pair kernel), mixed with ordinary proteins."""
    rng = np.random.default_rng(7)
    alpha = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", dtype=np.uint8)
    rnd = lambda m: alpha[rng.integers(0, 20, m)].tobytes()  # noqa: E731
    base = rnd(21000)
    other = rnd(6000)
    seqs = [base[:300], base, rnd(500), base[2000:19500], other + base[5000:8000], b"MK" * 2500,
            base[4000:4300], other[:4000] + rnd(9000), base[:17500], rnd(200) + other[100:400]]
    cls = ["a", "b", "c", "d", "a", "b", "c", "d", "a", "b"]
    res, off, cl = make_batch(seqs, cls)
    o = oracle_mod.Oracle(res, off, cl, k=5)
    engine.load(batch(res, off, cl))
    engine.build_sets(5)
    so, sv = o.sets()
    for p in range(len(seqs)):
        np.testing.assert_array_equal(engine.get_set(p), sv[so[p]:so[p + 1]])
    rc, _ = o.repeat()
    rep_len = [int(np.isin(sv[so[p]:so[p + 1]], rc).sum()) for p in range(len(seqs))]
    assert sum(r > K._lib.geometry().tile_cap for r in rep_len) >= 2  # the long path really runs
    for eng in ENGINES:
        for diff in (False, True):
            assert_edges(engine.pairs(require_class_diff=diff, engine=eng), *o.pairs(require_class_diff=diff))
        for ms in (1, 50, 3000):
            assert_edges(engine.pairs(min_shared=ms, require_class_diff=False, engine=eng),
                         *o.pairs(min_shared=ms, require_class_diff=False))


def test_edge_cases(engine, oracle_mod):
    # L < k, L == k, empty records, all-one-class, identical proteins, unknown residues
    seqs = [b"", b"ACD", b"ACDEF", b"ACDEF", b"XXXXXXX", b"zzzzzzz", b"ACDEFACDEF", b"WWWW"]
    for classes in (["a"] * 8, list("abcdefgh")):
        res, off, cls = make_batch(seqs, classes)
        engine.load(batch(res, off, cls))
        for k in (1, 2, 5, 7):
            o = oracle_mod.Oracle(res, off, cls, k=k)
            engine.build_sets(k)
            for eng in ENGINES:
                assert_edges(engine.pairs(engine=eng), *o.pairs())
                assert_edges(engine.pairs(require_class_diff=False, engine=eng), *o.pairs(require_class_diff=False))
    # empty batch
    res, off, cls = make_batch([], [])
    engine.load(batch(res, off, cls))
    engine.build_sets(5)
    for eng in ENGINES:
        assert len(engine.pairs(engine=eng)) == 0


@pytest.mark.parametrize("n", [700, 3000, 60000])
def test_bucketed_small_batches(oracle_mod, n):
    """Small and mid-size batches (below rocprim's 1M-key merge-sort threshold) stay on the
    bucketed layout and are exact: regression for the rocprim 4.2 default-config sort defect on
    bit ranges [b, 64) (kmp_postings.hip SortCfg, tools/sort_check.hip)."""
    import torch
    from uniprot_kmer_based_clustering_amd.device import DevicePipeline
    b = K.synth(n, 13)
    p, q, w = oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=7, threads=8).pairs()
    pipe = DevicePipeline(b, 7, "cuda:0")
    for _ in range(2):
        m = pipe.step(engine="residues")
        torch.cuda.synchronize()
        assert pipe.last_layout() == "bucketed" and m == len(p)
        np.testing.assert_array_equal(pipe.edges()[0], p)
        np.testing.assert_array_equal(pipe.edges()[1], q)
        np.testing.assert_array_equal(pipe.edges()[2], w)


@pytest.mark.parametrize("tail", ["fast", "count"])
def test_residue_graph_replay(oracle_mod, tail):
    """The single-synchronisation residue step replayed from its HIP graph: every replay (stage
    timing off and on) is bit-exact, with either row-block tail (the fast tail's look-back words
    and cursors are reused across replays); an edge buffer that moves (overflow rerun) forces a new
    capture and stays exact."""
    import torch
    from uniprot_kmer_based_clustering_amd.device import DevicePipeline
    b = K.synth(20000, 21)
    p, q, w = oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=7, threads=8).pairs()
    pipe = DevicePipeline(b, 7, "cuda:0")
    pipe.set_tail(tail)
    for timing in (False, True):
        pipe.set_stage_timing(timing)
        for _ in range(4):
            assert pipe.step(engine="residues") == len(p)
            torch.cuda.synchronize()
            assert pipe.last_tail() == ("fast" if tail == "fast" else "rows")
            ep, eq, ew = pipe.edges()
            np.testing.assert_array_equal(ep, p)
            np.testing.assert_array_equal(eq, q)
            np.testing.assert_array_equal(ew, w)
    assert pipe.graph_replays() >= 2
    pipe._alloc_edges(1024)  # too small: EOVERFLOW, new buffers, new shape
    for _ in range(3):
        assert pipe.step(engine="residues") == len(p)
        np.testing.assert_array_equal(pipe.edges()[1], q)
    pipe.set_graph(False)
    r = pipe.graph_replays()
    assert pipe.step(engine="residues") == len(p) and pipe.graph_replays() == r
    np.testing.assert_array_equal(pipe.edges()[2], w)


@pytest.mark.parametrize("case", ["synthetic", "uniprot5", "uniprot7"])
def test_partitions_bit_exact(oracle_mod, uni, case):
    """The cursor partition (fixed-capacity regions, one atomic per run) and the counting
    partition group the same keys: bit-exact edges and statistics with either, repeated (graph
    replay); a batch whose frequent k-mers overflow a bucket region (the uniprot families) falls
    back to the counting partition and stays exact."""
    import torch
    from uniprot_kmer_based_clustering_amd.device import DevicePipeline
    if case == "synthetic":
        b, k = K.synth(30000, 23), 7
    else:
        b, k = K.Proteins(*uni), int(case[-1])
    o = oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=k, threads=8)
    p, q, w = o.pairs()
    seen = {}
    for mode in ("count", "auto"):
        pipe = DevicePipeline(b, k, "cuda:0")
        pipe.set_partition(mode)
        for _ in range(4):
            assert pipe.step(engine="residues") == len(p)
            torch.cuda.synchronize()
            assert pipe.last_layout() == "bucketed" and pipe.last_tail() in ("rows", "fast")
            np.testing.assert_array_equal(pipe.edges()[0], p)
            np.testing.assert_array_equal(pipe.edges()[1], q)
            np.testing.assert_array_equal(pipe.edges()[2], w)
        st = pipe.postings_stats.as_dict()
        assert st["distinct"] == o.counters()["distinct"] and st["max_df"] == o.counters()["max_df"]
        seen[mode] = pipe.last_partition()
    assert seen["count"] == "count"
    if case == "synthetic":  # hash-uniform buckets; the real families of uniprot may overflow one
        assert seen["auto"] == "cursor"


def test_rowtail_overflow_blocks(oracle_mod):
    """A protein whose row holds more pair keys than one row block of the LDS reduction (kPtCap):
    its block is listed and finished by the segmented sort, the rest stay on the LDS path; edges
    exact with the long row first (overflow) and last (every block short)."""
    import torch
    from uniprot_kmer_based_clustering_amd.device import DevicePipeline
    rng = np.random.default_rng(7)
    alpha = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", dtype=np.uint8)
    rnd = lambda m: alpha[rng.integers(0, 20, m)].tobytes()  # noqa: E731
    base = rnd(15000)
    seqs = [base] + [rnd(30) + base[60 * i:60 * i + 60] + rnd(30) for i in range(220)]
    res, off, cls = make_batch(seqs, ["a"] + ["b"] * 220)
    p, q, w = oracle_mod.Oracle(res, off, cls, k=7, threads=8).pairs()
    assert int(w[p == 0].sum()) > 8192
    for long_first in (True, False):
        if not long_first:  # the long row last instead of first: every row short enough
            seqs2 = seqs[1:] + seqs[:1]
            res, off, cls = make_batch(seqs2, ["b"] * 220 + ["a"])
            p, q, w = oracle_mod.Oracle(res, off, cls, k=7, threads=8).pairs()
        for tail in ("count", "fast"):
            pipe = DevicePipeline(K.Proteins(res, off, cls), 7, "cuda:0")
            pipe.set_tail(tail)
            for it in range(3):
                m = pipe.step(engine="residues")
                torch.cuda.synchronize()
                # counting tail: the long row's block is listed and sorted; fast tail: the long row
                # (one row above a fast block's 8,192 keys) passes its region, so the shape takes
                # the counting tail from the first call on; the long row last holds no pair
                fast = tail == "fast" and not long_first
                assert pipe.last_tail() == ("fast" if fast else "rows") and m == len(p)
                if it == 0:
                    assert (pipe.overflow_blocks() > 0) == long_first
                np.testing.assert_array_equal(pipe.edges()[0], p)
                np.testing.assert_array_equal(pipe.edges()[1], q)
                np.testing.assert_array_equal(pipe.edges()[2], w)
        for ms in (2, 30):  # min_shared inside the overflow encoder too
            keep = w >= ms
            assert pipe.step(min_shared=ms, engine="residues") == int(keep.sum())
            np.testing.assert_array_equal(pipe.edges()[1], q[keep])
            np.testing.assert_array_equal(pipe.edges()[2], w[keep])


@pytest.mark.parametrize("copies", [3000, 12000])
def test_frequent_kmers_heavy_path(oracle_mod, copies):
    """A k-mer shared by thousands of proteins (a group above the LDS sub-bucket limit; at 12000
    copies its bucket is above every LDS capacity and its level-2 bin above its tile budget):
    the bucketed layout spills it to the heavy path and the edges stay exact, for both entry
    points, with and without the class filter, and with min_shared."""
    import torch
    from uniprot_kmer_based_clustering_amd.device import DevicePipeline
    rng = np.random.default_rng(11)
    alpha = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", dtype=np.uint8)
    seqs = [alpha[rng.integers(0, 20, 120)].tobytes() + b"WWWWWWW" * (1 + i % 2) for i in range(copies)]
    res, off, cls = make_batch(seqs, [str(i % 7) for i in range(copies)])
    o = oracle_mod.Oracle(res, off, cls, k=7, threads=8)
    pipe = DevicePipeline(K.Proteins(res, off, cls), 7, "cuda:0")
    for eng in ("postings", "residues", "residues"):
        for diff in (True, False):
            m = pipe.step(require_class_diff=diff, engine=eng)
            torch.cuda.synchronize()
            assert pipe.last_layout() == "bucketed" and pipe.last_heavy()
            p, q, w = o.pairs(require_class_diff=diff)
            assert m == len(p)
            np.testing.assert_array_equal(pipe.edges()[0], p)
            np.testing.assert_array_equal(pipe.edges()[1], q)
            np.testing.assert_array_equal(pipe.edges()[2], w)
    st, c = pipe.postings_stats.as_dict(), o.counters()
    assert st["max_df"] == c["max_df"] >= copies and st["distinct"] == c["distinct"]
    assert st["sum_cdf2_light"] == c["sum_cdf2"] and st["repeat"] == c["repeat"]
    p, q, w = o.pairs(min_shared=2)
    assert pipe.step(min_shared=2, engine="residues") == len(p)
    np.testing.assert_array_equal(pipe.edges()[1], q)


def test_whole_bucket_segment(oracle_mod):
    """A bucket between the large bucket kernel's 4,096 keys and the LDS segment sort's 8,192 (one
    7-mer in 4,500 proteins, once each, plus the bucket's other keys): spilled whole and sorted by
    heavy_seg_kernel<1024, 2048, 8192> on its compacted key (k-mer slot | varying low bits), in
    class order (class filter on) and plain order (off); the edges equal the oracle's."""
    import torch
    from uniprot_kmer_based_clustering_amd.device import DevicePipeline
    rng = np.random.default_rng(17)
    alpha = np.frombuffer(b"ACDEFGHIKLMNPQRSTVY", dtype=np.uint8)  # no W before the W block
    n = 4500
    seqs = [alpha[rng.integers(0, 19, 110)].tobytes() + b"WWWWWWW" for i in range(n)]
    res, off, cls = make_batch(seqs, [str(i % 5) for i in range(n)])
    o = oracle_mod.Oracle(res, off, cls, k=7, threads=8)
    pipe = DevicePipeline(K.Proteins(res, off, cls), 7, "cuda:0")
    for eng in ("residues", "postings"):
        for diff in (True, False):
            m = pipe.step(require_class_diff=diff, engine=eng)
            torch.cuda.synchronize()
            assert pipe.last_layout() == "bucketed" and pipe.last_heavy()
            p, q, w = o.pairs(require_class_diff=diff)
            assert m == len(p)
            np.testing.assert_array_equal(pipe.edges()[0], p)
            np.testing.assert_array_equal(pipe.edges()[1], q)
            np.testing.assert_array_equal(pipe.edges()[2], w)
    assert pipe.postings_stats.as_dict()["max_df"] == o.counters()["max_df"] == n


@pytest.mark.parametrize("tail", ["fast", "count"])
def test_uniprot_k5_on_bucketed_heavy_path(oracle_mod, uni, tail):
    """The reference's dataset at k = 5 (max df 3,694): bucketed layout with the heavy path and
    the row-block tail — the fast tail (its 8,192-key regions overflow on the densest rows: fewer
    rows per block, or the counting tail when one row passes them) or the counting tail — edge list sha equal
    to the golden one (repeat:
    graph replay is not used on the split step, every call recomputes); min_shared 2 against the
    oracle."""
    import torch
    from uniprot_kmer_based_clustering_amd.device import DevicePipeline
    res, off, cls = uni
    g = load_json("uniprot_counters.json")["5"]
    pipe = DevicePipeline(K.Proteins(res, off, cls), 5, "cuda:0")
    pipe.set_tail(tail)
    p5, _, w5 = oracle_mod.Oracle(res, off, cls, k=5, threads=8).pairs()
    row_max = int(np.bincount(p5, weights=w5).max())  # a row's pair keys = the sum of its w
    for _ in range(2):
        m = pipe.step(engine="residues")
        torch.cuda.synchronize()
        assert pipe.last_layout() == "bucketed" and pipe.last_heavy()
        # the fast tail's regions overflow on the densest rows: it takes fewer rows per block, and
        # the counting tail when a single row holds more than a fast block's 8,192 keys
        if tail == "count" or row_max > 8192:
            assert pipe.last_tail() == "rows"
        assert m == g["n_edges"]
        assert edges_sha256(*pipe.edges()) == g["edges_sha256"]
        st = pipe.postings_stats.as_dict()
        assert st["max_df"] == g["max_df"] and st["sum_cdf2_light"] == g["sum_cdf2"]
        assert st["incidences"] == g["sum_w_diff"] and st["distinct"] == g["distinct"]
    p, q, w = oracle_mod.Oracle(res, off, cls, k=5, threads=8).pairs(min_shared=2)
    assert pipe.step(min_shared=2, engine="residues") == len(p)
    ep, eq, ew = pipe.edges()
    np.testing.assert_array_equal(ep, p)
    np.testing.assert_array_equal(eq, q)
    np.testing.assert_array_equal(ew, w)


@pytest.mark.parametrize("k", [5, 7])
def test_row_ranges_concatenate(oracle_mod, k):
    """kmp_dev_pairs_rows: the edges of consecutive row ranges (the unit of a rank / a pass)
    concatenate to the canonical list, on light (k = 7) and heavy (k = 5, frequent 5-mers)
    batches; statistics of every range describe the whole batch."""
    import torch
    from uniprot_kmer_based_clustering_amd.device import DevicePipeline
    b = K.synth(6000, 5, 1)
    o = oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=k, threads=8)
    p, q, w = o.pairs()
    pipe = DevicePipeline(b, k, "cuda:0")
    for parts in (1, 3, 8):
        start = K._lib.row_split(b.n, parts)
        got = [[], [], []]
        for d in range(parts):
            pipe.rows(int(start[d]), int(start[d + 1]))
            torch.cuda.synchronize()
            for a, x in zip(got, pipe.edges()):
                a.append(x)
            assert np.all((got[0][-1] >= start[d]) & (got[0][-1] < start[d + 1]))
        np.testing.assert_array_equal(np.concatenate(got[0]), p)
        np.testing.assert_array_equal(np.concatenate(got[1]), q)
        np.testing.assert_array_equal(np.concatenate(got[2]), w)
    assert pipe.rows(5, 5) == 0


def test_errors(engine):
    with pytest.raises(_lib.KmpError) as e:
        engine.build_sets(9)
    assert e.value.status == _lib.KMP_EINVAL
    fresh = K.KmerPairEngine(0, 1)
    with pytest.raises(_lib.KmpError) as e:
        fresh.pairs()
    assert e.value.status == _lib.KMP_ESTATE
    fresh.close()


def test_device_pipeline_matches_oracle(oracle_mod):
    import torch
    from uniprot_kmer_based_clustering_amd.device import DevicePipeline
    b = K.synth(20000, 9)
    o = oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=7, threads=8)
    pipe = DevicePipeline(b, 7, "cuda:0", edge_cap=1024)  # forces the overflow/rerun path
    n = pipe.step(engine="tiles")
    torch.cuda.synchronize()
    p, q, w = o.pairs()
    assert n == len(p)
    ep, eq, ew = pipe.edges()
    np.testing.assert_array_equal(ep, p)
    np.testing.assert_array_equal(eq, q)
    np.testing.assert_array_equal(ew, w)
    # a second step on the same buffers is identical (no stale state); the postings engine too
    assert pipe.step(engine="tiles") == n
    np.testing.assert_array_equal(pipe.edges()[2], w)
    c = o.counters()
    for eng in ("postings", "residues"):
        pipe._alloc_edges(1024)
        for _ in range(2):
            assert pipe.step(engine=eng) == n
            ep, eq, ew = pipe.edges()
            np.testing.assert_array_equal(ep, p)
            np.testing.assert_array_equal(eq, q)
            np.testing.assert_array_equal(ew, w)
        st = pipe.postings_stats.as_dict()
        assert st["distinct"] == c["distinct"] and st["repeat"] == c["repeat"] and st["max_df"] == c["max_df"]
        assert st["sum_cdf2_light"] == c["sum_cdf2"] and st["incidences"] == c["sum_w_diff"]
        assert st["sum_S"] == c["sum_S"] and st["pairs"] == n
    # both key layouts, both entry points: identical edges
    for bucketed in (True, False):
        pipe.set_layout(bucketed)
        for eng in ("postings", "residues"):
            assert pipe.step(engine=eng) == n
            np.testing.assert_array_equal(pipe.edges()[0], p)
            np.testing.assert_array_equal(pipe.edges()[1], q)
            np.testing.assert_array_equal(pipe.edges()[2], w)
            assert pipe.last_layout() == ("bucketed" if bucketed else "flat")
            assert pipe.last_tail() in (("rows", "fast") if bucketed else ("sort",))
        for ms in (2, 5):  # min_shared filter inside both tails
            keep = w >= ms
            assert pipe.step(min_shared=ms, engine="residues") == int(keep.sum())
            np.testing.assert_array_equal(pipe.edges()[1], q[keep])
    pipe.set_layout(True)
    # stage timing: six non-negative stage times that add up to about one step
    pipe.set_stage_timing(True)
    assert pipe.step(engine="residues") == n
    stages = pipe.postings_stats.stages()
    assert len(stages) == 6 and all(v >= 0 for v in stages.values()) and sum(stages.values()) > 0
    pipe.set_stage_timing(False)
    # sliced set build (multi-GPU shape): two halves == one launch
    pipe.set.zero_()
    pipe.build_sets(0, 7000)
    pipe.build_sets(7000, None)
    so, sv = o.sets()
    for pr in (0, 6999, 7000, 7001, 19999):
        np.testing.assert_array_equal(pipe.set_of(pr), sv[so[pr]:so[pr + 1]])


def _shared_kmer_batch(n, seed):
    """n random proteins (~300 aa) that all carry one 7-mer: every pair shares it (w >= 1), so row p
    holds ~n - p distinct partners of other classes — rows far past the fast tail's rank bound."""
    rng = np.random.default_rng(seed)
    alpha = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", dtype=np.uint8)
    seqs, classes = [], []
    for _ in range(n):
        s = alpha[rng.integers(0, 20, 300)].tobytes()
        at = int(rng.integers(0, 290))
        seqs.append(s[:at] + b"WCWCWCW" + s[at + 7:])
        classes.append(f"c{int(rng.integers(0, 15))}")
    return make_batch(seqs, classes)


@pytest.mark.parametrize("tail", ["fast", "count"])
def test_fast_tail_sort_fallback(oracle_mod, tail):
    """Rows with more distinct partners than the fast tail's per-row rank bound (kFtRankMax = 256):
    those row blocks sort their keys (block radix sort + run-length encoding) inside the fast
    reduce; edges equal the oracle's with either tail, min_shared 1 and 2, over graph replays."""
    import torch
    from uniprot_kmer_based_clustering_amd.device import DevicePipeline
    res, off, cls = _shared_kmer_batch(700, 31)
    o = oracle_mod.Oracle(res, off, cls, k=7, threads=8)
    p, q, w = o.pairs()
    assert np.bincount(p).max() > 256  # a row past the rank bound
    pipe = DevicePipeline(K.Proteins(res, off, cls), 7, "cuda:0")
    pipe.set_tail(tail)
    for ms in (1, 2, 1):
        keep = w >= ms
        for _ in range(3):
            assert pipe.step(min_shared=ms, engine="residues") == int(keep.sum())
            torch.cuda.synchronize()
            assert pipe.last_tail() == ("fast" if tail == "fast" else "rows")
            ep, eq, ew = pipe.edges()
            np.testing.assert_array_equal(ep, p[keep])
            np.testing.assert_array_equal(eq, q[keep])
            np.testing.assert_array_equal(ew, w[keep])


@pytest.mark.parametrize("ms", [2, 3, 7])
def test_fast_tail_min_shared_synthetic(oracle_mod, ms):
    """min_shared > 1 on the fast tail (pairs below it dropped before the rank, so the kept pairs stay
    canonical and contiguous), against the oracle and the counting tail on a 30k synthetic batch."""
    import torch
    from uniprot_kmer_based_clustering_amd.device import DevicePipeline
    b = K.synth(30000, 29)
    p, q, w = oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=7, threads=8).pairs()
    keep = w >= ms
    got = {}
    for tail in ("fast", "count"):
        pipe = DevicePipeline(b, 7, "cuda:0")
        pipe.set_tail(tail)
        for _ in range(2):
            assert pipe.step(min_shared=ms, engine="residues") == int(keep.sum())
        torch.cuda.synchronize()
        got[tail] = pipe.edges()
        assert pipe.last_tail() == ("fast" if tail == "fast" else "rows")
    for t in got.values():
        np.testing.assert_array_equal(t[0], p[keep])
        np.testing.assert_array_equal(t[1], q[keep])
        np.testing.assert_array_equal(t[2], w[keep])
