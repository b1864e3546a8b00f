"""GPU parity of the repeat index: the device MPHF (boomphf surface,
main.rs:139-140), five_mer_hash_freq (main.rs:187-193) and hash_five_mers (protein.rs:151-174),
against the oracle.  MPHF ids are this build's, not boomphf's (parity unpinned for the id values,
SURVEY.md §8c): the tests check the properties boomphf guarantees (a bijection onto 0..n-1) and
everything observable through the ids (code_by_id, df_by_id, per-protein order)."""
import numpy as np
import pytest

from common import make_batch, tiny, uniprot
import uniprot_kmer_based_clustering_amd as K
from uniprot_kmer_based_clustering_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = K.KmerPairEngine(0, 4)
    yield e
    e.close()


@pytest.mark.parametrize("n", [0, 1, 2, 1000, 123_457, 2_000_000])
@pytest.mark.parametrize("gamma", [1.0, 3.0])
def test_mphf_is_a_bijection(engine, n, gamma):
    rng = np.random.default_rng(n + int(gamma))
    keys = rng.choice(np.uint64(21 ** 7), size=n, replace=False).astype(np.uint32) if n else np.zeros(0, np.uint32)
    m = engine.mphf(keys, gamma)
    ids = m.hash(keys)
    np.testing.assert_array_equal(np.sort(ids), np.arange(n, dtype=np.uint64))
    info = m.info()
    assert info["n"] == n
    if n > 1000:
        # BBHash: a level of gamma*m bits places a fraction exp(-1/gamma) of its m keys, so the
        # levels total gamma * exp(1/gamma) * n bits (2.72 n at gamma 1, 4.19 n at gamma 3)
        assert info["bits"] <= 1.1 * gamma * np.exp(1 / gamma) * n + 64 * info["levels"]
        assert info["fallback"] == 0
    m.close()


def test_mphf_dev_lookup_matches_host(engine):
    import torch
    rng = np.random.default_rng(7)
    keys = rng.choice(np.uint64(21 ** 5), size=50_000, replace=False).astype(np.uint32)
    m = engine.mphf(keys)
    host = m.hash(keys)
    dev = m.dev_hash(torch.from_numpy(keys.astype(np.int32)).cuda())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dev.cpu().numpy().astype(np.uint64), host)


def test_mphf_rejects_duplicates_and_bad_gamma(engine):
    with pytest.raises(_lib.KmpError) as ei:
        engine.mphf(np.array([5, 9, 5], np.uint32))
    assert ei.value.status == _lib.KMP_EINVAL
    with pytest.raises(_lib.KmpError) as ei:
        engine.mphf(np.array([1, 2], np.uint32), 0.5)
    assert ei.value.status == _lib.KMP_EINVAL


def check_repeat_index(engine, o, n):
    codes = engine.get_repeat_codes()
    df = engine.get_df()
    rep, rep_df = o.repeat()
    R = len(rep)
    assert len(codes) == R and len(df) == R
    assert engine.counters()["repeat"] == R
    # code_by_id is a permutation of the repeat k-mers, df_by_id their df
    order = np.argsort(codes, kind="stable")
    np.testing.assert_array_equal(codes[order], rep)
    np.testing.assert_array_equal(df[order], rep_df)
    # the context's MPHF maps each repeat code to its id
    m = engine.repeat_mphf()
    ids = m.hash(rep)
    np.testing.assert_array_equal(codes[ids.astype(np.int64)], rep)
    # hash_five_mers of every protein: ids in first-occurrence order
    hk, hk_off = engine.get_hash_kmers_all()
    want, want_off = o.hash_order()
    np.testing.assert_array_equal(hk_off, want_off)
    np.testing.assert_array_equal(codes[hk.astype(np.int64)], want)
    for p in (0, n // 2, n - 1):
        np.testing.assert_array_equal(engine.get_hash_kmers(p), hk[hk_off[p]:hk_off[p + 1]])
    # five_mer_hash_freq = number of proteins whose hash_five_mers hold the id
    freq = np.bincount(hk.astype(np.int64), minlength=R)
    np.testing.assert_array_equal(freq, df)


@pytest.mark.parametrize("k", [5, 7])
def test_repeat_index_tiny_and_uniprot(engine, oracle_mod, k):
    for res, off, cls, _ in (tiny(), uniprot()):
        o = oracle_mod.Oracle(res, off, cls, k=k, threads=8)
        engine.load(K.Proteins(res, off, cls))
        engine.build_sets(k)
        check_repeat_index(engine, o, len(off) - 1)


@pytest.mark.parametrize("n,seed,law", [(3000, 11, 0), (800, 12, 1)])
def test_repeat_index_synthetic(engine, oracle_mod, n, seed, law):
    b = K.synth(n, seed, law)
    res, off, cls = b.residues, b.offsets, b.class_id
    o = oracle_mod.Oracle(res, off, cls, k=5, threads=8)
    engine.load(K.Proteins(res, off, cls))
    engine.build_sets(5)
    check_repeat_index(engine, o, n)
    # rebuilding the sets at another k invalidates and rebuilds the index
    o7 = oracle_mod.Oracle(res, off, cls, k=7, threads=8)
    engine.build_sets(7)
    check_repeat_index(engine, o7, n)


def test_repeat_index_edge_cases(engine, oracle_mod):
    # empty and shorter-than-k proteins, a protein with only unique k-mers, repeats inside one protein
    seqs = [b"", b"MKV", b"ACDEFGHIKL", b"ACDEFGHIKLACDEF", b"WWWWWWWWWW", b"QQQQQQ", b"ACDEFXXXXACDEF"]
    res, off, cls = make_batch(seqs, [str(i) for i in range(len(seqs))])
    o = oracle_mod.Oracle(res, off, cls, k=5, threads=1)
    engine.load(K.Proteins(res, off, cls))
    engine.build_sets(5)
    check_repeat_index(engine, o, len(seqs))
    # a single protein has no repeat k-mers at all
    res1, off1, cls1 = make_batch([b"ACDEFGHIKL"], ["a"])
    engine.load(K.Proteins(res1, off1, cls1))
    engine.build_sets(5)
    assert len(engine.get_df()) == 0
    ids, offs = engine.get_hash_kmers_all()
    assert len(ids) == 0 and offs.tolist() == [0, 0]


def test_repeat_index_requires_sets(engine):
    res, off, cls, _ = tiny()
    engine.load(K.Proteins(res, off, cls))
    with pytest.raises(_lib.KmpError) as ei:
        engine.get_df()
    assert ei.value.status == _lib.KMP_ESTATE
