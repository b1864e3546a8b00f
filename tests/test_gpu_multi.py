"""GPU parity of the multi-GPU row split behind the C ABI (kmp_ctx_create_multi): G virtual ranks
on one GPU (each rank its own stream, workspace and copy of the batch, one host thread per
rank; the gather over device copies — RCCL admits one rank per device), against the oracle,
bit-exact, on config-3 / config-4's workload (100k proteins, seed 3, k = 7) and on the heavy
k = 5 dataset; the RCCL transport itself over the one real device (G = 1 communicator)."""
import numpy as np
import pytest

from common import edges_sha256, load_json, uniprot
import uniprot_kmer_based_clustering_amd as K
from uniprot_kmer_based_clustering_amd import _lib

pytestmark = pytest.mark.gpu


def assert_edges(e, p, q, w):
    np.testing.assert_array_equal(e.p, p)
    np.testing.assert_array_equal(e.q, q)
    np.testing.assert_array_equal(e.w, w)


@pytest.fixture(scope="module")
def config4(oracle_mod):
    b = K.synth(100000, 3)
    p, q, w = oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=7, threads=16).pairs()
    return b, (p, q, w)


@pytest.mark.parametrize("g", [2, 4, 8])
def test_virtual_ranks_config4(config4, g):
    """Config 4's workload split over G in {2, 4, 8} ranks: the gathered list equals the
    oracle's canonical list (and so the single-GPU one): invariant to the number of ranks."""
    b, (p, q, w) = config4
    with K.KmerPairEngine(0, 4, devices=[0] * g) as e:
        assert e.gpus == g and e.transport == "copy"
        e.load(b)
        e.build_sets(7)
        for _ in range(2):  # second call: learned capacities, same result
            got = e.pairs()
            assert len(got) == len(p) > 1_000_000
            assert_edges(got, p, q, w)
            assert e.last_split == "kmer"
        c = e.counters()
        assert c["n_edges"] == len(p)


def test_virtual_ranks_heavy_uniprot_k5():
    """The reference's dataset at k = 5 (frequent 5-mers, max df 3,694) over 3 ranks on the k-mer
    split: every rank compacts, plans and expands the spill of its own k-mers with the heavy path
    and routes those pair keys with the light ones (vertex.rs:59-140); golden edge sha, twice (the
    second call keeps the heavy path on without a rerun)."""
    res, off, cls, _ = uniprot()
    g = load_json("uniprot_counters.json")["5"]
    with K.KmerPairEngine(0, 4, devices=[0, 0, 0]) as e:
        e.load(K.Proteins(res, off, cls))
        e.build_sets(5)
        for _ in range(2):
            got = e.pairs()
            assert len(got) == g["n_edges"] and e.last_split == "kmer"
            assert edges_sha256(got.p, got.q, got.w) == g["edges_sha256"]
            c = e.counters()
            assert c["sum_w_diff"] == g["sum_w_diff"] and c["n_align"] == g["n_align"]


def test_virtual_ranks_options_and_scores(oracle_mod):
    """min_shared, the class filter off, and BLOSUM scores (computed on rank 0 over the
    gathered list) through the split; more ranks than proteins leaves ranks empty."""
    b = K.synth(3000, 5, 1)
    o = oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=5, threads=8)
    with K.KmerPairEngine(0, 2, devices=[0, 0, 0, 0]) as e:
        e.load(b)
        e.build_sets(5)
        for ms, diff in ((1, True), (3, False)):
            assert_edges(e.pairs(min_shared=ms, require_class_diff=diff),
                         *o.pairs(min_shared=ms, require_class_diff=diff))
        p, q, w = o.pairs()
        got = e.pairs(score=_lib.KMP_SCORE_BLOSUM)
        assert_edges(got, p, q, w)
        np.testing.assert_array_equal(got.score, o.blosum_scores(p, q).astype(np.float32))
    seqs = K.synth(5, 1)
    with K.KmerPairEngine(0, 1, devices=[0] * 8) as e:
        e.load(seqs)
        e.build_sets(5)
        o = oracle_mod.Oracle(seqs.residues, seqs.offsets, seqs.class_id, k=5)
        assert_edges(e.pairs(require_class_diff=False), *o.pairs(require_class_diff=False))


def test_rccl_transport_single_device(oracle_mod):
    """A one-device multi context (G = 1: no gather) and the RCCL transport: distinct devices
    make library-owned RCCL communicators (ncclCommInitAll); with one GPU only G = 1 runs."""
    b = K.synth(2000, 7)
    p, q, w = oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=7).pairs()
    with K.KmerPairEngine(0, 1, devices=[0]) as e:
        assert e.gpus == 1 and e.transport == "local"
        e.load(b)
        e.build_sets(7)
        assert_edges(e.pairs(), p, q, w)
    import torch
    if torch.cuda.device_count() >= 2:
        with K.KmerPairEngine(0, 1, devices=[0, 1]) as e:
            assert e.transport == "rccl"
            e.load(b)
            e.build_sets(7)
            assert_edges(e.pairs(), p, q, w)


def emulate_kmer_split(b, k, G, cap=None, min_shared=1, require_class_diff=True):
    """The k-mer split's G ranks on one GPU, in one process: every rank's kmp_dev_split_expand on
    its own DevicePipeline, the all-to-all done by slicing the send regions, every rank's
    kmp_dev_split_edges; flags reduced (max) over the ranks and fed back as `learn` on a rerun,
    as dist.kmer_split_step does over RCCL.  Returns the concatenated edges, the flags, the
    summed statistics and the number of reruns."""
    import torch
    from uniprot_kmer_based_clustering_amd.device import DevicePipeline
    pipes = [DevicePipeline(b, k, "cuda:0") for _ in range(G)]
    start = _lib.row_split(b.n, G)
    cap = cap or max(4096, pipes[0].total // 4 // (G * G))
    learn, reruns = None, 0
    for _ in range(6):
        sends = [torch.empty(G * cap, dtype=torch.int64, device="cuda:0") for _ in range(G)]
        flags = [torch.zeros(_lib.KMP_SPLIT_FLAGS, dtype=torch.int32, device="cuda:0") for _ in range(G)]
        stats = [torch.zeros(8, dtype=torch.int64, device="cuda:0") for _ in range(G)]
        for r in range(G):
            pipes[r].split_expand(r, G, cap, sends[r], flags[r], stats[r], learn=learn,
                                  require_class_diff=require_class_diff)
        fl = torch.stack(flags).max(dim=0).values.cpu().tolist()
        out = [[], [], []]
        for d in range(G):
            recv = torch.cat([sends[r][d * cap:(d + 1) * cap] for r in range(G)])
            pipes[d].split_edges(recv, int(start[d]), int(start[d + 1]), min_shared)
            for a, x in zip(out, pipes[d].edges()):
                a.append(x)
        if (fl[_lib.KMP_SPLIT_RERUN] or fl[_lib.KMP_SPLIT_HEAVY]) and not fl[_lib.KMP_SPLIT_CLASS]:
            reruns += 1
            learn = fl
            cap = max(cap, fl[_lib.KMP_SPLIT_MAX_PART] + fl[_lib.KMP_SPLIT_MAX_PART] // 16 + 1024)
            continue
        st = torch.stack(stats).cpu().numpy()
        tot = st.sum(axis=0)
        tot[4] = st[:, 4].max()
        return [np.concatenate(a) for a in out], fl, tot, reruns
    raise AssertionError("capacities unstable")


@pytest.mark.parametrize("g", [1, 2, 4, 8])
def test_kmer_split_config4(config4, oracle_mod, g):
    """Config 4's workload (100k proteins, k = 7) through the k-mer split's device stages at
    G ranks: the rank-order concatenation of the ranks' edges equals the oracle's canonical list,
    and the ranks' statistics add up to the whole batch's (Σ C(df,2), distinct, incidences)."""
    b, (p, q, w) = config4
    (ep, eq, ew), fl, tot, _ = emulate_kmer_split(b, 7, g)
    assert not fl[_lib.KMP_SPLIT_HEAVY] and not fl[_lib.KMP_SPLIT_CLASS]
    np.testing.assert_array_equal(ep, p)
    np.testing.assert_array_equal(eq, q)
    np.testing.assert_array_equal(ew, w)
    c = oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=7, threads=16).counters()
    assert tot[3] == c["sum_cdf2"] and tot[1] == c["distinct"] and tot[4] == c["max_df"]
    assert tot[6] == int(w.sum())  # incidences after the class filter = Σ w of the canonical list


def test_kmer_split_reruns_and_options(oracle_mod):
    """An exchange capacity far too small reruns with the capacity learned from the reduced
    flags (same edges); min_shared on the receiving side; the reference's dataset at k = 5
    (frequent 5-mers spill) raises HEAVY once, and the rerun with every rank's heavy path on gives
    the golden edge list at G = 2 and 3."""
    b = K.synth(20000, 9)
    o = oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=7, threads=8)
    for ms in (1, 2):
        (ep, eq, ew), fl, _, reruns = emulate_kmer_split(b, 7, 3, cap=64, min_shared=ms)
        p, q, w = o.pairs(min_shared=ms)
        assert reruns == 1
        np.testing.assert_array_equal(ep, p)
        np.testing.assert_array_equal(eq, q)
        np.testing.assert_array_equal(ew, w)
    res, off, cls, _ = uniprot()
    g = load_json("uniprot_counters.json")["5"]
    for G in (2, 3):
        (ep, eq, ew), fl, tot, reruns = emulate_kmer_split(K.Proteins(res, off, cls), 5, G)
        assert reruns >= 1 and not fl[_lib.KMP_SPLIT_HEAVY] and not fl[_lib.KMP_SPLIT_RERUN]
        assert len(ep) == g["n_edges"] and edges_sha256(ep, eq, ew) == g["edges_sha256"]


def dense_families(n_fam=40, members=60, length=300, mu=0.02, seed=11):
    """Families of near-identical proteins (per-site substitution rate mu), shuffled, 15 classes
    at random: most k-mers occur in ~`members` proteins, so bucket groups hold 32+ keys (below the
    heavy path's 128) and a bucket expands to thousands of pair keys."""
    rng = np.random.default_rng(seed)
    aa = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", dtype=np.uint8)
    seqs = []
    for _ in range(n_fam):
        anc = rng.choice(aa, length)
        for _ in range(members):
            s = anc.copy()
            mut = rng.random(length) < mu
            s[mut] = rng.choice(aa, int(mut.sum()))
            seqs.append(s)
    order = rng.permutation(len(seqs))
    res = np.concatenate([seqs[i] for i in order]).astype(np.uint8)
    off = np.arange(len(seqs) + 1, dtype=np.uint64) * length
    cls = rng.integers(0, 15, len(seqs)).astype(np.uint16)
    return K.Proteins(res, off, cls)


@pytest.mark.parametrize("g", [2, 3])
def test_kmer_split_routed_large_groups(oracle_mod, g):
    """The routed bucket output of the k-mer split on buckets above the LDS staging (groups of
    ~60 keys: a bucket expands to more pair keys than its stage holds, so it counts, reserves per
    destination and writes with LDS cursors), class filter on and off: bit-exact at G ranks."""
    b = dense_families()
    o = oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=7, threads=8)
    for diff in (True, False):
        (ep, eq, ew), fl, tot, _ = emulate_kmer_split(b, 7, g, require_class_diff=diff)
        assert not fl[_lib.KMP_SPLIT_HEAVY] and not fl[_lib.KMP_SPLIT_CLASS]
        c = o.counters()
        assert c["max_df"] >= 32
        p, q, w = o.pairs(require_class_diff=diff)
        assert len(p) > 10_000
        np.testing.assert_array_equal(ep, p)
        np.testing.assert_array_equal(eq, q)
        np.testing.assert_array_equal(ew, w)


def emulate_sharded_split(b, k, G, kcap=None, cap=None, min_shared=1, require_class_diff=True):
    """The k-mer split with a sharded start, G ranks on one GPU in one process: each rank's
    ShardPipeline holds only its residue slice; kmp_dev_split_keys per rank, the key all-to-all done
    by slicing the key regions, kmp_dev_split_group per rank, the pair-key all-to-all likewise,
    kmp_dev_split_edges per rank; flags max-reduced and fed back as `learn`, as
    dist.sharded_split_step does over RCCL.  Returns (edges, flags, summed stats, reruns)."""
    import torch
    from uniprot_kmer_based_clustering_amd.device import ShardPipeline
    pipes = [ShardPipeline(b.residues, b.offsets, b.class_id, k, r, G, "cuda:0") for r in range(G)]
    for r, pp in enumerate(pipes):  # the slice is the rank's share of the residues, not the batch
        assert pp.res.numel() <= int(b.offsets[-1]) // G + 4096 or G == 1
    start = _lib.row_split(b.n, G)
    kcap = kcap or int(pipes[0].span.key_cap)
    cap = cap or max(4096, pipes[0].total // 4 // (G * G))
    learn, reruns = None, 0
    for _ in range(8):
        ksend = [torch.empty(G * kcap, dtype=torch.int64, device="cuda:0") for _ in range(G)]
        sends = [torch.empty(G * cap, dtype=torch.int64, device="cuda:0") for _ in range(G)]
        flags = [torch.zeros(_lib.KMP_SPLIT_FLAGS, dtype=torch.int32, device="cuda:0") for _ in range(G)]
        stats = [torch.zeros(8, dtype=torch.int64, device="cuda:0") for _ in range(G)]
        for r in range(G):
            pipes[r].split_keys(r, G, kcap, ksend[r], flags[r])
        for d in range(G):
            krecv = torch.cat([ksend[r][d * kcap:(d + 1) * kcap] for r in range(G)])
            pipes[d].split_group(krecv, kcap, d, G, cap, sends[d], flags[d], stats[d], learn=learn,
                                 require_class_diff=require_class_diff)
        torch.cuda.synchronize()
        fl = torch.stack(flags).max(dim=0).values.cpu().tolist()
        out = [[], [], []]
        for d in range(G):
            recv = torch.cat([sends[r][d * cap:(d + 1) * cap] for r in range(G)])
            pipes[d].split_edges(recv, int(start[d]), int(start[d + 1]), min_shared)
            for a, x in zip(out, pipes[d].edges()):
                a.append(x)
        if (fl[_lib.KMP_SPLIT_RERUN] or fl[_lib.KMP_SPLIT_HEAVY]) and not fl[_lib.KMP_SPLIT_CLASS]:
            reruns += 1
            learn = fl
            cap = max(cap, fl[_lib.KMP_SPLIT_MAX_PART] + fl[_lib.KMP_SPLIT_MAX_PART] // 16 + 1024)
            kcap = max(kcap, fl[_lib.KMP_SPLIT_MAX_KEYS] + fl[_lib.KMP_SPLIT_MAX_KEYS] // 32 + 1024)
            continue
        st = torch.stack(stats).cpu().numpy()
        tot = st.sum(axis=0)
        tot[4] = st[:, 4].max()
        return [np.concatenate(a) for a in out], fl, tot, reruns
    raise AssertionError("capacities unstable")


@pytest.mark.parametrize("g", [1, 2, 4, 8])
def test_sharded_split_config4(config4, oracle_mod, g):
    """Config 4's workload through the k-mer split with a sharded start (each rank holds 1/G of the
    residues, keys its own windows once, the keys travel to their bins' owners): the rank-order
    concatenation equals the oracle's canonical list and the ranks' statistics add up to the batch's;
    no rerun with the default capacities."""
    b, (p, q, w) = config4
    (ep, eq, ew), fl, tot, reruns = emulate_sharded_split(b, 7, g)
    assert not fl[_lib.KMP_SPLIT_HEAVY] and not fl[_lib.KMP_SPLIT_CLASS] and reruns == 0
    np.testing.assert_array_equal(ep, p)
    np.testing.assert_array_equal(eq, q)
    np.testing.assert_array_equal(ew, w)
    c = oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=7, threads=16).counters()
    assert tot[3] == c["sum_cdf2"] and tot[1] == c["distinct"] and tot[4] == c["max_df"]
    assert tot[0] == c["sum_S"] and tot[6] == int(w.sum())


def test_sharded_split_reruns_heavy_and_options(oracle_mod):
    """Key regions and pair-key regions far too small rerun with the sizes the reduced flags report
    (same edges, capacities learned from counts: the same reruns every time); min_shared and the
    class filter off; the reference's dataset at k = 5 (frequent 5-mers: HEAVY, then every rank's
    heavy path) gives the golden edge list at G = 2 and 3; routed buckets above the LDS stage."""
    b = K.synth(20000, 9)
    o = oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=7, threads=8)
    seen = set()
    for ms in (1, 2, 1):
        (ep, eq, ew), fl, _, reruns = emulate_sharded_split(b, 7, 3, kcap=4096, cap=64, min_shared=ms)
        p, q, w = o.pairs(min_shared=ms)
        seen.add(reruns)
        np.testing.assert_array_equal(ep, p)
        np.testing.assert_array_equal(eq, q)
        np.testing.assert_array_equal(ew, w)
    assert len(seen) == 1 and seen.pop() >= 1
    (ep, eq, ew), _, _, _ = emulate_sharded_split(b, 7, 4, require_class_diff=False)
    p, q, w = o.pairs(require_class_diff=False)
    np.testing.assert_array_equal(ep, p)
    np.testing.assert_array_equal(ew, w)
    res, off, cls, _ = uniprot()
    g = load_json("uniprot_counters.json")["5"]
    for G in (2, 3):
        (ep, eq, ew), fl, tot, reruns = emulate_sharded_split(K.Proteins(res, off, cls), 5, G)
        assert reruns >= 1 and not fl[_lib.KMP_SPLIT_HEAVY] and not fl[_lib.KMP_SPLIT_RERUN]
        assert len(ep) == g["n_edges"] and edges_sha256(ep, eq, ew) == g["edges_sha256"]
    d = dense_families()
    (ep, eq, ew), fl, _, _ = emulate_sharded_split(d, 7, 2)
    p, q, w = oracle_mod.Oracle(d.residues, d.offsets, d.class_id, k=7, threads=8).pairs()
    np.testing.assert_array_equal(ep, p)
    np.testing.assert_array_equal(eq, q)
    np.testing.assert_array_equal(ew, w)


def test_sharded_split_small_batches(oracle_mod):
    """More ranks than chunks or bins (ranks with nothing to key or no bins), a protein shorter than
    k, and one class: every rank still steps in lockstep and the result is the oracle's."""
    for n, G in ((5, 8), (300, 8), (3000, 5)):
        b = K.synth(n, 4)
        o = oracle_mod.Oracle(b.residues, b.offsets, b.class_id, k=5, threads=4)
        (ep, eq, ew), fl, _, _ = emulate_sharded_split(b, 5, G, require_class_diff=False)
        p, q, w = o.pairs(require_class_diff=False)
        np.testing.assert_array_equal(ep, p)
        np.testing.assert_array_equal(eq, q)
        np.testing.assert_array_equal(ew, w)


def test_capacity_learning_is_order_independent(config4):
    """Every learned capacity (bucket and fast-tail regions, pair-key shards, send and key regions,
    spill regions) is sized from counts, not from fill levels reached in whatever order the device's
    atomics ran: the same inputs rerun the same number of times and replay the same number of graph
    steps, run after run — config 3 on one GPU and the reference's dataset at k = 5 (frequent 5-mers:
    the heavy path, learned bucket and fast-tail regions) on one GPU and on the sharded k-mer split."""
    import torch
    from uniprot_kmer_based_clustering_amd.device import DevicePipeline
    b, _ = config4
    res, off, cls, _ = uniprot()
    u = K.Proteins(res, off, cls)
    for batch, k in ((b, 7), (u, 5)):
        seen = []
        for trial in range(3):
            pipe = DevicePipeline(batch, k, "cuda:0")
            ms = [pipe.step() for _ in range(5)]
            torch.cuda.synchronize()
            seen.append((pipe.reruns(), pipe.graph_replays(), tuple(ms)))
            del pipe
        assert seen[0] == seen[1] == seen[2], seen
    runs = [emulate_sharded_split(u, 5, 2)[3] for _ in range(3)]
    assert runs[0] == runs[1] == runs[2] >= 1, runs
