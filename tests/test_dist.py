"""The multi-GPU flows (uniprot_kmer_based_clustering_amd/dist.py) on CPU: world_size 2 and 3
over gloo — the row split and the k-mer split (kmer_split_step: all-to-all of the routed pair
keys, flags reduced over the ranks, capacity reruns, row-split fallback).  Each rank's device stage (kmp_dev_pairs_rows, GPU-only) is stood in for by the
oracle's edge list restricted to the rank's rows; the test checks that the ranks' blocks,
gathered in place to rank 0, concatenate to exactly the single-process canonical list (the
result is invariant to the number of ranks), including empty blocks and a rank-0 destination
that has to grow.  The device stage itself: tests/test_gpu_parity.py::test_row_ranges_concatenate
and tests/test_gpu_multi.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from common import ROOT


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def build_case():
    import uniprot_kmer_based_clustering_amd as K
    from oracle.oracle import Oracle
    b = K.synth(3000, 21)
    o = Oracle(b.residues, b.offsets, b.class_id, k=7, threads=2)
    return b, o


class OraclePipe:
    """CPU stand-in for DevicePipeline.rows: the oracle's edges of rows [lo, hi) into ep/eq/ew."""

    def __init__(self, n, p, q, w, cap):
        self.n, self.P, self.Q, self.W = n, p, q, w
        self._alloc_edges(cap)

    def _alloc_edges(self, cap):
        self.edge_cap = cap
        self.ep = torch.zeros(cap, dtype=torch.int32)
        self.eq = torch.zeros(cap, dtype=torch.int32)
        self.ew = torch.zeros(cap, dtype=torch.int32)

    def rows(self, lo, hi, min_shared=1, require_class_diff=True):
        keep = (self.P >= lo) & (self.P < hi) & (self.W >= min_shared)
        m = int(keep.sum())
        if m > self.edge_cap:
            self._alloc_edges(m)
        for dst, src in zip((self.ep, self.eq, self.ew), (self.P, self.Q, self.W)):
            dst[:m] = torch.from_numpy(src[keep].view(np.int32).copy())
        return m


def worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, ROOT)
        from uniprot_kmer_based_clustering_amd.dist import distributed_step, row_ranges
        b, o = build_case()
        P, Q, W = o.pairs()
        # rank 0 starts with a destination smaller than the gathered list: it has to grow
        pipe = OraclePipe(b.n, P, Q, W, cap=16 if rank == 0 else 1 << 20)
        ranges = row_ranges(b.n, world)
        for ms in (1, 3, 10 ** 6):  # the last one: every block empty
            n = distributed_step(pipe, rank, world, min_shared=ms)
            if rank == 0:
                keep = W >= ms
                ok = (n == int(keep.sum())
                      and np.array_equal(pipe.ep[:n].numpy().view(np.uint32), P[keep])
                      and np.array_equal(pipe.eq[:n].numpy().view(np.uint32), Q[keep])
                      and np.array_equal(pipe.ew[:n].numpy().view(np.uint32), W[keep]))
                out_q.put(("edges", ms, ok, n))
        out_q.put(("ranges", rank, ranges))
    finally:
        dist.destroy_process_group()


def bits_for(v):
    b = 0
    while b < 64 and (v - 1) >> b:
        b += 1
    return max(b, 1)


class OracleSplitPipe(OraclePipe):
    """CPU stand-in for the k-mer split stages.  split_expand: rank `part` owns a share of every
    pair's w (w // parts, plus one for the first w % parts ranks: the shares of the k-mers of its
    hash range), emits one pair key p << bits(N) | q per incidence and routes it to the row owner,
    padded regions of cap keys (-1 = kNoKey), flags as the library's; split_edges: run-length
    counts of the received keys of its rows, canonical order."""

    def __init__(self, n, p, q, w, cap, heavy=False):
        super().__init__(n, p, q, w, cap)
        self.total = 300 * n
        self.dev = torch.device("cpu")
        self.heavy = heavy
        self.heavy_on = False
        self.pbits = bits_for(n)

    def split_expand(self, part, parts, cap, send, flags, stats, learn=None, require_class_diff=True):
        from uniprot_kmer_based_clustering_amd import _lib
        from uniprot_kmer_based_clustering_amd.dist import row_ranges
        share = self.W // parts + (part < self.W % parts)
        keys = np.repeat((self.P.astype(np.int64) << self.pbits) | self.Q.astype(np.int64), share)
        send.fill_(-1)
        most = 0
        for d, (lo, hi) in enumerate(row_ranges(self.n, parts)):
            kd = keys[((keys >> self.pbits) >= lo) & ((keys >> self.pbits) < hi)][::-1]  # any order
            most = max(most, len(kd))
            send[d * cap:d * cap + min(cap, len(kd))] = torch.from_numpy(kd[:cap].copy())
        flags.zero_()
        flags[_lib.KMP_SPLIT_MAX_PART] = most
        flags[_lib.KMP_SPLIT_RERUN] = int(most > cap)
        # a spilling batch raises HEAVY until the learned flags turn the heavy path on (the library
        # keeps it on for the batch from then on)
        if learn is not None and learn[_lib.KMP_SPLIT_HEAVY]:
            self.heavy_on = True
        flags[_lib.KMP_SPLIT_HEAVY] = int(self.heavy and not self.heavy_on)
        stats.zero_()
        stats[6] = int(share.sum())

    def split_edges(self, recv, lo, hi, min_shared=1):
        x = recv.numpy()
        x = x[x != -1]
        assert np.all(((x >> self.pbits) >= lo) & ((x >> self.pbits) < hi))
        u, c = np.unique(x, return_counts=True)
        keep = c >= min_shared
        u, c = u[keep], c[keep]
        m = len(u)
        if m > self.edge_cap:
            self._alloc_edges(m)
        self.ep[:m] = torch.from_numpy((u >> self.pbits).astype(np.int32))
        self.eq[:m] = torch.from_numpy((u & ((1 << self.pbits) - 1)).astype(np.int32))
        self.ew[:m] = torch.from_numpy(c.astype(np.int32))
        self.n_edges = m
        return m


def split_worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, ROOT)
        from uniprot_kmer_based_clustering_amd.dist import SplitState, kmer_split_step
        b, o = build_case()
        P, Q, W = o.pairs()
        for heavy in (False, True):
            pipe = OracleSplitPipe(b.n, P, Q, W, cap=16 if rank == 0 else 1 << 20, heavy=heavy)
            state = SplitState()
            state.cap = 64  # far too small: the first step reruns with the learned capacity
            for ms in (1, 3):
                n = kmer_split_step(pipe, rank, world, min_shared=ms, gather=True, state=state)
                if rank == 0:
                    keep = W >= ms
                    ok = (n == int(keep.sum())
                          and np.array_equal(pipe.ep[:n].numpy().view(np.uint32), P[keep])
                          and np.array_equal(pipe.eq[:n].numpy().view(np.uint32), Q[keep])
                          and np.array_equal(pipe.ew[:n].numpy().view(np.uint32), W[keep]))
                    out_q.put(("split", heavy, ms, ok, n, state.reruns, state.row_split, state.cap))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_kmer_split_exchange(world):
    """kmer_split_step over gloo: the all-to-all of routed pair keys and the per-rank reduction
    give the canonical list gathered on rank 0; an undersized exchange capacity reruns once with
    the capacity learned from the reduced flags; a spilling batch reruns once with the heavy path
    on and stays on the k-mer split."""
    port = free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=split_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    msgs = [q.get(timeout=300) for _ in range(4)]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert all(m[3] for m in msgs), msgs
    light = [m for m in msgs if not m[1]]
    assert light[0][5] == 1 and not light[0][6] and light[0][7] > 64  # one rerun, then the learned cap
    heavy = [m for m in msgs if m[1]]
    assert not any(m[6] for m in heavy)  # spilling: stays on the k-mer split, the heavy path on
    assert heavy[0][5] >= 1  # (after a rerun that turned it on)


@pytest.mark.parametrize("world", [2, 3])
def test_row_split_gather(world):
    port = free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    msgs = [q.get(timeout=300) for _ in range(3 + world)]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    edges = [m for m in msgs if m[0] == "edges"]
    assert len(edges) == 3 and all(m[2] for m in edges), edges
    assert edges[0][3] > 1000 and edges[2][3] == 0
    ranges = [m[2] for m in msgs if m[0] == "ranges"]
    assert all(r == ranges[0] for r in ranges)
    r = ranges[0]
    assert r[0][0] == 0 and r[-1][1] == 3000 and all(a[1] == b[0] for a, b in zip(r, r[1:]))


def test_row_split_balance():
    """kmp_row_split: range d starts at N (1 - sqrt(1 - d/parts)), so the expected pair counts
    (row p holds N - 1 - p pairs) are equal within one row's worth."""
    from uniprot_kmer_based_clustering_amd import _lib
    n = 100_000
    for parts in (1, 2, 4, 8, 64):
        s = _lib.row_split(n, parts).astype(np.int64)
        assert s[0] == 0 and s[-1] == n and np.all(np.diff(s) > 0)
        pairs = [(s[d + 1] - s[d]) * (n - 1) - (s[d + 1] * (s[d + 1] - 1) - s[d] * (s[d] - 1)) // 2
                 for d in range(parts)]
        total = n * (n - 1) // 2
        assert sum(pairs) == total
        assert max(abs(x - total / parts) for x in pairs) <= n


class OracleShardPipe(OracleSplitPipe):
    """CPU stand-in for the sharded start's stages (ShardPipeline).  split_keys: rank `part` holds
    proteins [part N / parts, (part + 1) N / parts) and sends every window (code, p) of them to the
    rank owning the code's bin (code mod parts here), region d = [count, keys...] of kcap words;
    split_group: the received windows grouped by code, df = distinct proteins, every pair (p < q)
    of a code with different classes one incidence key p << bits(N) | q routed to its row owner;
    the keys phase's overflow (RERUN, MAX_KEYS) merged into the flags, as the library does."""

    def __init__(self, b, o, cap, part, parts):
        P, Q, W = o.pairs()
        super().__init__(b.n, P, Q, W, cap)
        self.cls = np.asarray(b.class_id)
        self.part, self.parts = part, parts
        codes, woff = o.codes(), o.win_off()
        lo, hi = part * b.n // parts, (part + 1) * b.n // parts
        self.win = [(int(c), p) for p in range(lo, hi) for c in codes[woff[p]:woff[p + 1]]]
        self.kflags = (0, 0)
        self.b, self.o = b, o
        self.offsets_host = np.asarray(b.offsets, dtype=np.uint64)
        self.total = int(self.offsets_host[-1])
        self.res_lo, self.res_hi = int(self.offsets_host[lo]), int(self.offsets_host[hi])
        self.res = torch.from_numpy(np.asarray(b.residues, dtype=np.uint8)[self.res_lo:self.res_hi].copy())
        self.cap0 = cap
        self.gathered = []

    def own_residues(self):
        return self.res_lo, self.res_hi, self.res

    def gathered_pipeline(self, residues):
        """The residue start's rebuilt batch: an OracleSplitPipe (kmer_split_step's stand-in)
        carrying the gathered residues, kept for the test to compare with the batch."""
        P, Q, W = self.o.pairs()
        full = OracleSplitPipe(self.n, P, Q, W, self.cap0)
        full.res = residues.clone()
        full.k = 7
        self.gathered.append(full)
        return full

    def split_keys(self, part, parts, kcap, ksend, flags):
        need = 0
        ksend.fill_(0)
        for d in range(parts):
            mine = [(c << 32) | p for c, p in self.win if c % parts == d]
            need = max(need, len(mine) + 1)
            if len(mine) + 1 <= kcap:
                ksend[d * kcap] = len(mine)
                ksend[d * kcap + 1:d * kcap + 1 + len(mine)] = torch.tensor(mine, dtype=torch.int64)
            else:
                ksend[d * kcap] = 0  # dropped: the receiver reads nothing, the flags rerun the step
        self.kflags = (int(need > kcap), need)

    def split_group(self, krecv, kcap, part, parts, cap, send, flags, stats, learn=None, require_class_diff=True):
        from uniprot_kmer_based_clustering_amd import _lib
        from uniprot_kmer_based_clustering_amd.dist import row_ranges
        x = krecv.numpy()
        groups = {}
        for s in range(parts):
            m = int(x[s * kcap])
            for v in x[s * kcap + 1:s * kcap + 1 + m]:
                groups.setdefault(int(v) >> 32, set()).add(int(v) & 0xFFFFFFFF)
        keys = []
        for ps in groups.values():
            ps = sorted(ps)
            for i, p in enumerate(ps):
                for q in ps[i + 1:]:
                    if not require_class_diff or self.cls[p] != self.cls[q]:
                        keys.append((p << self.pbits) | q)
        keys = np.array(keys, dtype=np.int64)
        send.fill_(-1)
        most = 0
        for d, (lo, hi) in enumerate(row_ranges(self.n, parts)):
            kd = keys[((keys >> self.pbits) >= lo) & ((keys >> self.pbits) < hi)]
            most = max(most, len(kd))
            send[d * cap:d * cap + min(cap, len(kd))] = torch.from_numpy(kd[:cap].copy())
        flags.zero_()
        flags[_lib.KMP_SPLIT_MAX_PART] = most
        flags[_lib.KMP_SPLIT_MAX_KEYS] = self.kflags[1]
        flags[_lib.KMP_SPLIT_RERUN] = int(most > cap or self.kflags[0])
        stats.zero_()
        stats[6] = len(keys)


def shard_worker(rank, world, port, out_q, start="keys"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, ROOT)
        from uniprot_kmer_based_clustering_amd.dist import SplitState, sharded_split_step
        b, o = build_case()
        P, Q, W = o.pairs()
        pipe = OracleShardPipe(b, o, cap=16 if rank == 0 else 1 << 20, part=rank, parts=world)
        state = SplitState()
        state.cap, state.kcap = 64, 256  # far too small: the first step reruns with both learned
        for ms in (1, 3):
            n = sharded_split_step(pipe, rank, world, min_shared=ms, gather=True, state=state, start=start)
            if rank == 0:
                keep = W >= ms
                ok = (n == int(keep.sum())
                      and np.array_equal(pipe.ep[:n].numpy().view(np.uint32), P[keep])
                      and np.array_equal(pipe.eq[:n].numpy().view(np.uint32), Q[keep])
                      and np.array_equal(pipe.ew[:n].numpy().view(np.uint32), W[keep]))
                out_q.put(("sharded", ms, ok, n, state.reruns, state.cap, state.kcap))
    finally:
        dist.destroy_process_group()


def residue_start_worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, ROOT)
        from uniprot_kmer_based_clustering_amd.dist import SplitState, sharded_split_step, start_mode
        b, o = build_case()
        P, Q, W = o.pairs()
        pipe = OracleShardPipe(b, o, cap=16 if rank == 0 else 1 << 20, part=rank, parts=world)
        state = SplitState()
        res = np.asarray(b.residues, dtype=np.uint8)
        for step, ms in enumerate((1, 3)):
            if step:  # the rebuilt batch is refreshed in place from the slices every step
                state.full.res.zero_()
            n = sharded_split_step(pipe, rank, world, min_shared=ms, gather=True, state=state)
            same = np.array_equal(state.full.res.numpy(), res)
            if rank == 0:
                keep = W >= ms
                ok = (n == int(keep.sum())
                      and np.array_equal(pipe.ep[:n].numpy().view(np.uint32), P[keep])
                      and np.array_equal(pipe.eq[:n].numpy().view(np.uint32), Q[keep])
                      and np.array_equal(pipe.ew[:n].numpy().view(np.uint32), W[keep]))
                out_q.put(("residues", ms, ok and same, n, len(pipe.gathered), start_mode("auto", world)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_split_residue_start(world):
    """sharded_split_step's residue start (the default below 8 ranks): the ranks' residue slices
    all-gathered into the whole batch on every rank (built once, then refreshed in place by
    point-to-point receives), the k-mer split over it, the canonical list gathered on rank 0."""
    port = free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=residue_start_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    msgs = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert all(m[2] for m in msgs), msgs
    assert all(m[4] == 1 and m[5] == "residues" for m in msgs)  # built once; auto picks residues


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_split_exchange(world):
    """sharded_split_step over gloo: the key all-to-all (each rank's windows to their bins' owners),
    the grouping, the pair-key all-to-all and the per-rank reduction give the canonical list
    gathered on rank 0; undersized key and pair-key regions rerun with sizes learned from the
    reduced flags (the same on every rank), and the learned sizes stay for the next step."""
    port = free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    msgs = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert all(m[2] for m in msgs), msgs
    assert msgs[0][4] >= 1 and msgs[0][5] > 64 and msgs[0][6] > 256
    assert msgs[1][4] == msgs[0][4]  # the second step reran nothing


class OracleClassWidePipe(OracleSplitPipe):
    """The rebuilt batch of a class-wide batch: every split_expand raises KMP_SPLIT_CLASS (class ids
    too wide for the k-mer split's key), as the library's flags do."""

    def split_expand(self, part, parts, cap, send, flags, stats, learn=None, require_class_diff=True):
        from uniprot_kmer_based_clustering_amd import _lib
        super().split_expand(part, parts, cap, send, flags, stats, learn, require_class_diff)
        flags[_lib.KMP_SPLIT_CLASS] = 1


class OracleClassWideShardPipe(OracleShardPipe):
    def gathered_pipeline(self, residues):
        P, Q, W = self.o.pairs()
        full = OracleClassWidePipe(self.n, P, Q, W, self.cap0)
        full.res = residues.clone()
        full.k = 7
        self.gathered.append(full)
        return full


def class_fallback_worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, ROOT)
        from uniprot_kmer_based_clustering_amd.dist import SplitState, row_ranges, sharded_split_step
        b, o = build_case()
        P, Q, W = o.pairs()
        lo, hi = row_ranges(b.n, world)[rank]
        for gather in (True, False):
            pipe = OracleClassWideShardPipe(b, o, cap=16 if rank == 0 else 1 << 20, part=rank, parts=world)
            state = SplitState()
            for step in range(2):  # the first step falls back inside the split, the second starts there
                n = sharded_split_step(pipe, rank, world, gather=gather, state=state, start="residues")
                if gather and rank != 0:
                    continue
                keep = np.ones(len(P), bool) if gather else (P >= lo) & (P < hi)
                ok = (n == int(keep.sum())
                      and np.array_equal(pipe.ep[:n].numpy().view(np.uint32), P[keep])
                      and np.array_equal(pipe.eq[:n].numpy().view(np.uint32), Q[keep])
                      and np.array_equal(pipe.ew[:n].numpy().view(np.uint32), W[keep]))
                out_q.put(("class", gather, step, rank, ok, n, state.row_split, len(pipe.gathered)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_class_fallback_on_residue_start(world):
    """Class ids too wide for the key on the residue start: the split's reduced CLASS flag sends the
    step to the row split over the same rebuilt batch, once — rank 0 holds the canonical list exactly
    (no rank's block gathered twice) with gather, and every rank its own rows without it, on the
    step that falls back and on the next one."""
    port = free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=class_fallback_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    msgs = [q.get(timeout=300) for _ in range(2 + 2 * world)]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert all(m[4] and m[6] for m in msgs), msgs
    assert all(m[7] == 1 for m in msgs)  # the batch rebuilt once


def test_own_residues_with_fewer_chunks_than_ranks():
    """ShardPipeline.own_residues: with 2 key chunks on 4 ranks, two ranks hold no chunk.  The
    ranks' contributions still tile the residues every window reads, so the batch the residue start
    and the row-split fallback rebuild is the batch (host-only: the split plan and the slices)."""
    import uniprot_kmer_based_clustering_amd as K
    from uniprot_kmer_based_clustering_amd import _lib
    from uniprot_kmer_based_clustering_amd.device import ShardPipeline
    b = K.synth(20, 3)  # ~6,000 residues: two 4,096-slot chunks
    res = np.asarray(b.residues, dtype=np.uint8)
    off = np.asarray(b.offsets, dtype=np.uint64)
    for parts in (2, 3, 4, 8):
        spans = []
        for part in range(parts):
            sp = ShardPipeline(res, off, b.class_id, 7, part, parts, device="cpu")
            lo, hi, own = sp.own_residues()
            assert own.numel() == hi - lo and np.array_equal(own.numpy(), res[lo:hi])
            if hi > lo:
                spans.append((lo, hi))
        assert spans[0][0] == 0 and spans[-1][1] == int(off[-1]), (parts, spans)
        assert all(a[1] == c[0] for a, c in zip(spans, spans[1:])), (parts, spans)
        if parts == 4:
            empty = [d for d in range(parts) if int(_lib.split_plan(off, 7, d, parts).res_hi) ==
                     int(_lib.split_plan(off, 7, d, parts).res_lo)]
            assert empty, "the case needs a rank without chunks"


def test_sharded_split_world8_auto_start():
    """The collective sequence the 8-GPU bench runs (bench.py --gpus 8: sharded_split_step with
    start='auto', which resolves to the key start from KEYS_START_MIN_WORLD ranks): key all-to-all,
    pair-key all-to-all, flag all-reduce, reruns with learned capacities and the rank-order gather,
    in 8 processes over gloo — the canonical list on rank 0."""
    from uniprot_kmer_based_clustering_amd.dist import KEYS_START_MIN_WORLD, start_mode
    world = 8
    assert start_mode("auto", world) == "keys" and KEYS_START_MIN_WORLD <= world
    port = free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=shard_worker, args=(r, world, port, q, "auto")) for r in range(world)]
    for p in procs:
        p.start()
    msgs = [q.get(timeout=600) for _ in range(2)]
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    assert all(m[2] for m in msgs), msgs
    assert msgs[0][4] >= 1 and msgs[1][4] == msgs[0][4]  # reran once with the learned sizes, then not
