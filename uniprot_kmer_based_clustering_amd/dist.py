"""Multi-GPU split of the pair path: one process per GPU, torch.distributed over RCCL.

Postings engines (default; ``distributed_postings``) — the reference's algorithm sharded by
k-mer, two all-to-all exchanges:
  1. rank r turns the k-mer windows of its protein slice into keys, sorted by k-mer bucket
     (kmp_dev_keys_part);
  2. all-to-all: every key goes to the owner of its bucket range (RCCL over xGMI);
  3. the owner groups, deduplicates and expands its k-mers into (p, q) pair keys
     (kmp_dev_pairs_keys; the bucketed engine on 1/G of the keys), sorted;
  4. all-to-all: every pair key goes to the owner of its p range;
  5. the owner reduces the runs to edges w(p, q) (kmp_dev_edges_pairkeys): its p range of the
     canonical edge list;
  6. edges are gathered to rank 0 in rank order — already canonical, no final sort.

Tiles engine (``distributed_step(engine="tiles")``) — the N x N pair space shards with one
exchange step:
  1. rank r builds K(p) for its contiguous protein slice (balanced by residue count);
  2. all-gather of the slices' set slots and set sizes (RCCL over xGMI) -> every rank holds
     every K(p) in the same layout;
  3. every rank applies the repeat filter and plans the same (tile, chunk) item list, then
     runs the pair kernel on its contiguous, cost-balanced share of the items (no further
     communication during compute);
  4. per-rank edge counts and edges are gathered to rank 0, which sorts them into the
     canonical (p, q) order.

The collective helpers only move tensors, so the same code runs on gloo with CPU tensors in
the multi-process CPU tests (tests/test_dist.py).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from . import _lib


def protein_slices(offsets: np.ndarray, world: int) -> list:
    """Contiguous [lo, hi) protein ranges with about equal residue counts."""
    n = len(offsets) - 1
    if world <= 1:
        return [(0, n)]
    total = int(offsets[-1])
    cuts = [0]
    for r in range(1, world):
        c = int(np.searchsorted(offsets, total * r / world, side="left"))
        cuts.append(min(max(c, cuts[-1]), n))
    cuts.append(n)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def slot_range(offsets: np.ndarray, lo: int, hi: int) -> tuple:
    """Element range of the per-protein slot buffer owned by proteins [lo, hi)."""
    L = _lib.lib()
    return int(L.kmp_set_base(int(offsets[lo]), lo)), int(L.kmp_set_base(int(offsets[hi]), hi))


def allgather_ranges(buf: torch.Tensor, ranges: list, rank: int, group=None) -> None:
    """Every rank contributes buf[ranges[rank]]; afterwards every rank's buf holds all ranges.
    Equal-size (padded) all_gather: works on RCCL and on gloo."""
    world = len(ranges)
    if world == 1:
        return
    width = max(1, max(h - l for l, h in ranges))
    lo, hi = ranges[rank]
    send = torch.zeros(width, dtype=buf.dtype, device=buf.device)
    send[:hi - lo] = buf[lo:hi]
    parts = [torch.empty_like(send) for _ in range(world)]
    dist.all_gather(parts, send, group=group)
    for r, (l, h) in enumerate(ranges):
        if r != rank and h > l:
            buf[l:h] = parts[r][:h - l]


def allgather_sets(set_buf: torch.Tensor, set_len: torch.Tensor, offsets: np.ndarray, slices: list,
                   rank: int, group=None) -> None:
    allgather_ranges(set_buf, [slot_range(offsets, lo, hi) for lo, hi in slices], rank, group)
    allgather_ranges(set_len, slices, rank, group)


def gather_edges(ep: torch.Tensor, eq: torch.Tensor, ew: torch.Tensor, count: int, rank: int, group=None):
    """All ranks' (p, q, w) concatenated in rank order on rank 0 (None elsewhere)."""
    world = dist.get_world_size(group)
    dev = ep.device
    if _staged(ep, group):
        got = gather_edges(ep[:count].cpu(), eq[:count].cpu(), ew[:count].cpu(), count, rank, group)
        return None if got is None else tuple(t.to(dev) for t in got)
    cnt = torch.tensor([count], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    width = max(1, max(counts))
    send = torch.zeros((3, width), dtype=torch.int32, device=dev)
    send[0, :count] = ep[:count]
    send[1, :count] = eq[:count]
    send[2, :count] = ew[:count]
    parts = [torch.empty_like(send) for _ in range(world)]
    dist.all_gather(parts, send, group=group)
    if rank != 0:
        return None
    out = torch.cat([parts[r][:, :counts[r]] for r in range(world)], dim=1)
    return out[0].contiguous(), out[1].contiguous(), out[2].contiguous()


def _staged(t: torch.Tensor, group) -> bool:
    """gloo moves CPU tensors only: device tensors are staged through the host."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def exchange(send: torch.Tensor, counts: list, group=None) -> torch.Tensor:
    """all-to-all with uneven splits: send[sum(counts[:j]) : sum(counts[:j+1])] goes to rank j;
    returns what every rank sent to this one, in source-rank order."""
    dev = send.device
    staged = _staged(send, group)
    cdev = torch.device("cpu") if staged or not send.is_cuda else dev
    cnt = torch.tensor([int(c) for c in counts], dtype=torch.int64, device=cdev)
    rcnt = torch.empty_like(cnt)
    dist.all_to_all_single(rcnt, cnt, group=group)
    rc = [int(x) for x in rcnt.tolist()]
    src = send[:sum(int(c) for c in counts)]
    if staged:
        src = src.cpu()
    recv = torch.empty(sum(rc), dtype=send.dtype, device=src.device)
    dist.all_to_all_single(recv, src, rc, [int(c) for c in counts], group=group)
    return recv.to(dev) if staged else recv


class DeviceStages:
    """The three device stages of the distributed postings flow on a DevicePipeline (the
    kmp_dev_keys_part / kmp_dev_pairs_keys / kmp_dev_edges_pairkeys entry points)."""

    def __init__(self, pipe, min_shared: int = 1, require_class_diff: bool = True):
        import ctypes as C
        self.C = C
        self.pipe = pipe
        self.L = _lib.lib()
        self.ws = pipe._workspace()
        self.slots = int(self.L.kmp_set_capacity(pipe.n, pipe.total))
        self.min_shared = min_shared
        self.require_class_diff = require_class_diff
        self.pk_cap = 1 << 20
        self.stats = _lib.PostingsStats()

    def _stream(self):
        return self.C.c_void_p(torch.cuda.current_stream(self.pipe.dev).cuda_stream)

    def _ptr(self, t):
        return self.C.c_void_p(t.data_ptr())

    def keys_part(self, lo: int, hi: int, parts: int):
        C, L, p = self.C, self.L, self.pipe
        off = p.offsets_host
        slot_lo = int(L.kmp_set_base(int(off[lo]), lo))
        slot_hi = int(L.kmp_set_base(int(off[hi]), hi))
        out = torch.empty(max(1, slot_hi - slot_lo), dtype=torch.int64, device=p.dev)
        counts = (C.c_uint64 * parts)()
        _lib.check(L.kmp_dev_keys_part(self.ws, self._ptr(p.res), self._ptr(p.off), self._ptr(p.cls), p.n, p.k,
                                       self.slots, lo, hi, slot_lo, slot_hi, parts, self._ptr(out), out.numel(),
                                       counts, self._stream()), "kmp_dev_keys_part")
        return out, [int(c) for c in counts]

    def pairs_keys(self, keys: torch.Tensor, parts: int):
        C, L, p = self.C, self.L, self.pipe
        counts = (C.c_uint64 * parts)()
        ni = C.c_uint64()
        for _ in range(3):
            out = torch.empty(max(1, self.pk_cap), dtype=torch.int64, device=p.dev)
            st = L.kmp_dev_pairs_keys(self.ws, self._ptr(keys), keys.numel(), p.n, p.k, self.slots, 0xFFFFFFFF,
                                      int(self.require_class_diff), parts, self._ptr(out), out.numel(),
                                      C.byref(ni), counts, C.byref(self.stats), self._stream())
            if st == _lib.KMP_EOVERFLOW:
                self.pk_cap = ni.value + ni.value // 8 + 1024
                continue
            _lib.check(st, "kmp_dev_pairs_keys")
            return out[:ni.value], [int(c) for c in counts]
        raise RuntimeError("pair-key count unstable across reruns")

    def edges_pairkeys(self, pk: torch.Tensor):
        C, L, p = self.C, self.L, self.pipe
        m = pk.numel()  # every edge is at least one incidence: m bounds the edge count
        ep, eq, ew = (torch.empty(max(1, m), dtype=torch.int32, device=p.dev) for _ in range(3))
        ne, npairs = C.c_uint64(), C.c_uint64()
        _lib.check(L.kmp_dev_edges_pairkeys(self.ws, self._ptr(pk), m, p.n, self.min_shared, self._ptr(ep),
                                            self._ptr(eq), self._ptr(ew), max(1, m), C.byref(ne), C.byref(npairs),
                                            self._stream()), "kmp_dev_edges_pairkeys")
        return ep, eq, ew, ne.value


def distributed_postings(stages, offsets: np.ndarray, rank: int, world: int, group=None):
    """The postings flow above on `stages` (DeviceStages, or a stand-in with the same three
    methods).  Returns rank 0's gathered canonical edges (p, q, w) and None elsewhere, plus this
    rank's edge count."""
    lo, hi = protein_slices(offsets, world)[rank]
    keys, kc = stages.keys_part(lo, hi, world)
    mine = exchange(keys, kc, group)
    pk, pc = stages.pairs_keys(mine, world)
    pk_mine = exchange(pk, pc, group)
    ep, eq, ew, m = stages.edges_pairkeys(pk_mine)
    return gather_edges(ep, eq, ew, m, rank, group), m


def exchange_equal(send: torch.Tensor, group=None) -> torch.Tensor:
    """all-to-all of `world` equal regions (region j -> rank j); no count exchange."""
    dev = send.device
    staged = _staged(send, group)
    src = send.cpu() if staged else send
    recv = torch.empty_like(src)
    dist.all_to_all_single(recv, src, group=group)
    return recv.to(dev) if staged else recv


def gather_to_rank0(flat: torch.Tensor, count: int, counts: list, rank: int, group=None):
    """Rank r's first `count` elements -> rank 0, concatenated in rank order (one uneven
    all-to-all: every rank sends only to rank 0)."""
    world = len(counts)
    dev = flat.device
    staged = _staged(flat, group)
    src = flat[:count].cpu() if staged else flat[:count]
    in_splits = [count] + [0] * (world - 1)
    out_splits = counts if rank == 0 else [0] * world
    recv = torch.empty(sum(out_splits), dtype=flat.dtype, device=src.device)
    dist.all_to_all_single(recv, src.contiguous(), out_splits, in_splits, group=group)
    return (recv.to(dev) if staged else recv) if rank == 0 else None


class DeviceRouteStages:
    """The fixed-capacity device stages (kmp_dev_keys_route / kmp_dev_pairs_route /
    kmp_dev_edges_route) on a DevicePipeline.  Capacities are learned: a flagged step reports
    the sizes it needed and the caller reruns after grow()."""

    def __init__(self, pipe, require_class_diff: bool = True):
        import ctypes as C
        self.C = C
        self.pipe = pipe
        self.L = _lib.lib()
        self.ws = pipe._workspace()
        self.slots = int(self.L.kmp_set_capacity(pipe.n, pipe.total))
        self.require_class_diff = require_class_diff
        self.cap_keys = 0
        self.cap_pairs = 0
        self.shard_cap = 0
        self.flags = torch.zeros(8, dtype=torch.int32, device=pipe.dev)
        self.count = torch.zeros(1, dtype=torch.int64, device=pipe.dev)
        self.stats = _lib.PostingsStats()

    def _stream(self):
        return self.C.c_void_p(torch.cuda.current_stream(self.pipe.dev).cuda_stream)

    def _ptr(self, t):
        return self.C.c_void_p(t.data_ptr())

    def begin(self, world: int):
        p = self.pipe
        if self.cap_keys == 0:  # first guesses: an even split + 10 %
            self.cap_keys = self.slots // (world * world) + self.slots // (10 * world * world) + 4096
            self.shard_cap = self.slots // (4 * 64 * world) + 4096
            self.cap_pairs = self.slots // (4 * world * world) + 4096
        self.flags.zero_()

    def keys_route(self, lo: int, hi: int, parts: int) -> torch.Tensor:
        L, p = self.L, self.pipe
        off = p.offsets_host
        slot_lo = int(L.kmp_set_base(int(off[lo]), lo))
        slot_hi = int(L.kmp_set_base(int(off[hi]), hi))
        send = torch.empty(parts * self.cap_keys, dtype=torch.int64, device=p.dev)
        _lib.check(L.kmp_dev_keys_route(self.ws, self._ptr(p.res), self._ptr(p.off), self._ptr(p.cls), p.n, p.k,
                                        self.slots, lo, hi, slot_lo, slot_hi, parts, self.cap_keys,
                                        self._ptr(send), self._ptr(self.flags), self._stream()),
                   "kmp_dev_keys_route")
        return send

    def pairs_route(self, keys: torch.Tensor, part: int, parts: int) -> torch.Tensor:
        L, p = self.L, self.pipe
        send = torch.empty(parts * self.cap_pairs, dtype=torch.int64, device=p.dev)
        _lib.check(L.kmp_dev_pairs_route(self.ws, self._ptr(keys), keys.numel(), p.n, p.k, self.slots, 0xFFFFFFFF,
                                         int(self.require_class_diff), self.shard_cap, part, parts, self.cap_pairs,
                                         self._ptr(send), self._ptr(self.flags), self.C.byref(self.stats),
                                         self._stream()), "kmp_dev_pairs_route")
        return send

    def edges_route(self, pk: torch.Tensor, part: int, parts: int):
        """Interleaved (p, q, w) int32 triples (a flat [3 m] buffer) and the edge count (device): the
        row-block tail over this part's rows (kmp_dev_edges_rows; the count is KMP_EDGES_RETRY when a
        row block did not fit in LDS, see disable_rowtail)."""
        L, p = self.L, self.pipe
        m = pk.numel()
        e = torch.empty(3 * max(1, m), dtype=torch.int32, device=p.dev)
        rows = (self.C.c_uint32 * (parts + 1))()
        L.kmp_row_split(p.n, parts, rows)
        _lib.check(L.kmp_dev_edges_rows(self.ws, self._ptr(pk), m, p.n, rows[part], rows[part + 1], self._ptr(e),
                                        max(1, m), self._ptr(self.count), self._stream()), "kmp_dev_edges_rows")
        return e, self.count

    def disable_rowtail(self) -> None:
        """A row block exceeded the LDS capacity somewhere: reduce with the global sort tail."""
        _lib.check(self.L.kmp_postings_set_rowtail(self.ws, 0), "kmp_postings_set_rowtail")

    def status(self) -> torch.Tensor:
        """flags[0..7] + edge count, as one int64 device tensor (gathered across ranks)."""
        return torch.cat([self.flags.to(torch.int64), self.count])

    def grow(self, worst: np.ndarray) -> None:
        """worst = element-wise max of every rank's flags."""
        if worst[0]:
            self.cap_keys = max(self.cap_keys, int(worst[4]) + int(worst[4]) // 16 + 1024)
            self.cap_pairs = max(self.cap_pairs, int(worst[6]) + int(worst[6]) // 16 + 1024)
        if worst[3]:
            self.shard_cap = max(self.shard_cap, int(worst[5]) + int(worst[5]) // 16 + 1024)


EDGES_RETRY = 1 << 62  # KMP_EDGES_RETRY (kmerpair.h)


class RouteFallback(RuntimeError):
    """The batch needs the single-GPU flat layout (a very frequent k-mer or wide class ids)."""


def distributed_postings_padded(stages, offsets: np.ndarray, rank: int, world: int, group=None,
                                max_attempts: int = 4):
    """The fixed-capacity flow: keys routed by bucket range, pair keys routed by p range, edges
    to rank 0 in rank order (= canonical).  One host synchronisation per attempt: the all-gather
    of every rank's flags and edge count.  Returns rank 0's flat int32 tensor of interleaved
    (p, q, w) triples (all ranks' edges, canonical order) and the per-rank counts; None elsewhere."""
    lo, hi = protein_slices(offsets, world)[rank]
    for _ in range(max_attempts):
        stages.begin(world)
        mine = exchange_equal(stages.keys_route(lo, hi, world), group)
        pk = exchange_equal(stages.pairs_route(mine, rank, world), group)
        e, count = stages.edges_route(pk, rank, world)
        st = stages.status()
        parts = [torch.empty_like(st) for _ in range(world)]
        if _staged(st, group):
            cpu = [torch.empty_like(st, device="cpu") for _ in range(world)]
            dist.all_gather(cpu, st.cpu(), group=group)
            table = torch.stack(cpu).numpy()
        else:
            dist.all_gather(parts, st, group=group)
            table = torch.stack(parts).cpu().numpy()  # the step's one host synchronisation
        worst = table[:, :8].max(axis=0)
        if worst[1] or worst[2]:
            raise RouteFallback("batch needs the single-GPU flat layout (frequent k-mer or wide class id)")
        if worst[0] or worst[3]:
            stages.grow(worst)
            continue
        if (table[:, 8] >= EDGES_RETRY).any():  # a row too long for the LDS row-block tail
            stages.disable_rowtail()
            continue
        counts = [int(c) for c in table[:, 8]]
        c = counts[rank]
        got = gather_to_rank0(e, 3 * c, [3 * x for x in counts], rank, group)  # triples: no repacking
        return got, counts
    raise RuntimeError("exchange capacities did not converge")


def distributed_step(pipe, rank: int, world: int, group=None, min_shared: int = 1,
                     require_class_diff: bool = True, timers: dict | None = None, engine: str = "residues") -> int:
    """One multi-GPU pass of the path on a DevicePipeline holding the whole batch.
    Returns the canonical edge count (rank 0) or this rank's share (others)."""
    if engine in ("residues", "postings") and min_shared == 1:
        stages = getattr(pipe, "_route_stages", None)
        if stages is None or stages.require_class_diff != require_class_diff:
            stages = pipe._route_stages = DeviceRouteStages(pipe, require_class_diff)
        got, counts = distributed_postings_padded(stages, pipe.offsets_host, rank, world, group)
        if rank == 0:
            n = sum(counts)
            if n > pipe.edge_cap:
                pipe._alloc_edges(n + n // 8 + 1024)
            tri = got[:3 * n].view(n, 3)  # interleaved triples, already in canonical order
            pipe.ep[:n] = tri[:, 0]
            pipe.eq[:n] = tri[:, 1]
            pipe.ew[:n] = tri[:, 2]
            pipe.n_edges = n
            return n
        return counts[rank]
    if engine in ("residues", "postings"):
        stages = getattr(pipe, "_dist_stages", None)
        if stages is None or stages.min_shared != min_shared or stages.require_class_diff != require_class_diff:
            stages = pipe._dist_stages = DeviceStages(pipe, min_shared, require_class_diff)
        got, m = distributed_postings(stages, pipe.offsets_host, rank, world, group)
        if rank == 0:
            n = got[0].numel()
            if n > pipe.edge_cap:
                pipe._alloc_edges(n + n // 8 + 1024)
            pipe.ep[:n] = got[0]
            pipe.eq[:n] = got[1]
            pipe.ew[:n] = got[2]
            pipe.n_edges = n
            return n
        return m
    slices = protein_slices(pipe.offsets_host, world)
    lo, hi = slices[rank]
    pipe.build_sets(lo, hi)
    allgather_sets(pipe.set, pipe.set_len, pipe.offsets_host, slices, rank, group)
    pipe.filter()
    pipe.plan(rank, world)
    ev = timers.get("pairs") if timers is not None else None
    if ev is not None:
        ev[0].record()
    n_local = pipe.pairs(min_shared, require_class_diff)
    if ev is not None:
        ev[1].record()
    got = gather_edges(pipe.ep, pipe.eq, pipe.ew, n_local, rank, group)
    if rank == 0:
        n = got[0].numel()
        if n > pipe.edge_cap:
            pipe._alloc_edges(n + n // 8 + 1024)
        pipe.ep[:n] = got[0]
        pipe.eq[:n] = got[1]
        pipe.ew[:n] = got[2]
        pipe.n_edges = n
        pipe.sort(n)
        return n
    return n_local
