"""Multi-GPU split of the pair path: one process per GPU, torch.distributed over RCCL.

The N x N pair space shards with one real exchange step:
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


def distributed_step(pipe, rank: int, world: int, group=None, min_shared: int = 1,
                     require_class_diff: bool = True, timers: dict | None = None) -> int:
    """One multi-GPU pass of the path on a DevicePipeline holding the whole batch.
    Returns the canonical edge count (rank 0) or this rank's share (others)."""
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
