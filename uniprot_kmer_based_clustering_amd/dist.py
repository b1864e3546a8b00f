"""Multi-GPU split of the pair path: one process per GPU, torch.distributed over
RCCL (``nccl`` backend) — the path used by ``bench.py --gpus N`` under torch.distributed.run.

The pair space is split by ROWS.  A pair (p, q), p < q, belongs to its smaller protein p, and
rank r owns the rows [start[r], start[r+1]) of ``kmp_row_split`` (equal expected pair counts:
row p holds about N - p pairs).  Every rank holds the whole packed residue batch (ΣL bytes:
30 MB at config 3), groups every k-mer itself and expands only its own rows
(``kmp_dev_pairs_rows``): a k-mer group is never split, so every pair's w is complete on the
rank that owns it.  There is no exchange in the data path — the ranks' edge lists are disjoint
and each is already canonical — and rank 0 gathers them in rank order: the concatenation IS the
canonical list, no final sort (cf. main.rs:84-121 / mod.rs:81-124, the reference's own split of
the same work over `threads` workers).

Why not an all-to-all: sharding the k-mers instead (each rank groups 1/G of them) moves every
pair key to its row owner — 42 MB per step at config 3, but Σ C(df,2) x 8 B ≈ 10^12 B at
config 5, far more than recomputing the grouping on each rank (≈ 5·10^8 windows).

The gather only moves tensors, so the same code runs on gloo with CPU tensors in the
multi-process CPU tests (tests/test_dist.py).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from . import _lib


def row_ranges(n: int, world: int) -> list:
    """[(lo, hi)] per rank: kmp_row_split's equal-pair-count row ranges."""
    s = _lib.row_split(n, world)
    return [(int(s[r]), int(s[r + 1])) for r in range(world)]


def gather_rows(parts: list, count: int, rank: int, world: int, group=None, grow=None) -> int:
    """Rank-order concatenation on rank 0 of every rank's `count` leading elements of the
    tensors in `parts` (same dtype on every rank), in place: rank 0's own block is already at
    the front of its tensors and the other ranks' blocks are received straight behind it
    (point-to-point over xGMI on RCCL).  Counts travel with one all_gather.  grow(total), on
    rank 0, may replace `parts` with larger tensors holding the same leading block (it returns
    them).  Returns the total count on rank 0 and `count` elsewhere."""
    dev = parts[0].device
    cnt = torch.tensor([count], dtype=torch.int64, device=dev)
    counts = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    if rank != 0:
        ops = [dist.P2POp(dist.isend, t[:count], 0, group=group) for t in parts] if count else []
        for w in (dist.batch_isend_irecv(ops) if ops else []):
            w.wait()
        return count
    total = sum(counts)
    if total > parts[0].numel():
        if grow is None:
            raise ValueError("gather_rows: destination too small")
        parts = grow(total)
    ops, off = [], counts[0]
    for r in range(1, world):
        if counts[r]:
            ops += [dist.P2POp(dist.irecv, t[off:off + counts[r]], r, group=group) for t in parts]
        off += counts[r]
    for w in (dist.batch_isend_irecv(ops) if ops else []):
        w.wait()
    return total


def distributed_step(pipe, rank: int, world: int, group=None, min_shared: int = 1,
                     require_class_diff: bool = True) -> int:
    """One multi-GPU step on a DevicePipeline: this rank's rows, then the gather to rank 0.
    Rank 0 returns the total edge count and holds the canonical list in pipe.ep/eq/ew (first
    n entries); the other ranks return their own row range's edge count."""
    lo, hi = row_ranges(pipe.n, world)[rank]
    m = pipe.rows(lo, hi, min_shared=min_shared, require_class_diff=require_class_diff)
    if world == 1:
        return m

    def grow(total):
        old = (pipe.ep[:m].clone(), pipe.eq[:m].clone(), pipe.ew[:m].clone())
        pipe._alloc_edges(total + total // 8)
        for dst, src in zip((pipe.ep, pipe.eq, pipe.ew), old):
            dst[:m].copy_(src)
        return [pipe.ep, pipe.eq, pipe.ew]

    total = gather_rows([pipe.ep, pipe.eq, pipe.ew], m, rank, world, group, grow)
    if rank == 0:
        pipe.n_edges = total
    return total
