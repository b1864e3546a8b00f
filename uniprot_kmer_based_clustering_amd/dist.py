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

The k-mer split (``kmer_split_step``, the default of ``bench.py --gpus N``) divides the work
instead of repeating the grouping on every rank: rank r keys every window but keeps only the
k-mers of its share of the bucket hash range, groups and expands them, and routes each pair key
to the rank owning the pair's row (kmp_dev_split_expand); one all-to-all of equal, padded splits
moves the pair keys (42 MB in total per step at config 4, about 5 MB per rank at 8 ranks); every
rank reduces its rows (kmp_dev_split_edges).  Frequent k-mers stay on the k-mer split: a rank
whose share spills raises KMP_SPLIT_HEAVY, the step reruns with the heavy path on in every rank
(each compacts, plans and expands the spill of its own k-mers into the keys it routes).  The row
split stays the fallback for class ids wider than the key's field and the bounded-memory mode: at
config 5 Σ C(df,2) ≈ 10^10-10^11 pair keys would cross the links, far more than recomputing the
grouping.
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
    allc = torch.zeros(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(allc, cnt, group=group)
    counts = [int(c) for c in allc.tolist()]  # one read-back, not one per rank
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


class SplitState:
    """Learned state of the k-mer split, identical on every rank (it only changes from flags
    reduced over the ranks): the per-destination send capacity, the flags to learn from on a
    rerun, the exchange buffers, the host copy of the reduced flags, and whether the batch needs
    the row split."""

    def __init__(self, key=None):
        self.key = key  # (n, total residues, k, residue buffer) of the batch it was learned on
        self.cap = 0
        self.learn = None
        self.bufs = None
        self.host_flags = None  # pinned (CUDA) host copy of the reduced flags, copied asynchronously
        self.row_split = False
        self.reruns = 0
        self.rerun_flags = []  # the reduced flags of each rerun (diagnostics)


def _pipe_state(pipe) -> SplitState:
    """The pipe's cached SplitState, reset when its batch or k changed (a k that spills frequent
    k-mers must not pin the row split, or its capacities, on another k of the same batch)."""
    key = (pipe.n, pipe.total, pipe.k, pipe.res.data_ptr() if hasattr(pipe, "res") else 0)
    st = pipe.__dict__.get("_split_state")
    if st is None or st.key != key:
        st = SplitState(key)
        pipe.__dict__["_split_state"] = st
    return st


def kmer_split_step(pipe, rank: int, world: int, group=None, min_shared: int = 1, require_class_diff: bool = True,
                    gather: bool = False, state: SplitState | None = None, timings: list | None = None) -> int:
    """One multi-GPU step of the k-mer split: expand this rank's k-mers, exchange the pair keys by
    row owner (all-to-all), reduce this rank's rows.  Every rank ends holding the canonical edges
    of its row range in pipe.ep/eq/ew (rank order = canonical order) and returns their count; with
    gather, rank 0 also receives every rank's block behind its own and returns the total.  A batch
    that spills frequent k-mers reruns with the heavy path on (KMP_SPLIT_HEAVY in the reduced flags);
    one whose class ids overflow the key falls back to the row split (distributed_step).  timings: a
    list to append this rank's (expand, exchange, edges) milliseconds to (CUDA events on the
    current stream, which the library's stages and the collectives are ordered with)."""
    st = state if state is not None else _pipe_state(pipe)
    if st.row_split:
        return distributed_step(pipe, rank, world, group, min_shared, require_class_diff)
    lo, hi = row_ranges(pipe.n, world)[rank]
    dev = pipe.dev if hasattr(pipe, "dev") else torch.device("cpu")
    if world == 1 and hasattr(pipe, "step"):
        # one rank owns every k-mer and every row: nothing to route or exchange, so the fused
        # single-GPU step (0.567 ms at config 3 against 0.618 for split_expand + split_edges)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)] if timings is not None else None
        if ev:
            ev[0].record()
        m = pipe.step(min_shared, require_class_diff)
        if ev:
            ev[1].record()
            torch.cuda.synchronize()
            timings.append((ev[0].elapsed_time(ev[1]), 0.0, 0.0))
        return m
    if st.cap == 0:  # expected pair keys per (source, destination): a quarter of the windows / world^2
        st.cap = max(4096, int(pipe.total // 4 // (world * world)))
    m = 0
    for _ in range(8):
        if st.bufs is None or st.bufs[0].numel() != world * st.cap:
            st.bufs = (torch.empty(world * st.cap, dtype=torch.int64, device=dev),
                       torch.empty(world * st.cap, dtype=torch.int64, device=dev),
                       torch.zeros(_lib.KMP_SPLIT_FLAGS, dtype=torch.int32, device=dev),
                       torch.zeros(8, dtype=torch.int64, device=dev))
        send, recv, flags, stats = st.bufs
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if timings is not None else None
        if ev:
            ev[0].record()
        pipe.split_expand(rank, world, st.cap, send, flags, stats, learn=st.learn,
                          require_class_diff=require_class_diff)
        if ev:
            ev[1].record()
        if world > 1:
            dist.all_to_all_single(recv, send, group=group)
            dist.all_reduce(flags, op=dist.ReduceOp.MAX, group=group)
        else:
            recv = send
        # the reduced flags go to the host behind the collectives on the same stream, with an event
        # behind the copy; split_edges usually synchronises the stream already, so waiting on the
        # event below costs nothing more (no read-back of its own per step)
        if st.host_flags is None or st.host_flags.numel() != flags.numel():
            st.host_flags = torch.empty(flags.shape, dtype=flags.dtype, pin_memory=dev.type == "cuda")
        st.host_flags.copy_(flags, non_blocking=dev.type == "cuda")
        copied = torch.cuda.Event() if dev.type == "cuda" else None
        if copied is not None:
            copied.record()
        if ev:
            ev[2].record()
        m = pipe.split_edges(recv, lo, hi, min_shared)
        if ev:
            ev[3].record()
        if copied is not None:
            copied.synchronize()  # the host copy of the flags has landed
        fl = [int(x) for x in st.host_flags.tolist()]
        if fl[_lib.KMP_SPLIT_CLASS]:
            st.row_split = True
            return distributed_step(pipe, rank, world, group, min_shared, require_class_diff)
        if fl[_lib.KMP_SPLIT_RERUN] or fl[_lib.KMP_SPLIT_HEAVY]:  # HEAVY: the heavy path on every rank
            st.reruns += 1
            st.rerun_flags.append(fl)
            st.learn = fl
            if fl[_lib.KMP_SPLIT_MAX_PART] > st.cap:
                st.cap = fl[_lib.KMP_SPLIT_MAX_PART] + fl[_lib.KMP_SPLIT_MAX_PART] // 16 + 1024
            continue
        st.learn = None
        if ev:
            torch.cuda.synchronize()
            timings.append(tuple(ev[i].elapsed_time(ev[i + 1]) for i in range(3)))
        break
    else:
        raise RuntimeError("k-mer split: capacities unstable across reruns")
    if not gather or world == 1:
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
