"""Multi-GPU split of the pair path: one process per GPU, torch.distributed over
RCCL (``nccl`` backend) — the path of ``bench.py --gpus N`` under torch.distributed.run.  The
reference's own parallelism is a pool of `threads` workers over the same work (main.rs:84-121,
graph/mod.rs:81-124); here the work is split over GPUs by k-mer and by row.

**Default: the k-mer split with a sharded start** (``sharded_split_step`` on a ``ShardPipeline``).
Rank r holds only the residues of its own 4,096-slot chunks (about 1/G of the packed batch; the
offsets and class ids are replicated metadata).  One step:
  1. split_keys: the rank keys its windows once (radix-21 codes, protein.rs:29-37) and ranks them
     by coarse bin of h(code); the keys of rank d's bins go to region d of the key buffer;
  2. all-to-all of the key regions (8 B per window: 29 MB per rank at config 4 and G = 8, the same
     volume an all-gather of the residues would move, but nothing is keyed twice);
  3. split_group: the received keys of the rank's bins grouped by k-mer and expanded to pair keys
     (Graph::new + update_graph_edges with the class filter, vertex.rs:59-140, mod.rs:580-587),
     each routed to the rank owning the pair's row (the smaller protein; ``kmp_row_split`` ranges
     of equal pair counts);
  4. all-to-all of the pair keys (8 B per incidence: 42 MB in total at config 4) and a max-reduce
     of the flags (capacities learned identically on every rank; frequent k-mers turn every rank's
     heavy path on);
  5. split_edges: the rank's rows reduced to canonical (p, q, w) (combine_edges, mod.rs:322-546).
A pair's incidences from every k-mer meet on its row owner, so w is complete there; the rank-order
concatenation of the ranks' edges is the canonical list, and with ``gather`` rank 0 receives every
rank's block behind its own (point-to-point) so the timed step ends with the whole list on rank 0.

**The start exchange** (``start_mode``): from KEYS_START_MIN_WORLD = 8 ranks up the keys
all-to-all above; below it the ranks all-gather their residue slices instead (1 B per residue:
15 MB per rank at G = 2 against 67 MB of padded key regions) and every rank keys every window,
keeping its own bins (``kmer_split_step`` on the rebuilt batch, refreshed in place every step).

**Fallbacks.**  Class ids wider than the key's class field (every rank sees KMP_SPLIT_CLASS in the
reduced flags) rebuild the batch on every rank with an all-gather of the residue slices and take
the row split (``distributed_step``: every rank groups every k-mer and expands only its own rows,
no exchange in the data path).  ``kmer_split_step`` on a ``DevicePipeline`` is the split with a
replicated start (every rank holds the whole batch and keys every window, keeping its bins): the
C ABI's multi-GPU context runs that flow.  Config 5 (bounded-memory row passes) keeps the row split:
its Σ C(df,2) ≈ 10^10-10^11 pair keys would cross the links, far more than recomputing the grouping.

The collectives only move tensors, so the same code runs on gloo with CPU tensors and stand-in
stages in the multi-process CPU tests (tests/test_dist.py).
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
        self.kcap = 0  # sharded start: key-region size (u64 words per destination)
        self.kbufs = None  # ... its send and receive buffers
        self.reruns = 0
        self.rerun_flags = []  # the reduced flags of each rerun (diagnostics)
        self.full = None  # residue start: the whole batch rebuilt on this rank (a DevicePipeline)
        self.spans = None  # ... and every rank's residue range


def _pipe_state(pipe) -> SplitState:
    """The pipe's cached SplitState, reset when its batch or k changed (a k that spills frequent
    k-mers must not pin the row split, or its capacities, on another k of the same batch)."""
    key = (pipe.n, pipe.total, pipe.k, pipe.res.data_ptr() if hasattr(pipe, "res") else 0,
           getattr(pipe, "parts", 0))
    st = pipe.__dict__.get("_split_state")
    if st is None or st.key != key:
        st = SplitState(key)
        pipe.__dict__["_split_state"] = st
    return st


def kmer_split_step(pipe, rank: int, world: int, group=None, min_shared: int = 1, require_class_diff: bool = True,
                    gather: bool = False, state: SplitState | None = None, timings: list | None = None,
                    class_fallback: bool = True) -> int | None:
    """One multi-GPU step of the k-mer split: expand this rank's k-mers, exchange the pair keys by
    row owner (all-to-all), reduce this rank's rows.  Every rank ends holding the canonical edges
    of its row range in pipe.ep/eq/ew (rank order = canonical order) and returns their count; with
    gather, rank 0 also receives every rank's block behind its own and returns the total.  A batch
    that spills frequent k-mers reruns with the heavy path on (KMP_SPLIT_HEAVY in the reduced flags);
    one whose class ids overflow the key falls back to the row split (distributed_step).  timings: a
    list to append this rank's (expand, exchange, edges) milliseconds to (CUDA events on the
    current stream, which the library's stages and the collectives are ordered with).
    class_fallback=False: a batch whose class ids overflow the key sets state.row_split and returns
    None instead of running the row split here (the caller's start runs it over its own batch)."""
    st = state if state is not None else _pipe_state(pipe)
    lo, hi = row_ranges(pipe.n, world)[rank]
    if st.row_split:
        if gather:
            return distributed_step(pipe, rank, world, group, min_shared, require_class_diff)
        return pipe.rows(lo, hi, min_shared=min_shared, require_class_diff=require_class_diff)
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
            if not class_fallback:
                return None
            return distributed_step(pipe, rank, world, group, min_shared, require_class_diff) if gather else \
                pipe.rows(lo, hi, min_shared=min_shared, require_class_diff=require_class_diff)
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


# the sharded start's first exchange: keys (all-to-all of 8-B window keys, each rank keys only its
# own windows) from this many ranks up, residues (all-gather of the 1-B residue slices, then every
# rank keys every window and keeps its bins) below.  Bytes per rank at config 4: keys 66.7 / 50.3
# / 30.1 MB (G = 2 / 4 / 8, padded regions) against residues 15.0 / 22.5 / 26.3 MB; the residue
# start re-keys the whole batch (~0.09 ms per rank) where the key start keys 1/G of it
KEYS_START_MIN_WORLD = 8


def start_mode(start: str, world: int) -> str:
    """'keys' or 'residues' for sharded_split_step's `start` ('auto' picks by world size)."""
    if start == "auto":
        return "keys" if world >= KEYS_START_MIN_WORLD else "residues"
    if start not in ("keys", "residues"):
        raise ValueError(f"unknown sharded start {start!r}")
    return start


def residue_spans(pipe, group=None) -> list:
    """[(lo, hi)] per rank: the residue ranges the ranks contribute (own_residues), all-gathered."""
    world = dist.get_world_size(group)
    lo, hi, own = pipe.own_residues()
    spans = torch.zeros(2 * world, dtype=torch.int64, device=own.device)
    dist.all_gather_into_tensor(spans, torch.tensor([lo, hi], dtype=torch.int64, device=own.device), group=group)
    return [tuple(x) for x in spans.view(world, 2).tolist()]


def gather_residues_into(pipe, dst: torch.Tensor, spans: list, group=None) -> None:
    """The packed batch in dst on every rank: this rank's slice copied in, every other rank's slice
    received straight into its place (point-to-point over xGMI on RCCL; no staging buffer)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi, own = pipe.own_residues()
    if hi > lo:
        dst[lo:hi].copy_(own)
    ops = []
    for r in range(world):
        if r == rank:
            continue
        if hi > lo:
            ops.append(dist.P2POp(dist.isend, dst[lo:hi], r, group=group))
        l, h = spans[r]
        if h > l:
            ops.append(dist.P2POp(dist.irecv, dst[l:h], r, group=group))
    for w in (dist.batch_isend_irecv(ops) if ops else []):
        w.wait()


def gather_residues(pipe, group=None):
    """The whole packed batch on every rank, from the ranks' slices (an all-gather over RCCL): the
    row-split fallback of the sharded start.  Bytes no rank holds belong to proteins with fewer than
    k residues, which have no window and so no edge; they stay zero."""
    world = dist.get_world_size(group)
    lo, hi, own = pipe.own_residues()
    dev = own.device
    spans = torch.zeros(2 * world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(spans, torch.tensor([lo, hi], dtype=torch.int64, device=dev), group=group)
    sp = spans.view(world, 2).tolist()
    width = max(1, max(h - l for l, h in sp))
    buf = torch.zeros(width, dtype=torch.uint8, device=dev)
    buf[:hi - lo] = own
    allb = torch.empty(world * width, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(allb, buf, group=group)
    res = torch.zeros(max(1, pipe.total), dtype=torch.uint8, device=dev)
    for r, (l, h) in enumerate(sp):
        if h > l:
            res[l:h] = allb[r * width:r * width + (h - l)]
    return res[:pipe.total]


def _row_split_from_shards(pipe, rank, world, group, min_shared, require_class_diff, gather, st):
    """The row split over the rebuilt batch (class ids too wide for the k-mer split's key)."""
    if st.full is None:
        st.full = pipe.gathered_pipeline(gather_residues(pipe, group))
    full = st.full
    if gather:
        m = distributed_step(full, rank, world, group, min_shared, require_class_diff)
    else:
        lo, hi = row_ranges(full.n, world)[rank]
        m = full.rows(lo, hi, min_shared=min_shared, require_class_diff=require_class_diff)
    pipe.ep, pipe.eq, pipe.ew, pipe.n_edges = full.ep, full.eq, full.ew, full.n_edges
    return m


def _residue_start(pipe, rank, world, group, min_shared, require_class_diff, st, timings, gather):
    """The sharded start through the residues: the ranks' slices all-gathered into a whole batch
    (built once per batch, refreshed in place every step), then the k-mer split with every rank
    keying every window (kmer_split_step).  The rank's edges end in pipe.ep/eq/ew; with gather,
    rank 0's hold every rank's block and it returns the total.  Class ids too wide for the key:
    the row split over the same rebuilt batch (once: the split's own fallback is not taken, so no
    rank's block is gathered twice)."""
    cuda = pipe.dev.type == "cuda"
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)] if timings is not None and cuda else None
    if ev:
        ev[0].record()
    if st.full is None:
        st.spans = residue_spans(pipe, group)
        st.full = pipe.gathered_pipeline(gather_residues(pipe, group))
    else:
        gather_residues_into(pipe, st.full.res, st.spans, group)
    if ev:
        ev[1].record()
    inner = [] if timings is not None else None
    # the same SplitState: the pair-key capacity, reruns and fallback are the step's
    m = kmer_split_step(st.full, rank, world, group, min_shared, require_class_diff, state=st, timings=inner,
                        class_fallback=False)
    if m is None:  # class ids too wide (st.row_split is set)
        return _row_split_from_shards(pipe, rank, world, group, min_shared, require_class_diff, gather, st)
    full = st.full
    pipe.ep, pipe.eq, pipe.ew, pipe.n_edges = full.ep, full.eq, full.ew, m
    pipe.edge_cap = full.edge_cap
    if timings is not None and inner:
        gx = ev[0].elapsed_time(ev[1]) if ev else 0.0
        timings.append((0.0, gx) + tuple(inner[-1]))
    if not gather:
        return m
    return _gather_to_rank0(pipe, m, rank, world, group)


def sharded_split_step(pipe, rank: int, world: int, group=None, min_shared: int = 1,
                       require_class_diff: bool = True, gather: bool = False, state: SplitState | None = None,
                       timings: list | None = None, start: str = "auto") -> int:
    """One multi-GPU step of the k-mer split with a sharded start (module docstring): keys, key
    all-to-all, group + expand, pair-key all-to-all, edges.  Every rank ends holding the canonical
    edges of its row range in pipe.ep/eq/ew and returns their count; with gather, rank 0 also
    receives every rank's block behind its own and returns the total.  start: 'keys' (the key
    all-to-all), 'residues' (all-gather of the residue slices, then every rank keys the batch) or
    'auto' (keys from KEYS_START_MIN_WORLD ranks up).  timings: a list to append this rank's
    (keys, start exchange, group, pair exchange, edges) milliseconds to (CUDA events on the current
    stream, which the library's stages and the collectives are ordered with; the residue start's
    keys are 0 and its group is the whole expand)."""
    st = state if state is not None else _pipe_state(pipe)
    if st.row_split:
        return _row_split_from_shards(pipe, rank, world, group, min_shared, require_class_diff, gather, st)
    if world > 1 and start_mode(start, world) == "residues":
        return _residue_start(pipe, rank, world, group, min_shared, require_class_diff, st, timings, gather)
    lo, hi = row_ranges(pipe.n, world)[rank]
    dev = pipe.dev
    cuda = dev.type == "cuda"
    if st.kcap == 0:
        st.kcap = int(pipe.span.key_cap)
    if st.cap == 0:  # expected pair keys per (source, destination): a quarter of the windows / world^2
        st.cap = max(4096, int(pipe.total // 4 // (world * world)))
    m = 0
    for _ in range(8):
        if st.kbufs is None or st.kbufs[0].numel() != world * st.kcap:
            st.kbufs = (torch.empty(world * st.kcap, dtype=torch.int64, device=dev),
                        torch.empty(world * st.kcap, dtype=torch.int64, device=dev))
        if st.bufs is None or st.bufs[0].numel() != world * st.cap:
            st.bufs = (torch.empty(world * st.cap, dtype=torch.int64, device=dev),
                       torch.empty(world * st.cap, dtype=torch.int64, device=dev),
                       torch.zeros(_lib.KMP_SPLIT_FLAGS, dtype=torch.int32, device=dev),
                       torch.zeros(8, dtype=torch.int64, device=dev))
        ksend, krecv = st.kbufs
        send, recv, flags, stats = st.bufs
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)] if timings is not None else None
        if ev:
            ev[0].record()
        pipe.split_keys(rank, world, st.kcap, ksend, flags)
        if ev:
            ev[1].record()
        if world > 1:
            dist.all_to_all_single(krecv, ksend, group=group)
        else:
            krecv = ksend
        if ev:
            ev[2].record()
        pipe.split_group(krecv, st.kcap, rank, world, st.cap, send, flags, stats, learn=st.learn,
                         require_class_diff=require_class_diff)
        if ev:
            ev[3].record()
        if world > 1:
            dist.all_to_all_single(recv, send, group=group)
            dist.all_reduce(flags, op=dist.ReduceOp.MAX, group=group)
        else:
            recv = send
        # the reduced flags go to the host behind the collectives on the same stream, with an event
        # behind the copy (split_edges synchronises the stream anyway: no read-back of its own)
        if st.host_flags is None or st.host_flags.numel() != flags.numel():
            st.host_flags = torch.empty(flags.shape, dtype=flags.dtype, pin_memory=cuda)
        st.host_flags.copy_(flags, non_blocking=cuda)
        copied = torch.cuda.Event() if cuda else None
        if copied is not None:
            copied.record()
        if ev:
            ev[4].record()
        m = pipe.split_edges(recv, lo, hi, min_shared)
        if ev:
            ev[5].record()
        if copied is not None:
            copied.synchronize()
        fl = [int(x) for x in st.host_flags.tolist()]
        if fl[_lib.KMP_SPLIT_CLASS]:
            st.row_split = True
            return _row_split_from_shards(pipe, rank, world, group, min_shared, require_class_diff, gather, st)
        if fl[_lib.KMP_SPLIT_RERUN] or fl[_lib.KMP_SPLIT_HEAVY]:  # HEAVY: the heavy path on every rank
            st.reruns += 1
            st.rerun_flags.append(fl)
            st.learn = fl
            if fl[_lib.KMP_SPLIT_MAX_PART] > st.cap:
                st.cap = fl[_lib.KMP_SPLIT_MAX_PART] + fl[_lib.KMP_SPLIT_MAX_PART] // 16 + 1024
            if fl[_lib.KMP_SPLIT_MAX_KEYS] > st.kcap:
                st.kcap = fl[_lib.KMP_SPLIT_MAX_KEYS] + fl[_lib.KMP_SPLIT_MAX_KEYS] // 32 + 1024
            continue
        st.learn = None
        if ev:
            torch.cuda.synchronize()
            timings.append(tuple(ev[i].elapsed_time(ev[i + 1]) for i in range(5)))
        break
    else:
        raise RuntimeError("k-mer split: capacities unstable across reruns")
    if not gather or world == 1:
        return m
    return _gather_to_rank0(pipe, m, rank, world, group)


def _gather_to_rank0(pipe, m, rank, world, group):
    """gather_rows of the rank's m edges onto rank 0 (which grows its arrays when they are short)."""

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
