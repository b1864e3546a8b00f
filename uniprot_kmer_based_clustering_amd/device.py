"""Device-resident pipeline over the kmp_dev_* stages (include/kmerpair.h).

PyTorch is plumbing here: it owns the HBM buffers and the stream; every byte of k-mer work
runs in libkmerpair's HIP kernels.  One ``DevicePipeline`` holds one protein batch resident
on one GPU and runs the reference's hot path as stages:

  build_sets   Protein::new + per-protein sort/dedup      (protein.rs:107-132, main.rs:99-101,187-189)
  filter       remove_unique_five_mers (df >= 2)           (protein.rs:151-162, main.rs:127-149)
  plan         dense CSR of the filtered sets, column blocks, row tiles (host, from set sizes)
  pairs        Graph::new + remove_uninteresting_edges + combine_edges (graph/mod.rs)
  sort         canonical (p, q) order

A multi-GPU host (dist.py) runs build_sets on a protein slice, all-gathers the sets over RCCL
and runs ``pairs`` on its share of the work items.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from ._lib import check, lib
from .engine import Proteins

CHUNK_COST = 0  # column k-mers per work item (0: the library default, one L2-shared chunk)


def _np(a: np.ndarray):
    return None if a.size == 0 else C.c_void_p(a.ctypes.data)


def _p(t: torch.Tensor | None):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream() -> C.c_void_p:
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


class Plan:
    """Host plan of the pair kernel (kmp_plan_pairs): dense CSR offsets of the filtered sets
    and the chunk-major work items (row tile x column chunk)."""

    def __init__(self, set_len: np.ndarray, chunk_cost: int = CHUNK_COST):
        L = lib()
        lens = np.ascontiguousarray(set_len, dtype=np.uint32)
        n = len(lens)
        self.dense_off = np.zeros(n + 1, dtype=np.uint64)
        ni = C.c_uint64()
        st = L.kmp_plan_pairs(_np(lens), n, chunk_cost, _np(self.dense_off), None, 0, C.byref(ni))
        if st not in (_lib.KMP_OK, _lib.KMP_EOVERFLOW):
            check(st, "kmp_plan_pairs")
        items = np.zeros((max(1, ni.value), 4), dtype=np.uint32)
        check(L.kmp_plan_pairs(_np(lens), n, chunk_cost, _np(self.dense_off), _np(items), ni.value,
                               C.byref(ni)), "kmp_plan_pairs")
        self.items = items[:ni.value]
        self.set_len = lens

    def item_costs(self) -> np.ndarray:
        """Estimated cost per item: column k-mers streamed + row k-mers inserted + a fixed
        per-item start-up."""
        if len(self.items) == 0:
            return np.zeros(0)
        d = self.dense_off.astype(np.int64)
        it = self.items.astype(np.int64)
        return (d[it[:, 3]] - d[np.maximum(it[:, 2], it[:, 0] + 1)]) + (d[it[:, 1]] - d[it[:, 0]]) + 4096

    def share(self, rank: int, world: int) -> np.ndarray:
        """Contiguous, cost-balanced share of the chunk-major items for `rank` of `world`."""
        if world <= 1 or len(self.items) == 0:
            return self.items if rank == 0 else self.items[:0]
        cum = np.cumsum(self.item_costs())
        cuts = np.searchsorted(cum, cum[-1] * np.arange(1, world) / world)
        return np.split(self.items, cuts)[rank]


def order_xcd(items: np.ndarray) -> np.ndarray:
    """XCD-aware launch order (kmp_order_items_xcd); may add empty padding items."""
    L = lib()
    items = np.ascontiguousarray(items, dtype=np.uint32).reshape(-1, 4)
    n = C.c_uint64()
    L.kmp_order_items_xcd(_np(items), len(items), None, 0, C.byref(n))
    out = np.zeros((max(1, n.value), 4), dtype=np.uint32)
    check(L.kmp_order_items_xcd(_np(items), len(items), _np(out), n.value, C.byref(n)),
          "kmp_order_items_xcd")
    return out[:n.value]


class _SplitEdges:
    """The stages the two multi-GPU pipelines share: the workspace, the edge arrays and the k-mer
    split's edges phase (kmp_dev_split_edges)."""

    def _workspace(self):
        if self._postings is None:
            ws = C.c_void_p()
            check(lib().kmp_postings_create(C.byref(ws)), "kmp_postings_create")
            self._postings = ws
        return self._postings

    def _alloc_edges(self, cap):
        self.edge_cap = cap
        self.ep = torch.empty(cap, dtype=torch.int32, device=self.dev)
        self.eq = torch.empty(cap, dtype=torch.int32, device=self.dev)
        self.ew = torch.empty(cap, dtype=torch.int32, device=self.dev)

    def split_edges(self, recv: torch.Tensor, row_lo: int, row_hi: int, min_shared: int = 1) -> int:
        """Multi-GPU k-mer split, last phase (kmp_dev_split_edges): the received pair keys -> the
        canonical edges of rows [row_lo, row_hi) in ep/eq/ew (syncs)."""
        for _ in range(2):
            ne = C.c_uint64()
            st = lib().kmp_dev_split_edges(self._workspace(), _p(recv), recv.numel(), self.n, row_lo, row_hi,
                                           min_shared, _p(self.ep), _p(self.eq), _p(self.ew), self.edge_cap,
                                           C.byref(ne), _stream())
            if st == _lib.KMP_EOVERFLOW:
                self._alloc_edges(ne.value + ne.value // 8 + 1024)
                continue
            check(st, "kmp_dev_split_edges")
            self.n_edges = ne.value
            return self.n_edges
        raise RuntimeError("edge count unstable across reruns")

    def last_layout(self) -> str:
        """Layout of the last postings call: 'bucketed' (LDS group + expand per hash bucket,
        frequent k-mers on the heavy path) or 'flat' (the fallback for very wide class ids)."""
        return "flat" if lib().kmp_postings_last_layout(self._workspace()) == _lib.KMP_LAYOUT_FLAT else "bucketed"

    def last_heavy(self) -> bool:
        """Whether the last call spilled frequent k-mers (df > 128) to the heavy path."""
        return lib().kmp_postings_last_layout(self._workspace()) == _lib.KMP_LAYOUT_BUCKETED_HEAVY

    def last_tail(self) -> str:
        """How the last postings call reduced its pair keys: 'fast' (fixed row-block regions, LDS
        hash-aggregate + rank, edges written at look-back offsets), 'rows' (the counting row-block
        tail: histogram, scan, scatter, block sort, emit) or 'sort' (global pair-key sort, flat
        layout)."""
        if self.last_layout() == "flat":
            return "sort"
        return "fast" if lib().kmp_postings_last_tail(self._workspace()) == _lib.KMP_TAIL_FAST else "rows"

    def overflow_blocks(self) -> int:
        """Row blocks of the last call above the LDS capacity (finished by the segmented sort)."""
        return int(lib().kmp_postings_last_overflow_blocks(self._workspace()))

    def reruns(self) -> int:
        """Calls of this pipeline's workspace run again after a learned capacity grew."""
        return int(lib().kmp_postings_reruns(self._workspace()))

    def edges(self):
        n = self.n_edges
        return (self.ep[:n].cpu().numpy().view(np.uint32), self.eq[:n].cpu().numpy().view(np.uint32),
                self.ew[:n].cpu().numpy().view(np.uint32))

    def __del__(self):
        if getattr(self, "_postings", None) is not None:
            try:
                lib().kmp_postings_destroy(self._postings)
            except Exception:
                pass
            self._postings = None


class ShardPipeline(_SplitEdges):
    """One rank of the multi-GPU k-mer split with a SHARDED START: this GPU
    holds the batch's offsets and class ids (metadata: 10 B per protein) and only the residues its
    own 4,096-slot chunks read (kmp_split_plan: about 1/parts of the packed residues).  A step:
      split_keys    the rank's windows keyed once, each key sent toward the rank owning its coarse
                    bin (no rank keys another rank's windows);
      (all-to-all of the key regions over RCCL)
      split_group   the received keys of the rank's bins grouped and expanded, pair keys routed to
                    their row owners;
      (all-to-all of the pair keys, max-reduce of the flags)
      split_edges   the rank's rows reduced to canonical edges.
    `residues` is a host copy of the packed batch (the bench generates it whole); only the rank's
    slice is copied to the device."""

    def __init__(self, residues: np.ndarray, offsets: np.ndarray, class_id: np.ndarray, k: int, part: int,
                 parts: int, device: torch.device | str = "cuda", edge_cap: int | None = None):
        self.k = k
        self.part, self.parts = part, parts
        self.dev = torch.device(device)
        self.offsets_host = np.ascontiguousarray(offsets, dtype=np.uint64)
        self.n = len(self.offsets_host) - 1
        self.total = int(self.offsets_host[-1])
        self.span = _lib.split_plan(self.offsets_host, k, part, parts)
        lo, hi = int(self.span.res_lo), int(self.span.res_hi)
        self.res_lo, self.res_hi = lo, hi
        sl = np.ascontiguousarray(np.asarray(residues, dtype=np.uint8)[lo:hi])
        self.res = torch.from_numpy(sl if sl.size else np.zeros(16, dtype=np.uint8)).to(self.dev)
        self.off = torch.from_numpy(self.offsets_host.view(np.int64)).to(self.dev)
        cls = np.ascontiguousarray(class_id, dtype=np.uint16)
        self.cls = torch.from_numpy((cls if cls.size else np.zeros(1, np.uint16)).view(np.int16)).to(self.dev)
        self._postings = None
        self._alloc_edges(edge_cap or max(1 << 20, 4 * self.n // max(1, parts)))
        self.n_edges = 0

    def split_keys(self, part: int, parts: int, kcap: int, ksend: torch.Tensor, flags: torch.Tensor) -> None:
        """kmp_dev_split_keys: this rank's windows keyed, region d of ksend (kcap int64 words) bound
        for rank d; flags (int32[KMP_SPLIT_FLAGS]) on the stream.  No host synchronisation."""
        assert (part, parts) == (self.part, self.parts), "the slice was planned for another split"
        check(lib().kmp_dev_split_keys(self._workspace(), _p(self.res), self.res_lo, self.res_hi, _p(self.off),
                                       _p(self.cls), self.n, self.k, int(self.span.slots), part, parts, kcap,
                                       _p(ksend), _p(flags), _stream()), "kmp_dev_split_keys")

    def split_group(self, krecv: torch.Tensor, kcap: int, part: int, parts: int, cap: int, send: torch.Tensor,
                    flags: torch.Tensor, stats: torch.Tensor, learn=None, require_class_diff: bool = True,
                    heavy_df: int = 0xFFFFFFFF) -> None:
        """kmp_dev_split_group: the received keys (parts regions of kcap words) of this rank's bins
        grouped and expanded, pair keys routed to their row owners in `send` (parts regions of cap);
        its flags merged into `flags` (the keys phase's, same step), stats (int64[8])."""
        lp = None if learn is None else (C.c_uint32 * _lib.KMP_SPLIT_FLAGS)(*[int(x) for x in learn])
        check(lib().kmp_dev_split_group(self._workspace(), _p(krecv), kcap, self.n, self.k, int(self.span.slots),
                                        heavy_df, int(require_class_diff), part, parts, cap, lp, _p(send),
                                        _p(flags), _p(stats), _stream()), "kmp_dev_split_group")

    def gathered_pipeline(self, residues: torch.Tensor) -> "DevicePipeline":
        """A DevicePipeline over the whole batch rebuilt from every rank's slice (the residue start
        and the row-split fallback of dist.sharded_split_step); built once per batch, its residues
        refreshed in place afterwards."""
        from .engine import Proteins
        cls = self.cls.cpu().numpy().view(np.uint16)[:self.n]
        return DevicePipeline(Proteins(residues.cpu().numpy(), self.offsets_host, cls), self.k, self.dev)

    def own_residues(self):
        """(lo, hi, tensor): the residues this rank contributes when the batch is rebuilt on every
        rank (the residue start and the row-split fallback): [res_lo, the res_lo of the next rank
        that holds chunks) within its slice.  With fewer chunks than ranks some ranks hold none
        (kmp_split_plan reports an empty span for them) and contribute nothing; the rank before
        them contributes up to the next rank that does."""
        if self.res_hi <= self.res_lo:
            return self.res_lo, self.res_lo, self.res[:0]
        nxt = self.total
        for d in range(self.part + 1, self.parts):
            sp = _lib.split_plan(self.offsets_host, self.k, d, self.parts)
            if int(sp.res_hi) > int(sp.res_lo):
                nxt = int(sp.res_lo)
                break
        hi = max(self.res_lo, min(nxt, self.res_hi))
        return self.res_lo, hi, self.res[:hi - self.res_lo]


class DevicePipeline(_SplitEdges):
    def __init__(self, proteins: Proteins, k: int, device: torch.device | str = "cuda",
                 edge_cap: int | None = None):
        self.k = k
        self.dev = torch.device(device)
        self.n = proteins.n
        self.offsets_host = np.ascontiguousarray(proteins.offsets, dtype=np.uint64)
        self.total = int(self.offsets_host[-1])
        lens = np.diff(self.offsets_host.astype(np.int64))
        self.max_len = int(lens.max()) if self.n else 0
        L = lib()
        dev = self.dev
        self.res = torch.from_numpy(np.ascontiguousarray(proteins.residues, dtype=np.uint8)).to(dev)
        self.off = torch.from_numpy(self.offsets_host.view(np.int64)).to(dev)
        self.cls = torch.from_numpy(np.ascontiguousarray(proteins.class_id, dtype=np.uint16).view(np.int16)).to(dev)
        cap = int(L.kmp_set_capacity(self.n, self.total))
        self.set = torch.empty(cap, dtype=torch.int32, device=dev)
        self.rep = torch.empty(cap, dtype=torch.int32, device=dev)
        self.set_len = torch.zeros(max(1, self.n), dtype=torch.int32, device=dev)
        self.rep_len = torch.zeros(max(1, self.n), dtype=torch.int32, device=dev)
        words = int(L.kmp_dev_repeat_bitmap_words(k))
        self.bits = torch.empty(2 * words, dtype=torch.int32, device=dev)
        long_path = self.max_len - k + 1 > _lib.KMP_LDS_SORT_MAX
        self.scratch = torch.empty(cap, dtype=torch.int32, device=dev) if long_path else None
        self.edge_cap = edge_cap or max(1 << 20, 4 * self.n)
        self._alloc_edges(self.edge_cap)
        self.count = torch.zeros(1, dtype=torch.int64, device=dev)
        self.items = None
        self.n_items = 0
        self.dense = None
        self.plan_host = None
        self._sort_tmp = None
        self.n_long = 0
        self.long_ids = None
        self.long_rank = None
        self._postings = None
        self.postings_stats = _lib.PostingsStats()

    # -- stages ---------------------------------------------------------------------
    def build_sets(self, lo: int = 0, hi: int | None = None) -> None:
        """K(p) for proteins [lo, hi) (all by default)."""
        hi = self.n if hi is None else hi
        if hi <= lo:
            return
        check(lib().kmp_dev_build_sets(_p(self.res), C.c_void_p(self.off.data_ptr() + 8 * lo), hi - lo, self.k,
                                       self.max_len, _sub(self.set, lo), _p(self.set_len[lo:]),
                                       _sub(self.scratch, lo), _stream()), "kmp_dev_build_sets")

    def filter(self) -> None:
        check(lib().kmp_dev_filter_repeats(_p(self.set), _p(self.set_len), _p(self.off), self.n, self.k,
                                           _p(self.bits), _p(self.rep), _p(self.rep_len), _stream()),
              "kmp_dev_filter_repeats")

    def plan(self, rank: int = 0, world: int = 1, chunk_cost: int = CHUNK_COST) -> Plan:
        """Host plan from the filtered set sizes (one D2H of N u32), then the dense CSR pack."""
        rep_len = self.rep_len[:self.n].cpu().numpy().view(np.uint32)
        tile_cap = _lib.geometry().tile_cap
        long_ids = np.flatnonzero(rep_len > tile_cap).astype(np.uint32)
        plan_len = np.where(rep_len > tile_cap, 0, rep_len).astype(np.uint32)
        plan = Plan(plan_len, chunk_cost)
        self.col_window = int(lib().kmp_pair_col_window(_np(plan_len), len(plan_len)))
        mine = order_xcd(plan.share(rank, world))
        self.long_rank = rank == world - 1  # the (rare) long-protein pairs run on one rank
        dev = self.dev
        self.dense_off = torch.from_numpy(plan.dense_off.view(np.int64)).to(dev)
        self.n_items = len(mine)
        self.items = (torch.from_numpy(np.ascontiguousarray(mine).view(np.int32).reshape(-1)).to(dev)
                      if len(mine) else None)
        total = int(plan.dense_off[-1])
        if self.dense is None or self.dense.numel() < max(1, total):
            self.dense = torch.empty(max(1, total), dtype=torch.int32, device=dev)
        check(lib().kmp_dev_pack_dense(_p(self.rep), _p(self.off), _p(self.dense_off), self.n, _p(self.dense),
                                       _stream()), "kmp_dev_pack_dense")
        self.long_ids = torch.from_numpy(long_ids.view(np.int32)).to(dev) if len(long_ids) else None
        self.n_long = len(long_ids)
        self.plan_host = plan
        self.rep_len_host = rep_len
        return plan

    def pairs(self, min_shared: int = 1, require_class_diff: bool = True) -> int:
        """Runs the pair kernel over the planned items; returns the edge count (syncs)."""
        for _ in range(2):
            self.count.zero_()
            check(lib().kmp_dev_pairs(_p(self.dense), _p(self.dense_off), _p(self.cls), self.n, _p(self.items),
                                      self.n_items, self.col_window, min_shared, int(require_class_diff), _p(self.ep), _p(self.eq),
                                      _p(self.ew), self.edge_cap, _p(self.count), _stream()), "kmp_dev_pairs")
            if self.n_long and (self.long_rank is None or self.long_rank):
                check(lib().kmp_dev_pairs_long(_p(self.rep), _p(self.rep_len), _p(self.off), _p(self.cls), self.n,
                                               _p(self.long_ids), self.n_long, min_shared, int(require_class_diff),
                                               _p(self.ep), _p(self.eq), _p(self.ew), self.edge_cap, _p(self.count),
                                               _stream()), "kmp_dev_pairs_long")
            cnt = int(self.count.item())
            if cnt <= self.edge_cap:
                self.n_edges = cnt
                return cnt
            self._alloc_edges(cnt + cnt // 8 + 1024)
        raise RuntimeError("edge count unstable across reruns")

    def sort(self, n_edges: int | None = None) -> None:
        n = self.n_edges if n_edges is None else n_edges
        if n == 0:
            return
        L = lib()
        nbytes = int(L.kmp_dev_sort_edges_tmp_bytes(n, self.n))
        if self._sort_tmp is None or self._sort_tmp.numel() < nbytes:
            self._sort_tmp = torch.empty(nbytes + 256, dtype=torch.uint8, device=self.dev)
        check(L.kmp_dev_sort_edges(_p(self.ep), _p(self.eq), _p(self.ew), n, self.n, _p(self._sort_tmp),
                                   self._sort_tmp.numel(), _stream()), "kmp_dev_sort_edges")

    def set_stage_timing(self, enable: bool = True) -> None:
        """Per-stage HIP-event times of the postings engine into postings_stats.stage_ms."""
        check(lib().kmp_postings_set_timing(self._workspace(), int(enable)), "kmp_postings_set_timing")

    def set_layout(self, bucketed: bool = True) -> None:
        """Postings key layout: bucketed (LDS group + expand per hash bucket) or flat."""
        check(lib().kmp_postings_set_layout(self._workspace(), int(bucketed)), "kmp_postings_set_layout")

    def set_graph(self, enable: bool = True) -> None:
        """Residue path: capture the single-synchronisation step as a HIP graph and replay it."""
        check(lib().kmp_postings_set_graph(self._workspace(), int(enable)), "kmp_postings_set_graph")

    def set_reuse(self, enable: bool = True) -> None:
        """Keep the batch's keys / grouping / heavy compaction across calls on the same batch
        (the row passes of one step): kmp_postings_set_reuse."""
        check(lib().kmp_postings_set_reuse(self._workspace(), int(enable)), "kmp_postings_set_reuse")

    def set_partition(self, mode: str = "auto") -> None:
        """Residue path's bucket partition: 'auto' (cursor partition, the counting partition for a
        shape whose regions overflow) or 'count' (the counting partition only)."""
        m = {"auto": _lib.KMP_PARTITION_AUTO, "count": _lib.KMP_PARTITION_COUNT}[mode]
        check(lib().kmp_postings_set_partition(self._workspace(), m), "kmp_postings_set_partition")

    def last_partition(self) -> str:
        """Partition of the last bucketed call: 'cursor' or 'count' ('' on the flat layout)."""
        r = lib().kmp_postings_last_partition(self._workspace())
        return {_lib.KMP_PARTITION_CURSOR: "cursor", _lib.KMP_PARTITION_COUNT: "count"}.get(r, "")

    def graph_replays(self) -> int:
        return int(lib().kmp_postings_graph_replays(self._workspace()))


    def set_tail(self, mode: str = "fast") -> None:
        """Row-block tail of unscored calls: 'fast' (default, where it applies) or 'count'."""
        m = {"fast": _lib.KMP_TAIL_FAST, "count": _lib.KMP_TAIL_COUNT}[mode]
        check(lib().kmp_postings_set_tail(self._workspace(), m), "kmp_postings_set_tail")

    def rows(self, row_lo: int, row_hi: int, min_shared: int = 1, require_class_diff: bool = True,
             heavy_df: int = 0xFFFFFFFF) -> int:
        """Edges of rows [row_lo, row_hi) only (kmp_dev_pairs_rows), canonical, into ep/eq/ew."""
        ws = self._workspace()
        slots = int(lib().kmp_set_capacity(self.n, self.total))
        for _ in range(2):
            ne = C.c_uint64()
            st = lib().kmp_dev_pairs_rows(ws, _p(self.res), _p(self.off), _p(self.cls), self.n, self.k, slots,
                                          heavy_df, min_shared, int(require_class_diff), row_lo, row_hi,
                                          _p(self.ep), _p(self.eq), _p(self.ew), self.edge_cap, C.byref(ne),
                                          C.byref(self.postings_stats), _stream())
            if st == _lib.KMP_EOVERFLOW:
                self._alloc_edges(ne.value + ne.value // 8 + 1024)
                continue
            check(st, "kmp_dev_pairs_rows")
            self.n_edges = ne.value
            return self.n_edges
        raise RuntimeError("edge count unstable across reruns")

    def split_expand(self, part: int, parts: int, cap: int, send: torch.Tensor, flags: torch.Tensor,
                     stats: torch.Tensor, learn=None, require_class_diff: bool = True,
                     heavy_df: int = 0xFFFFFFFF) -> None:
        """Multi-GPU k-mer split, phase 1 (kmp_dev_split_expand): this rank's share of the k-mers
        grouped and expanded, pair keys routed to their row owners in `send` (parts regions of cap
        keys, int64); flags (int32[KMP_SPLIT_FLAGS]) and stats (int64[8]) on the stream.  No host
        synchronisation (one with the heavy path on).  learn: the last call's flags reduced over the
        ranks (or None); HEAVY in them turns the rank's heavy path on."""
        slots = int(lib().kmp_set_capacity(self.n, self.total))
        lp = None if learn is None else (C.c_uint32 * _lib.KMP_SPLIT_FLAGS)(*[int(x) for x in learn])
        check(lib().kmp_dev_split_expand(self._workspace(), _p(self.res), _p(self.off), _p(self.cls), self.n, self.k,
                                         slots, heavy_df, int(require_class_diff), part, parts, cap, lp, _p(send),
                                         _p(flags), _p(stats), _stream()), "kmp_dev_split_expand")

    def postings(self, min_shared: int = 1, require_class_diff: bool = True,
                 heavy_df: int = 0xFFFFFFFF, from_residues: bool = False) -> int:
        """Postings engine: canonical edges into ep/eq/ew (syncs).  Reads the K(p) slots
        (after build_sets), or with from_residues the packed residues directly (fused path)."""
        ws = self._workspace()
        slots = int(lib().kmp_set_capacity(self.n, self.total))
        for _ in range(2):
            ne = C.c_uint64()
            if from_residues:
                # the argument tuple is cached while buffers, stream and options stay put (the
                # step is launch-bound: the library replays a HIP graph)
                stream = torch.cuda.current_stream().cuda_stream
                key = (self.ep.data_ptr(), self.edge_cap, stream, heavy_df, min_shared, require_class_diff, slots)
                cached = getattr(self, "_res_call", None)
                if cached is None or cached[0] != key:
                    ne_c = C.c_uint64()
                    args = (ws, _p(self.res), _p(self.off), _p(self.cls), self.n, self.k, slots, heavy_df,
                            min_shared, int(require_class_diff), _p(self.ep), _p(self.eq), _p(self.ew),
                            self.edge_cap, C.byref(ne_c), C.byref(self.postings_stats), C.c_void_p(stream))
                    cached = self._res_call = (key, args, ne_c)
                st = lib().kmp_dev_pairs_residues(*cached[1])
                ne = cached[2]
            else:
                st = lib().kmp_dev_pairs_postings(ws, _p(self.set), _p(self.set_len), _p(self.off),
                                                  _p(self.cls), self.n, self.k, slots, heavy_df, min_shared,
                                                  int(require_class_diff), _p(self.ep), _p(self.eq), _p(self.ew),
                                                  self.edge_cap, C.byref(ne), C.byref(self.postings_stats),
                                                  _stream())
            if st == _lib.KMP_EOVERFLOW:
                self._alloc_edges(ne.value + ne.value // 8 + 1024)
                continue
            check(st, "kmp_dev_pairs_postings")
            self.n_edges = ne.value
            return self.n_edges
        raise RuntimeError("edge count unstable across reruns")

    def submit(self, min_shared: int = 1, require_class_diff: bool = True, heavy_df: int = 0xFFFFFFFF) -> int:
        """kmp_dev_pairs_residues_submit: the fused residue step enqueued on the current stream (no host
        wait once its graph replays, so the next submission queues behind it); returns the ticket
        for wait().  At most two outstanding; both write ep/eq/ew (the later overwrites the earlier)."""
        ws = self._workspace()
        stream = torch.cuda.current_stream().cuda_stream
        key = (self.ep.data_ptr(), self.edge_cap, stream, heavy_df, min_shared, require_class_diff)
        cached = getattr(self, "_sub_call", None)
        if cached is None or cached[0] != key:
            t = C.c_uint64()
            slots = int(lib().kmp_set_capacity(self.n, self.total))
            args = (ws, _p(self.res), _p(self.off), _p(self.cls), self.n, self.k, slots, heavy_df, min_shared,
                    int(require_class_diff), _p(self.ep), _p(self.eq), _p(self.ew), self.edge_cap,
                    C.c_void_p(stream), C.byref(t))
            cached = self._sub_call = (key, args, t, (min_shared, require_class_diff, heavy_df))
        check(lib().kmp_dev_pairs_residues_submit(*cached[1]), "kmp_dev_pairs_residues_submit")
        return cached[2].value

    def wait(self, ticket: int) -> int:
        """kmp_postings_wait: the submitted step's edge count (its read-back checked; a step that asked
        for a rerun ran again at the wait) and its statistics in postings_stats."""
        ne = C.c_uint64()
        st = lib().kmp_postings_wait(self._workspace(), ticket, C.byref(ne), C.byref(self.postings_stats))
        if st == _lib.KMP_EOVERFLOW:  # the edge arrays were short: grown, and the step run again
            self._alloc_edges(ne.value + ne.value // 8 + 1024)
            ms, rcd, hd = self._sub_call[3]
            return self.postings(ms, rcd, hd, from_residues=True)
        check(st, "kmp_postings_wait")
        self.n_edges = ne.value
        return self.n_edges

    def step(self, min_shared: int = 1, require_class_diff: bool = True, engine: str = "residues") -> int:
        """The whole single-GPU path, packed residues in HBM -> canonical edges in HBM.
        residues: windows -> sort/expand/reduce (kmp_dev_pairs_residues, fused);
        postings: K(p) sets -> sort/expand/reduce;
        tiles: K(p) sets -> repeat filter -> plan -> tiled pair kernel -> canonical sort."""
        if engine == "residues":
            return self.postings(min_shared, require_class_diff, from_residues=True)
        self.build_sets()
        if engine == "postings":
            return self.postings(min_shared, require_class_diff)
        self.filter()
        self.plan()
        n = self.pairs(min_shared, require_class_diff)
        self.sort(n)
        return n

    def set_of(self, p: int, repeat_only: bool = False) -> np.ndarray:
        base = int(lib().kmp_set_base(int(self.offsets_host[p]), p))
        buf, ln = (self.rep, self.rep_len) if repeat_only else (self.set, self.set_len)
        m = int(ln[p].item())
        return buf[base:base + m].cpu().numpy().view(np.uint32)


def _sub(t: torch.Tensor | None, lo: int):
    """Device pointer of a per-protein slot buffer for a stage launched on proteins [lo, ...).
    The kernels compute slot(off[p], p_rel) with p_rel = p - lo; since kmp_set_base is
    round_up(off + 4p, 4) and 4*lo is a multiple of 4, slot(off, p_rel) = slot(off, p) - 4*lo,
    so the buffer pointer moves forward by 4*lo elements."""
    if t is None:
        return None
    return C.c_void_p(t.data_ptr() + 4 * 4 * lo)
