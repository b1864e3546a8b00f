"""ctypes binding of libkmerpair.so (include/kmerpair.h).

The library is built in-tree (``lib/libkmerpair.so``) by ``__graft_entry__.build()`` /
``make -C uniprot_kmer_based_clustering_amd/csrc``.  There is no fallback: if the library is
missing or fails to load, every entry point raises — the product path never substitutes a
CPU implementation.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# KMP_LIB: an alternative build of the same library (tools/_ab_kernels.sh A/B timing only)
_DEFAULT_LIB = os.path.join(HERE, "lib", "libkmerpair.so")
LIB_PATH = os.environ.get("KMP_LIB") or _DEFAULT_LIB
HEADER_PATH = os.path.join(os.path.dirname(HERE), "include", "kmerpair.h")

KMP_OK, KMP_EINVAL, KMP_ENOMEM, KMP_EDEVICE, KMP_ERCCL, KMP_EOVERFLOW, KMP_ESTATE, KMP_EIO = range(8)
KMP_LEN_NORMAL300, KMP_LEN_LOGUNIFORM = 0, 1
KMP_SCORE_COUNT, KMP_SCORE_JACCARD, KMP_SCORE_BLOSUM = 0, 1, 2
KMP_ENGINE_AUTO, KMP_ENGINE_POSTINGS, KMP_ENGINE_TILES, KMP_ENGINE_RESIDUES = 0, 1, 2, 3
KMP_KMERS_CODES, KMP_KMERS_IDS = 0, 1
KMP_LAYOUT_FLAT, KMP_LAYOUT_BUCKETED, KMP_LAYOUT_BUCKETED_HEAVY = 0, 1, 2
KMP_TAIL_COUNT, KMP_TAIL_FAST = 0, 1
KMP_PARTITION_AUTO, KMP_PARTITION_COUNT, KMP_PARTITION_CURSOR = 0, 1, 2
(KMP_SPLIT_RERUN, KMP_SPLIT_CLASS, KMP_SPLIT_HEAVY, KMP_SPLIT_MAX_PART, KMP_SPLIT_MAX_SHARD, KMP_SPLIT_BIN_TILES,
 KMP_SPLIT_CURSOR, KMP_SPLIT_MAX_KEYS, KMP_SPLIT_LARGE) = range(9)
KMP_SPLIT_FLAGS = 16
KMP_LDS_SORT_MAX = 4096


class SplitSpan(C.Structure):
    """kmp_split_span: a rank's chunk range and residue slice of the sharded k-mer split."""
    _fields_ = [("slots", C.c_uint64), ("n_chunks", C.c_uint32), ("c_lo", C.c_uint32), ("c_hi", C.c_uint32),
                ("res_lo", C.c_uint64), ("res_hi", C.c_uint64), ("key_table_words", C.c_uint64),
                ("key_cap", C.c_uint64)]


class KmpError(RuntimeError):
    def __init__(self, status: int, where: str, detail: str = ""):
        self.status = status
        msg = f"{where}: {status_string(status)} ({status})"
        if detail:
            msg += f": {detail}"
        super().__init__(msg)


class Counters(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "n_proteins", "n_windows", "sum_S", "distinct", "repeat", "sum_cdf2", "sum_w_diff",
        "n_edges", "n_align", "max_df")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class PairOpts(C.Structure):
    _fields_ = [("min_shared", C.c_uint32), ("require_class_diff", C.c_int32),
                ("align_threshold", C.c_uint32), ("score", C.c_int32), ("engine", C.c_int32)]


KMP_POSTINGS_STAGES = 6
POSTINGS_STAGE_NAMES = ("keys", "code_sort", "count", "write", "pair_sort", "rle_emit")


class PostingsStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "sum_S", "distinct", "repeat", "sum_cdf2_light", "max_df", "heavy_entries", "incidences", "pairs")] + [
        ("stage_ms", C.c_float * KMP_POSTINGS_STAGES)]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_ if n != "stage_ms"}

    def stages(self) -> dict:
        return dict(zip(POSTINGS_STAGE_NAMES, (float(x) for x in self.stage_ms)))


KMP_MULTI_K_MAX = 4
KMP_DIGEST_SEGMENTS = 64


class EdgeChunk(C.Structure):
    """kmp_edge_chunk: one streamed pass of edges (kmp_pairs_stream)."""
    _fields_ = [("rank", C.c_uint32), ("device", C.c_int), ("row_lo", C.c_uint32), ("row_hi", C.c_uint32),
                ("n", C.c_uint64), ("on_device", C.c_int),
                ("p", C.c_void_p), ("q", C.c_void_p), ("w", C.c_void_p), ("score", C.c_void_p),
                ("wk", C.c_void_p * KMP_MULTI_K_MAX)]


EDGE_SINK = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(EdgeChunk))


class StreamSummary(C.Structure):
    """kmp_stream_summary: counters and digest of a streamed edge list."""
    _fields_ = [(n, C.c_uint64) for n in ("n_edges", "sum_w", "sum_score", "n_align", "sum_w_diff", "incidences",
                                           "digest")] + [
        ("seg_edges", C.c_uint64 * KMP_DIGEST_SEGMENTS), ("seg_digest", C.c_uint64 * KMP_DIGEST_SEGMENTS),
        ("passes", C.c_uint32), ("ordered", C.c_int32), ("stage_ms", C.c_float * 4)]

    def as_dict(self):
        d = {n: int(getattr(self, n)) for n, _ in self._fields_ if not n.startswith("seg_") and n != "stage_ms"}
        d["seg_edges"] = [int(x) for x in self.seg_edges]
        d["seg_digest"] = [int(x) for x in self.seg_digest]
        d["stage_ms"] = dict(zip(("expand_k0", "expand_k1", "reduce", "summary"), (float(x) for x in self.stage_ms)))
        return d


class WorkItem(C.Structure):
    _fields_ = [("row_beg", C.c_uint32), ("row_end", C.c_uint32),
                ("col_beg", C.c_uint32), ("col_end", C.c_uint32)]


class PairGeometry(C.Structure):
    _fields_ = [("tile_slots", C.c_uint32), ("tile_cap", C.c_uint32),
                ("rows_max", C.c_uint32), ("threads", C.c_uint32)]


P = C.c_void_p
U8P = C.POINTER(C.c_uint8)
U64P = C.POINTER(C.c_uint64)

# name -> (restype, argtypes); every function declared in include/kmerpair.h
SIGNATURES = {
    "kmp_version": (C.c_int, []),
    "kmp_status_string": (C.c_char_p, [C.c_int]),
    "kmp_pair_opts_default": (None, [P]),
    "kmp_ctx_create": (C.c_int, [C.POINTER(P), C.c_int, C.c_int]),
    "kmp_ctx_destroy": (None, [P]),
    "kmp_last_error": (C.c_char_p, [P]),
    "kmp_load_proteins": (C.c_int, [P, P, P, C.c_uint32, P]),
    "kmp_extract": (C.c_int, [P, C.c_int]),
    "kmp_get_kmers": (C.c_int, [P, C.c_uint32, P, C.c_uint64, U64P]),
    "kmp_build_sets": (C.c_int, [P, C.c_int]),
    "kmp_get_set": (C.c_int, [P, C.c_uint32, P, C.c_uint64, U64P]),
    "kmp_counters_get": (C.c_int, [P, P]),
    "kmp_get_df": (C.c_int, [P, P, C.c_uint64, U64P]),
    "kmp_get_repeat_codes": (C.c_int, [P, P, C.c_uint64, U64P]),
    "kmp_get_hash_kmers": (C.c_int, [P, C.c_uint32, P, C.c_uint64, U64P]),
    "kmp_get_hash_kmers_all": (C.c_int, [P, P, C.c_uint64, P, U64P]),
    "kmp_repeat_mphf": (C.c_int, [P, C.POINTER(P)]),
    "kmp_edges_kmers": (C.c_int, [P, P, C.c_int]),
    "kmp_edges_get_kmers": (C.c_int, [P, P, P, C.c_uint64, U64P]),
    "kmp_edges_reference_keys": (C.c_int, [P, P, C.c_uint64, U64P]),
    "kmp_write_candidates": (C.c_int, [P, P, P, C.c_uint32, P, C.c_uint64, C.c_uint32, C.c_char_p, C.c_int, U64P]),
    "kmp_write_graph_debug": (C.c_int, [P, C.c_uint32, C.c_char_p, C.c_int]),
    "kmp_mphf_build": (C.c_int, [P, P, C.c_uint64, C.c_double, C.POINTER(P)]),
    "kmp_mphf_lookup": (C.c_int, [P, P, C.c_uint64, P]),
    "kmp_mphf_dev_lookup": (C.c_int, [P, P, C.c_uint64, P, P]),
    "kmp_mphf_info": (C.c_int, [P, U64P, C.POINTER(C.c_uint32), U64P, U64P]),
    "kmp_mphf_free": (None, [P]),
    "kmp_pairs": (C.c_int, [P, P, C.POINTER(P)]),
    "kmp_edges_count": (C.c_int, [P, U64P]),
    "kmp_edges_get": (C.c_int, [P, P, P, P, P, C.c_uint64, U64P]),
    "kmp_edges_free": (None, [P]),
    "kmp_set_capacity": (C.c_uint64, [C.c_uint32, C.c_uint64]),
    "kmp_set_base": (C.c_uint64, [C.c_uint64, C.c_uint32]),
    "kmp_dev_extract": (C.c_int, [P, P, C.c_uint32, C.c_int, P, P]),
    "kmp_dev_build_sets": (C.c_int, [P, P, C.c_uint32, C.c_int, C.c_uint32, P, P, P, P]),
    "kmp_dev_repeat_bitmap_words": (C.c_uint64, [C.c_int]),
    "kmp_dev_filter_repeats": (C.c_int, [P, P, P, C.c_uint32, C.c_int, P, P, P, P]),
    "kmp_pair_geometry_get": (None, [P]),
    "kmp_plan_pairs": (C.c_int, [P, C.c_uint32, C.c_uint64, P, P, C.c_uint64, U64P]),
    "kmp_order_items_xcd": (C.c_int, [P, C.c_uint64, P, C.c_uint64, U64P]),
    "kmp_dev_pack_dense": (C.c_int, [P, P, P, C.c_uint32, P, P]),
    "kmp_dev_pairs": (C.c_int, [P, P, P, C.c_uint32, P, C.c_uint64, C.c_uint32, C.c_uint32, C.c_int,
                                P, P, P, C.c_uint64, P, P]),
    "kmp_pair_col_window": (C.c_uint32, [P, C.c_uint32]),
    "kmp_dev_pairs_long": (C.c_int, [P, P, P, P, C.c_uint32, P, C.c_uint32, C.c_uint32, C.c_int,
                                     P, P, P, C.c_uint64, P, P]),
    "kmp_ctx_create_multi": (C.c_int, [C.POINTER(P), C.c_int, C.POINTER(C.c_int), C.c_int]),
    "kmp_ctx_gpus": (C.c_int, [P]),
    "kmp_ctx_set_pass_keys": (C.c_int, [P, C.c_uint64]),
    "kmp_ctx_set_direct_tail": (C.c_int, [P, C.c_int]),
    "kmp_ctx_last_tail_windows": (C.c_uint64, [P]),
    "kmp_postings_set_direct": (C.c_int, [P, C.c_int]),
    "kmp_postings_set_flat_heavy": (C.c_int, [P, C.c_int]),
    "kmp_postings_set_row_span": (C.c_int, [P, C.c_uint32, C.c_uint32]),
    "kmp_ctx_set_flat_heavy": (C.c_int, [P, C.c_int]),
    "kmp_ctx_last_passes": (C.c_uint32, [P]),
    "kmp_ctx_transport": (C.c_char_p, [P]),
    "kmp_ctx_last_split": (C.c_char_p, [P]),
    "kmp_postings_create": (C.c_int, [C.POINTER(P)]),
    "kmp_postings_destroy": (None, [P]),
    "kmp_dev_pairs_postings": (C.c_int, [P, P, P, P, P, C.c_uint32, C.c_int, C.c_uint64, C.c_uint32,
                                         C.c_uint32, C.c_int, P, P, P, C.c_uint64, U64P, P, P]),
    "kmp_postings_set_timing": (C.c_int, [P, C.c_int]),
    "kmp_postings_set_layout": (C.c_int, [P, C.c_int]),
    "kmp_postings_last_layout": (C.c_int, [P]),
    "kmp_postings_last_tail": (C.c_int, [P]),
    "kmp_postings_set_tail": (C.c_int, [P, C.c_int]),
    "kmp_pairs_multi_k": (C.c_int, [P, P, C.POINTER(C.c_int), C.c_uint32, C.POINTER(P)]),
    "kmp_edges_get_wk": (C.c_int, [P, C.c_uint32, P, C.c_uint64, C.POINTER(C.c_uint64)]),
    "kmp_postings_set_graph": (C.c_int, [P, C.c_int]),
    "kmp_postings_graph_replays": (C.c_uint64, [P]),
    "kmp_postings_reruns": (C.c_uint64, [P]),
    "kmp_postings_set_partition": (C.c_int, [P, C.c_int]),
    "kmp_postings_last_partition": (C.c_int, [P]),
    "kmp_postings_set_reuse": (C.c_int, [P, C.c_int]),
    "kmp_postings_set_shard_floor": (C.c_int, [P, C.c_uint64]),
    "kmp_dev_pairs_residues": (C.c_int, [P, P, P, P, C.c_uint32, C.c_int, C.c_uint64, C.c_uint32,
                                         C.c_uint32, C.c_int, P, P, P, C.c_uint64, U64P, P, P]),
    "kmp_dev_pairs_residues_submit": (C.c_int, [P, P, P, P, C.c_uint32, C.c_int, C.c_uint64, C.c_uint32,
                                                C.c_uint32, C.c_int, P, P, P, C.c_uint64, P, U64P]),
    "kmp_postings_wait": (C.c_int, [P, C.c_uint64, U64P, P]),
    "kmp_dev_split_expand": (C.c_int, [P, P, P, P, C.c_uint32, C.c_int, C.c_uint64, C.c_uint32, C.c_int,
                                        C.c_uint32, C.c_uint32, C.c_uint64, P, P, P, P, P]),
    "kmp_dev_split_edges": (C.c_int, [P, P, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, P, P, P,
                                       C.c_uint64, U64P, P]),
    "kmp_split_plan": (C.c_int, [P, C.c_uint32, C.c_int, C.c_uint32, C.c_uint32, C.POINTER(SplitSpan)]),
    "kmp_dev_split_keys": (C.c_int, [P, P, C.c_uint64, C.c_uint64, P, P, C.c_uint32, C.c_int, C.c_uint64,
                                      C.c_uint32, C.c_uint32, C.c_uint64, P, P, P]),
    "kmp_dev_split_group": (C.c_int, [P, P, C.c_uint64, C.c_uint32, C.c_int, C.c_uint64, C.c_uint32, C.c_int,
                                       C.c_uint32, C.c_uint32, C.c_uint64, P, P, P, P, P]),
    "kmp_dev_pairs_rows": (C.c_int, [P, P, P, P, C.c_uint32, C.c_int, C.c_uint64, C.c_uint32, C.c_uint32,
                                     C.c_int, C.c_uint32, C.c_uint32, P, P, P, C.c_uint64, U64P, P, P]),
    "kmp_row_split": (None, [C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32)]),
    "kmp_dev_rows_max": (C.c_uint32, [C.c_uint32, C.c_int]),
    "kmp_dev_pairs_rows_scored": (C.c_int, [P, P, P, P, C.c_uint32, C.c_int, C.c_uint64, C.c_uint32, C.c_uint32,
                                            C.c_int, C.c_uint32, C.c_uint32, P, P, P, P, C.c_uint64, U64P, P, P]),
    "kmp_dev_pairs_rows_multi": (C.c_int, [P, C.POINTER(C.c_int), C.c_uint32, P, P, P, C.c_uint32, C.c_uint64,
                                           C.c_uint32, C.c_int, C.c_uint32, C.c_uint32, P, P, P, P, P, P,
                                           C.c_uint64, U64P, P, P]),
    "kmp_pairs_stream": (C.c_int, [P, P, C.POINTER(C.c_int), C.c_uint32, C.c_int, EDGE_SINK, P, P]),
    "kmp_edge_digest_term": (C.c_uint64, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]),
    "kmp_ctx_set_rows": (C.c_int, [P, C.c_uint32, C.c_uint32]),
    "kmp_postings_last_overflow_blocks": (C.c_uint32, [P]),
    "kmp_dev_sort_edges_tmp_bytes": (C.c_uint64, [C.c_uint64, C.c_uint32]),
    "kmp_dev_sort_edges": (C.c_int, [P, P, P, C.c_uint64, C.c_uint32, P, C.c_uint64, P]),
    "kmp_read_fasta": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint32), C.POINTER(P), C.POINTER(P),
                                 C.POINTER(P), C.POINTER(P), U64P, C.POINTER(C.c_uint32)]),
    "kmp_read_fasta_threads": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(C.c_uint32), C.POINTER(P), C.POINTER(P),
                                         C.POINTER(P), C.POINTER(P), U64P, C.POINTER(C.c_uint32)]),
    "kmp_synth_packed": (C.c_int, [C.c_uint32, C.c_uint64, C.c_int, C.POINTER(P), P, P, P]),
    "kmp_synth_write_fasta": (C.c_int, [C.c_char_p, C.c_uint32, C.c_uint64, C.c_int]),
    "kmp_free_host": (None, [P]),
}

_lib = None


def _bind_hip_runtime():
    """One HIP runtime per process: torch ships its own libamdhip64.so.7 and the soname is
    shared with /opt/rocm's, so whichever loads first serves both.  Import torch first so
    its runtime is the one libkmerpair binds to (device pointers and streams from torch are
    then valid in the library).  Without torch the library binds /opt/rocm's runtime."""
    try:
        import torch  # noqa: F401
    except ImportError:  # pragma: no cover - torch is part of the image
        pass


def lib():
    """Load libkmerpair.so (raises if it is missing: no CPU fallback exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
                "(hipcc --offload-arch=gfx950); the k-mer pair path has no CPU fallback")
        _bind_hip_runtime()
        L = C.CDLL(LIB_PATH)
        ab = LIB_PATH != _DEFAULT_LIB  # an A/B variant (KMP_LIB) may predate newer entry points
        for name, (res, args) in SIGNATURES.items():
            if ab and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def status_string(s: int) -> str:
    try:
        return lib().kmp_status_string(s).decode()
    except Exception:  # pragma: no cover - used while formatting another error
        return "status"


def check(status: int, where: str, ctx=None) -> None:
    if status != KMP_OK:
        detail = ""
        if ctx:
            msg = lib().kmp_last_error(ctx)
            detail = msg.decode() if msg else ""
        raise KmpError(status, where, detail)


def geometry() -> PairGeometry:
    g = PairGeometry()
    lib().kmp_pair_geometry_get(C.byref(g))
    return g


def split_plan(offsets, k: int, part: int, parts: int) -> SplitSpan:
    """kmp_split_plan over host offsets (u64[N+1])."""
    import numpy as np
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    sp = SplitSpan()
    check(lib().kmp_split_plan(C.c_void_p(off.ctypes.data), len(off) - 1, k, part, parts, C.byref(sp)),
          "kmp_split_plan")
    return sp


def row_split(n: int, parts: int):
    """kmp_row_split: parts + 1 row boundaries of equal expected pair counts."""
    import numpy as np
    out = (C.c_uint32 * (parts + 1))()
    lib().kmp_row_split(n, parts, out)
    return np.array(out[:], dtype=np.uint32)
