"""Python face of the host-buffer C ABI (include/kmerpair.h), used by tests and tools.

``KmerPairEngine`` follows the reference's call order in src/main.rs: load the proteins
(``Protein::new`` batch, main.rs:65-72), build the k-mer sets and the repeat filter
(main.rs:77-199), then the fused graph pass (``Graph::new`` + ``remove_uninteresting_edges``
+ ``combine_edges``, main.rs:217-227) that returns the collapsed edge list.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import check, lib


def _ptr(a: np.ndarray | None):
    return None if a is None or a.size == 0 else C.c_void_p(a.ctypes.data)


@dataclass
class Proteins:
    """Packed protein batch: residues u8[ΣL], offsets u64[N+1], class ids u16[N]."""
    residues: np.ndarray
    offsets: np.ndarray
    class_id: np.ndarray
    ids: list | None = None
    n_classes: int = 0

    @property
    def n(self) -> int:
        return len(self.offsets) - 1


def read_fasta(path: str, threads: int = 0) -> Proteins:
    """FASTA ingest with seq_io semantics (libkmerpair kmp_read_fasta_threads; threads 0: the
    library's default, min(16, hardware threads))."""
    L = lib()
    n = C.c_uint32()
    res, off, cls, ids = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_void_p()
    ids_bytes = C.c_uint64()
    ncls = C.c_uint32()
    st = L.kmp_read_fasta_threads(path.encode(), threads, C.byref(n), C.byref(res), C.byref(off), C.byref(cls),
                                  C.byref(ids), C.byref(ids_bytes), C.byref(ncls))
    check(st, f"kmp_read_fasta({path})")
    try:
        N = n.value
        offsets = np.ctypeslib.as_array(C.cast(off, C.POINTER(C.c_uint64)), shape=(N + 1,)).copy()
        total = int(offsets[-1])
        residues = (np.ctypeslib.as_array(C.cast(res, C.POINTER(C.c_uint8)), shape=(total,)).copy()
                    if total else np.zeros(0, np.uint8))
        class_id = (np.ctypeslib.as_array(C.cast(cls, C.POINTER(C.c_uint16)), shape=(N,)).copy()
                    if N else np.zeros(0, np.uint16))
        raw = C.string_at(ids, ids_bytes.value) if ids_bytes.value else b""
        id_list = [s.decode() for s in raw.split(b"\0")[:N]] if N else []
    finally:
        for p in (res, off, cls, ids):
            L.kmp_free_host(p)
    return Proteins(residues, offsets, class_id, id_list, ncls.value)


def synth(n: int, seed: int, law: int = _lib.KMP_LEN_NORMAL300, with_family=False):
    """Synthetic protein batch of SURVEY.md §8d (deterministic in (n, seed, law))."""
    L = lib()
    offsets = np.zeros(n + 1, dtype=np.uint64)
    cls = np.zeros(n, dtype=np.uint16)
    fam = np.zeros(n, dtype=np.uint32)
    res = C.c_void_p()
    check(L.kmp_synth_packed(n, seed, law, C.byref(res), _ptr(offsets), _ptr(cls), _ptr(fam)),
          "kmp_synth_packed")
    total = int(offsets[-1])
    try:
        residues = np.ctypeslib.as_array(C.cast(res, C.POINTER(C.c_uint8)), shape=(total,)).copy()
    finally:
        L.kmp_free_host(res)
    p = Proteins(residues, offsets, cls, None, 15)
    return (p, fam) if with_family else p


def write_synth_fasta(path: str, n: int, seed: int, law: int = _lib.KMP_LEN_NORMAL300) -> None:
    check(lib().kmp_synth_write_fasta(path.encode(), n, seed, law), "kmp_synth_write_fasta")


@dataclass
class Edges:
    p: np.ndarray
    q: np.ndarray
    w: np.ndarray
    score: np.ndarray

    def __len__(self):
        return len(self.p)


class KmerPairEngine:
    """One device context (kmp_ctx) holding a protein batch and its k-mer sets."""

    def __init__(self, device: int = 0, cpu_threads: int = 1, devices=None):
        """devices: HIP ordinals of a multi-GPU context (kmp_ctx_create_multi; repeating one
        runs several ranks on that GPU); None: the single-GPU context on `device`."""
        self._ctx = C.c_void_p()
        if devices is None:
            check(lib().kmp_ctx_create(C.byref(self._ctx), device, cpu_threads), "kmp_ctx_create")
        else:
            arr = (C.c_int * len(devices))(*devices)
            st = lib().kmp_ctx_create_multi(C.byref(self._ctx), len(devices), arr, cpu_threads)
            check(st, "kmp_ctx_create_multi")

    @property
    def gpus(self) -> int:
        return int(lib().kmp_ctx_gpus(self._ctx))

    @property
    def transport(self) -> str:
        return lib().kmp_ctx_transport(self._ctx).decode()

    @property
    def last_split(self) -> str:
        """Flow of the last multi-GPU pairs call: 'kmer' (k-mer split) or 'rows' (row split)."""
        return lib().kmp_ctx_last_split(self._ctx).decode()

    def set_pass_keys(self, keys: int) -> None:
        """Bounded-memory passes: pair keys per pass (0: auto, from the free device memory)."""
        self._check(lib().kmp_ctx_set_pass_keys(self._ctx, keys), "kmp_ctx_set_pass_keys")

    def set_direct_tail(self, enable: bool = True) -> None:
        """kmp_pairs_stream's fused reduction writes its edges in place (default) or stages them."""
        self._check(lib().kmp_ctx_set_direct_tail(self._ctx, int(enable)), "kmp_ctx_set_direct_tail")

    def set_flat_heavy(self, enable: bool = True) -> None:
        """pairs_stream's passes expand frequent k-mers by rows (default) or by per-k-mer tiles."""
        self._check(lib().kmp_ctx_set_flat_heavy(self._ctx, int(enable)), "kmp_ctx_set_flat_heavy")

    @property
    def last_tail_windows(self) -> int:
        """Sub-blocks of the last pairs_stream reduced in windows (above the LDS sort capacity)."""
        return int(lib().kmp_ctx_last_tail_windows(self._ctx))

    def set_rows(self, row_lo: int = 0, row_hi: int = 0) -> None:
        """Rows kmp_pairs_stream covers ([0, 0): all): a process's share of a multi-process split."""
        self._check(lib().kmp_ctx_set_rows(self._ctx, row_lo, row_hi), "kmp_ctx_set_rows")

    @property
    def last_passes(self) -> int:
        return int(lib().kmp_ctx_last_passes(self._ctx))

    def close(self):
        if self._ctx:
            lib().kmp_ctx_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, st, where):
        check(st, where, self._ctx)

    def load(self, proteins: Proteins) -> None:
        res = np.ascontiguousarray(proteins.residues, dtype=np.uint8)
        off = np.ascontiguousarray(proteins.offsets, dtype=np.uint64)
        cls = np.ascontiguousarray(proteins.class_id, dtype=np.uint16)
        self._check(lib().kmp_load_proteins(self._ctx, _ptr(res), _ptr(off), len(off) - 1, _ptr(cls)),
                    "kmp_load_proteins")
        self.n = len(off) - 1

    def extract(self, k: int) -> None:
        self._check(lib().kmp_extract(self._ctx, k), "kmp_extract")

    def _get(self, fn, name, p):
        n = C.c_uint64()
        st = fn(self._ctx, p, None, 0, C.byref(n))
        if st not in (_lib.KMP_OK, _lib.KMP_EOVERFLOW):
            self._check(st, name)
        out = np.zeros(n.value, dtype=np.uint32)
        self._check(fn(self._ctx, p, _ptr(out), n.value, C.byref(n)), name)
        return out

    def get_kmers(self, p: int) -> np.ndarray:
        return self._get(lib().kmp_get_kmers, "kmp_get_kmers", p)

    def build_sets(self, k: int) -> None:
        self._check(lib().kmp_build_sets(self._ctx, k), "kmp_build_sets")

    def get_set(self, p: int) -> np.ndarray:
        return self._get(lib().kmp_get_set, "kmp_get_set", p)

    # ---- repeat index (main.rs:127-149,187-193; protein.rs:151-174) ----
    def _get_all(self, fn, name):
        n = C.c_uint64()
        st = fn(self._ctx, None, 0, C.byref(n))
        if st not in (_lib.KMP_OK, _lib.KMP_EOVERFLOW):
            self._check(st, name)
        out = np.zeros(n.value, dtype=np.uint32)
        self._check(fn(self._ctx, _ptr(out), n.value, C.byref(n)), name)
        return out

    def get_df(self) -> np.ndarray:
        """five_mer_hash_freq: df of each repeat k-mer, indexed by its repeat-MPHF id."""
        return self._get_all(lib().kmp_get_df, "kmp_get_df")

    def get_repeat_codes(self) -> np.ndarray:
        """code of each repeat-MPHF id (the inverse of Mphf::hash over the repeat k-mers)."""
        return self._get_all(lib().kmp_get_repeat_codes, "kmp_get_repeat_codes")

    def get_hash_kmers(self, p: int) -> np.ndarray:
        """Protein.hash_five_mers (get_five_hash, protein.rs:146): repeat ids, first occurrence."""
        return self._get(lib().kmp_get_hash_kmers, "kmp_get_hash_kmers", p)

    def get_hash_kmers_all(self) -> tuple[np.ndarray, np.ndarray]:
        """hash_five_mers of every protein as CSR (ids, offsets[n+1])."""
        n = C.c_uint64()
        off = np.zeros(self.n + 1, dtype=np.uint64)
        st = lib().kmp_get_hash_kmers_all(self._ctx, None, 0, _ptr(off), C.byref(n))
        if st not in (_lib.KMP_OK, _lib.KMP_EOVERFLOW):
            self._check(st, "kmp_get_hash_kmers_all")
        ids = np.zeros(n.value, dtype=np.uint32)
        self._check(lib().kmp_get_hash_kmers_all(self._ctx, _ptr(ids), n.value, _ptr(off), C.byref(n)),
                    "kmp_get_hash_kmers_all")
        return ids, off

    def repeat_mphf(self) -> "Mphf":
        """The context's repeat-k-mer MPHF (valid until the next load / build_sets)."""
        m = C.c_void_p()
        self._check(lib().kmp_repeat_mphf(self._ctx, C.byref(m)), "kmp_repeat_mphf")
        return Mphf(m, owner=self)

    def mphf(self, keys, gamma: float = 3.0) -> "Mphf":
        """Mphf::new(gamma, &keys) on this context's device."""
        k = np.ascontiguousarray(keys, dtype=np.uint32)
        m = C.c_void_p()
        self._check(lib().kmp_mphf_build(self._ctx, _ptr(k), len(k), gamma, C.byref(m)), "kmp_mphf_build")
        return Mphf(m)

    def counters(self) -> dict:
        c = _lib.Counters()
        self._check(lib().kmp_counters_get(self._ctx, C.byref(c)), "kmp_counters_get")
        return c.as_dict()

    def edge_set(self, min_shared=1, require_class_diff=True, align_threshold=10,
                 score=_lib.KMP_SCORE_COUNT, engine=_lib.KMP_ENGINE_AUTO) -> "EdgeSet":
        """kmp_pairs, keeping the library-owned edge list for the k-mer lists and the writers."""
        o = _lib.PairOpts(min_shared, int(require_class_diff), align_threshold, score, engine)
        e = C.c_void_p()
        self._check(lib().kmp_pairs(self._ctx, C.byref(o), C.byref(e)), "kmp_pairs")
        return EdgeSet(self, e)

    def pairs(self, min_shared=1, require_class_diff=True, align_threshold=10,
              score=_lib.KMP_SCORE_COUNT, engine=_lib.KMP_ENGINE_AUTO) -> Edges:
        with self.edge_set(min_shared, require_class_diff, align_threshold, score, engine) as es:
            return es.get()

    def pairs_multi_k(self, ks=(5, 7), min_shared=1, require_class_diff=True, align_threshold=10,
                      score=_lib.KMP_SCORE_COUNT, engine=_lib.KMP_ENGINE_AUTO):
        """kmp_pairs_multi_k: the union over k of the per-k edge lists,
        w = Σ_k w_k, score = Σ_k score_k.  Returns (Edges, {k: w_k array})."""
        o = _lib.PairOpts(min_shared, int(require_class_diff), align_threshold, score, engine)
        karr = (C.c_int * len(ks))(*ks)
        h = C.c_void_p()
        self._check(lib().kmp_pairs_multi_k(self._ctx, C.byref(o), karr, len(ks), C.byref(h)), "kmp_pairs_multi_k")
        with EdgeSet(self, h) as es:
            edges = es.get()
            wk = {}
            for j, k in enumerate(ks):
                w = np.zeros(len(edges), np.uint32)
                n = C.c_uint64()
                check(lib().kmp_edges_get_wk(h, j, _ptr(w), len(w), C.byref(n)), "kmp_edges_get_wk")
                wk[k] = w
        return edges, wk


    def pairs_stream(self, ks=(5,), min_shared=1, require_class_diff=True, align_threshold=10,
                     score=_lib.KMP_SCORE_COUNT, sink=None, on_device=False) -> dict:
        """kmp_pairs_stream: the edges of ks (one k, or the config-5 union) in row passes, each
        handed to ``sink(chunk)`` (a dict: rank, row_lo, row_hi, n, and numpy arrays p, q, w, score,
        wk (list) when on_device is False; raw device pointers otherwise), never resident whole.
        Returns the stream summary (counters, digest, per-segment digests, passes, ordered)."""
        o = _lib.PairOpts(min_shared, int(require_class_diff), align_threshold, score, _lib.KMP_ENGINE_AUTO)
        karr = (C.c_int * len(ks))(*ks)
        err = []

        def _sink(user, chp):
            try:
                ch = chp.contents
                d = {"rank": ch.rank, "row_lo": ch.row_lo, "row_hi": ch.row_hi, "n": int(ch.n),
                     "on_device": bool(ch.on_device), "device": ch.device}
                if ch.on_device:
                    d.update(p=ch.p, q=ch.q, w=ch.w, score=ch.score, wk=[ch.wk[j] for j in range(len(ks))])
                else:
                    def arr(ptr):
                        if not ptr or ch.n == 0:
                            return np.zeros(0, np.uint32)
                        return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint32)), shape=(ch.n,)).copy()
                    d.update(p=arr(ch.p), q=arr(ch.q), w=arr(ch.w), score=arr(ch.score),
                             wk=[arr(ch.wk[j]) for j in range(len(ks))])
                r = sink(d)
                return int(r or 0)
            except Exception as exc:  # surfaced after the call
                err.append(exc)
                return _lib.KMP_EINVAL
        cb = _lib.EDGE_SINK(_sink) if sink is not None else _lib.EDGE_SINK()
        sm = _lib.StreamSummary()
        st = lib().kmp_pairs_stream(self._ctx, C.byref(o), karr, len(ks), int(bool(on_device)), cb, None,
                                    C.byref(sm))
        if err:
            raise err[0]
        self._check(st, "kmp_pairs_stream")
        return sm.as_dict()


def digest_term(p, q, w, s, w0) -> int:
    """kmp_edge_digest_term of one edge (the stream digest's per-edge term)."""
    return int(lib().kmp_edge_digest_term(p, q, w, s, w0))


class Mphf:
    """boomphf ``Mphf<u32>`` surface over the device MPHF (include/kmerpair.h "MPHF").
    ``owner`` set: a context-owned MPHF (kmp_repeat_mphf), never freed here."""

    def __init__(self, handle: C.c_void_p, owner=None):
        self._m = handle
        self._owner = owner

    def hash(self, keys) -> np.ndarray:
        k = np.ascontiguousarray(np.atleast_1d(keys), dtype=np.uint32)
        ids = np.zeros(len(k), dtype=np.uint64)
        check(lib().kmp_mphf_lookup(self._m, _ptr(k), len(k), _ptr(ids)), "kmp_mphf_lookup")
        return ids

    def dev_hash(self, keys, stream=None):
        """ids (int64 torch tensor) of a uint32-valued device tensor, on ``stream``."""
        import torch
        k = keys.contiguous()
        ids = torch.empty(k.numel(), dtype=torch.int64, device=k.device)
        s = stream if stream is not None else torch.cuda.current_stream(k.device)
        check(lib().kmp_mphf_dev_lookup(self._m, C.c_void_p(k.data_ptr()), k.numel(),
                                        C.c_void_p(ids.data_ptr()), C.c_void_p(s.cuda_stream)),
              "kmp_mphf_dev_lookup")
        return ids

    def info(self) -> dict:
        n, lv, bits, fb = C.c_uint64(), C.c_uint32(), C.c_uint64(), C.c_uint64()
        check(lib().kmp_mphf_info(self._m, C.byref(n), C.byref(lv), C.byref(bits), C.byref(fb)), "kmp_mphf_info")
        return {"n": n.value, "levels": lv.value, "bits": bits.value, "fallback": fb.value}

    def close(self):
        if self._m and self._owner is None:
            lib().kmp_mphf_free(self._m)
        self._m = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class EdgeSet:
    """A library-owned edge list (kmp_edges) and what the reference derives from its edges:
    shared k-mer lists (KmerEdge::get_kmers), the reference edge order, the w > 10 candidate
    files of align_and_output_pairs and the Debug dump of the final graph."""

    def __init__(self, engine: KmerPairEngine, handle: C.c_void_p):
        self._engine = engine
        self._e = handle

    def close(self):
        if self._e:
            lib().kmp_edges_free(self._e)
            self._e = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __len__(self):
        n = C.c_uint64()
        check(lib().kmp_edges_count(self._e, C.byref(n)), "kmp_edges_count")
        return n.value

    def get(self) -> Edges:
        m = len(self)
        n = C.c_uint64()
        p, q, w = (np.zeros(m, np.uint32) for _ in range(3))
        s = np.zeros(m, np.float32)
        check(lib().kmp_edges_get(self._e, _ptr(p), _ptr(q), _ptr(w), _ptr(s), m, C.byref(n)), "kmp_edges_get")
        return Edges(p, q, w, s)

    def kmers(self, space: str = "ids") -> tuple[np.ndarray, np.ndarray]:
        """(kmers, offsets[count+1]): edge i's shared k-mers, ascending MPHF ids or codes."""
        sp = {"ids": _lib.KMP_KMERS_IDS, "codes": _lib.KMP_KMERS_CODES}[space]
        self._engine._check(lib().kmp_edges_kmers(self._engine._ctx, self._e, sp), "kmp_edges_kmers")
        off = np.zeros(len(self) + 1, np.uint64)
        n = C.c_uint64()
        st = lib().kmp_edges_get_kmers(self._e, _ptr(off), None, 0, C.byref(n))
        if st not in (_lib.KMP_OK, _lib.KMP_EOVERFLOW):
            check(st, "kmp_edges_get_kmers")
        km = np.zeros(n.value, np.uint32)
        check(lib().kmp_edges_get_kmers(self._e, _ptr(off), _ptr(km), n.value, C.byref(n)), "kmp_edges_get_kmers")
        return km, off

    def reference_keys(self) -> np.ndarray:
        """Each edge's index in the reference's final edge list (needs kmers("ids"))."""
        m = len(self)
        out = np.zeros(m, np.uint64)
        n = C.c_uint64()
        check(lib().kmp_edges_reference_keys(self._e, _ptr(out), m, C.byref(n)), "kmp_edges_reference_keys")
        return out

    def write_candidates(self, proteins: Proteins, out_dir: str, threshold: int = 10, threads: int = 4) -> int:
        """fasta_files/{edge_key}_{prefix}.fasta pairs + blastp_output.tsv header (mod.rs:195-319)."""
        if proteins.ids is None:
            raise ValueError("write_candidates needs protein ids (read_fasta)")
        blob = b"\0".join(i.encode() for i in proteins.ids) + b"\0"
        buf = np.frombuffer(blob, np.uint8).copy()
        res = np.ascontiguousarray(proteins.residues, np.uint8)
        off = np.ascontiguousarray(proteins.offsets, np.uint64)
        n = C.c_uint64()
        check(lib().kmp_write_candidates(self._e, _ptr(res), _ptr(off), proteins.n, _ptr(buf), len(blob), threshold,
                                         out_dir.encode(), threads, C.byref(n)), "kmp_write_candidates")
        return n.value

    def write_debug(self, path: str, n_proteins: int, threads: int = 4) -> None:
        """The reference's final `println!("Graph right now:\\n{graph:#?}")` (needs kmers("ids"))."""
        check(lib().kmp_write_graph_debug(self._e, n_proteins, path.encode(), threads), "kmp_write_graph_debug")
