"""ctypes binding of the CPU restatement (oracle/kmp_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package.  PARITY UNPINNED — see kmp_oracle.c's
header and DESIGN.md "Oracle": the Rust reference cannot be built or run here and ships no
golden outputs, so this restatement is pinned by hand-derived known answers, an
independent NumPy restatement (tests/numpy_ref.py) and the dataset counters of SURVEY.md §8c.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None
P = C.c_void_p


class Counters(C.Structure):
    _fields_ = [(name, C.c_uint64) for name in (
        "n_windows", "sum_S", "distinct", "repeat", "sum_cdf2", "sum_w_diff", "n_edges",
        "n_align", "pairs_any", "max_df")]

    def as_dict(self):
        return {name: int(getattr(self, name)) for name, _ in self._fields_}


SEGMENTS = 64


class Digest(C.Structure):
    """orc_digest: the counters and digest kmp_pairs_stream's summary reports."""
    _fields_ = [(name, C.c_uint64) for name in (
        "n_edges", "sum_w", "sum_score", "n_align", "sum_w_diff", "incidences", "digest")] + [
        ("seg_edges", C.c_uint64 * SEGMENTS), ("seg_digest", C.c_uint64 * SEGMENTS)]

    def as_dict(self):
        d = {n: int(getattr(self, n)) for n, _ in self._fields_ if not n.startswith("seg_")}
        d["seg_edges"] = [int(x) for x in self.seg_edges]
        d["seg_digest"] = [int(x) for x in self.seg_digest]
        return d


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        P = C.c_void_p
        L.orc_build.restype = P
        L.orc_build.argtypes = [P, P, C.c_uint32, P, C.c_int, C.c_int]
        L.orc_pairs.restype = C.c_int
        L.orc_pairs.argtypes = [P, C.c_uint32, C.c_int, C.c_uint32, C.POINTER(P), C.POINTER(P),
                                C.POINTER(P), C.POINTER(C.c_uint64)]
        L.orc_get_counters.argtypes = [P, C.POINTER(Counters)]
        for name in ("orc_codes", "orc_win_off", "orc_set_val", "orc_set_off", "orc_rep_codes",
                     "orc_rep_df", "orc_distinct", "orc_distinct_df"):
            getattr(L, name).restype = P
            getattr(L, name).argtypes = [P]
        for name in ("orc_n_windows", "orc_n_repeat", "orc_n_distinct"):
            getattr(L, name).restype = C.c_uint64
            getattr(L, name).argtypes = [P]
        L.orc_shared.restype = C.c_uint64
        L.orc_shared.argtypes = [P, C.c_uint32, C.c_uint32, P, C.c_uint64]
        L.orc_free.argtypes = [P]
        L.orc_free_ctx.argtypes = [P]
        L.orc_stream.restype = C.c_int
        L.orc_stream.argtypes = [C.POINTER(P), C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_uint32,
                                 C.c_int, C.c_int, C.c_int, C.POINTER(Digest), C.POINTER(P), C.POINTER(P),
                                 C.POINTER(P), C.POINTER(P), C.POINTER(P), C.POINTER(C.c_uint64)]
        L.orc_pair_scores.restype = C.c_int
        L.orc_pair_scores.argtypes = [P, P, P, C.c_uint64, P, C.c_int]
        L.orc_digest_term.restype = C.c_uint64
        L.orc_digest_term.argtypes = [C.c_uint32] * 5
        L.orc_rows_direct.restype = C.c_int
        L.orc_rows_direct.argtypes = [P, P, C.c_uint32, P, P, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int,
                                      C.c_int, C.c_int, C.POINTER(P), C.POINTER(P), C.POINTER(P), C.POINTER(P),
                                      C.POINTER(P), C.POINTER(C.c_uint64)]
        L.orc_residue_code.restype = C.c_uint8
        L.orc_residue_code.argtypes = [C.c_uint8]
        L.orc_pack.restype = C.c_uint32
        L.orc_pack.argtypes = [C.c_char_p, C.c_int]
        _lib = L
    return _lib


def _view(ptr, n, dtype):
    if n == 0:
        return np.zeros(0, dtype=dtype)
    ct = {np.uint32: C.c_uint32, np.uint64: C.c_uint64}[dtype]
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ct)), shape=(n,)).copy()


class Oracle:
    """One restated pipeline run over packed proteins (residues u8, offsets u64[N+1])."""

    def __init__(self, residues, offsets, class_id=None, k=5, threads=1):
        L = lib()
        self.residues = np.ascontiguousarray(residues, dtype=np.uint8)
        self.offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        self.n = len(self.offsets) - 1
        self.cls = None if class_id is None else np.ascontiguousarray(class_id, dtype=np.uint16)
        self.k = k
        res_ptr = self.residues.ctypes.data if self.residues.size else None
        self._ctx = L.orc_build(res_ptr, self.offsets.ctypes.data, self.n,
                                None if self.cls is None else self.cls.ctypes.data, k, threads)
        if not self._ctx:
            raise ValueError("orc_build failed")

    def __del__(self):
        if getattr(self, "_ctx", None):
            lib().orc_free_ctx(self._ctx)
            self._ctx = None

    def counters(self):
        c = Counters()
        lib().orc_get_counters(self._ctx, C.byref(c))
        return c.as_dict()

    def codes(self):
        L = lib()
        return _view(L.orc_codes(self._ctx), L.orc_n_windows(self._ctx), np.uint32)

    def win_off(self):
        return _view(lib().orc_win_off(self._ctx), self.n + 1, np.uint64)

    def sets(self):
        L = lib()
        off = _view(L.orc_set_off(self._ctx), self.n + 1, np.uint64)
        return off, _view(L.orc_set_val(self._ctx), int(off[-1]), np.uint32)

    def repeat(self):
        L = lib()
        r = L.orc_n_repeat(self._ctx)
        return _view(L.orc_rep_codes(self._ctx), r, np.uint32), _view(L.orc_rep_df(self._ctx), r, np.uint32)

    def hash_order(self):
        """Per protein, its repeat k-mers in first-occurrence order, duplicates dropped: the codes
        behind Protein.hash_five_mers (remove_unique_five_mers, protein.rs:151-162, then
        modify_hash_five_mer, protein.rs:165-174).  CSR (codes, offsets[n+1]); a numpy loop over
        proteins, for small batches."""
        codes, woff = self.codes(), self.win_off()
        rep, _ = self.repeat()
        keep = np.isin(codes, rep)
        out, offs = [], [0]
        for p in range(self.n):
            c = codes[woff[p]:woff[p + 1]][keep[woff[p]:woff[p + 1]]]
            _, first = np.unique(c, return_index=True)
            c = c[np.sort(first)]
            out.append(c)
            offs.append(offs[-1] + len(c))
        return (np.concatenate(out) if out else np.zeros(0, np.uint32)).astype(np.uint32), np.array(offs, np.uint64)

    def distinct(self):
        L = lib()
        d = L.orc_n_distinct(self._ctx)
        return _view(L.orc_distinct(self._ctx), d, np.uint32), _view(L.orc_distinct_df(self._ctx), d, np.uint32)

    def pairs(self, min_shared=1, require_class_diff=True, align_threshold=10):
        L = lib()
        P, Q, W = C.c_void_p(), C.c_void_p(), C.c_void_p()
        n = C.c_uint64()
        st = L.orc_pairs(self._ctx, min_shared, int(require_class_diff), align_threshold,
                         C.byref(P), C.byref(Q), C.byref(W), C.byref(n))
        if st != 0:
            raise RuntimeError(f"orc_pairs status {st}")
        out = (_view(P.value, n.value, np.uint32), _view(Q.value, n.value, np.uint32),
               _view(W.value, n.value, np.uint32))
        for ptr in (P, Q, W):
            L.orc_free(ptr)
        return out

    def pair_scores(self, p, q, threads=8):
        """BLOSUM score of each pair (the C restatement of blosum_scores below, threaded)."""
        p = np.ascontiguousarray(p, dtype=np.uint32)
        q = np.ascontiguousarray(q, dtype=np.uint32)
        out = np.zeros(len(p), dtype=np.uint32)
        if len(p):
            st = lib().orc_pair_scores(self._ctx, p.ctypes.data, q.ctypes.data, len(p), out.ctypes.data, threads)
            if st != 0:
                raise RuntimeError(f"orc_pair_scores status {st}")
        return out

    def blosum_scores(self, p, q):
        """BLOSUM-weighted score of each pair (p[i], q[i]) (a build
        extension, parity unpinned): Σ over the shared k-mers x of Σ_j B62[x_j][x_j], the diagonal
        of blosum.rs:8-30 in residue-code order (C S T A G P D E Q N H R K M I L V W Y F,
        AMINO_ACID_LIST of protein.rs:9-13), code 20 scored 0.  A loop over pairs, small batches."""
        out = np.zeros(len(p), dtype=np.int64)
        for i, (a, b) in enumerate(zip(np.asarray(p).tolist(), np.asarray(q).tolist())):
            x = self.shared(a, b).astype(np.int64)
            s = 0
            for _ in range(self.k):
                s += int(B62_DIAG[x % 21].sum())
                x //= 21
            out[i] = s
        return out

    def shared(self, p, q):
        buf = np.zeros(4096, dtype=np.uint32)
        m = lib().orc_shared(self._ctx, p, q, buf.ctypes.data, buf.size)
        if m > buf.size:
            buf = np.zeros(m, dtype=np.uint32)
            lib().orc_shared(self._ctx, p, q, buf.ctypes.data, buf.size)
        return buf[:m].copy()


def stream(oracles, row_lo=0, row_hi=None, min_shared=1, require_class_diff=True, align_threshold=10,
           blosum=True, threads=8, collect=False):
    """The config-5 union over `oracles` (one Oracle per k, same batch) of rows [row_lo, row_hi):
    the summary kmp_pairs_stream reports (counters, digest, per-segment digests) and, with
    collect, the edges (p, q, w, score, [w_k per oracle]) in canonical order."""
    L = lib()
    nk = len(oracles)
    arr = (P * nk)(*[o._ctx for o in oracles])
    n = oracles[0].n
    row_hi = n if row_hi is None else row_hi
    dg = Digest()
    ptrs = [P() for _ in range(5)]
    ne = C.c_uint64()
    st = L.orc_stream(arr, nk, row_lo, row_hi, min_shared, int(require_class_diff), align_threshold, int(blosum),
                      threads, int(collect), C.byref(dg), *[C.byref(x) for x in ptrs], C.byref(ne))
    if st != 0:
        raise RuntimeError(f"orc_stream status {st}")
    out = dg.as_dict()
    if collect:
        m = ne.value
        p, q, w, s = (_view(x.value, m, np.uint32) for x in ptrs[:4])
        wk = _view(ptrs[4].value, m * nk, np.uint32).reshape(nk, m) if m else np.zeros((nk, 0), np.uint32)
        for x in ptrs:
            L.orc_free(x)
        return out, (p, q, w, s, list(wk))
    return out


def rows_direct(residues, offsets, class_id, ks, row_lo, row_hi, min_shared=1, require_class_diff=True, blosum=True,
                threads=8):
    """Edges of the few rows [row_lo, row_hi) over every q > p, from the definition w_k(p, q) =
    |K_k(p) ∩ K_k(q)| (oracle/kmp_oracle.c orc_rows_direct; no posting lists, no global sort):
    (p, q, w, score, [w_k]) in canonical order.  An independent check of the library (and of
    orc_stream) at sizes where the posting-list oracle does not run live."""
    L = lib()
    res = np.ascontiguousarray(residues, dtype=np.uint8)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    cls = None if class_id is None else np.ascontiguousarray(class_id, dtype=np.uint16)
    karr = (C.c_int * len(ks))(*ks)
    ptrs = [P() for _ in range(5)]
    ne = C.c_uint64()
    st = L.orc_rows_direct(res.ctypes.data, off.ctypes.data, len(off) - 1, None if cls is None else cls.ctypes.data,
                           karr, len(ks), row_lo, row_hi, min_shared, int(require_class_diff), int(blosum), threads,
                           *[C.byref(x) for x in ptrs], C.byref(ne))
    if st != 0:
        raise RuntimeError(f"orc_rows_direct status {st}")
    m = ne.value
    p, q, w, s = (_view(x.value, m, np.uint32) for x in ptrs[:4])
    wk = _view(ptrs[4].value, m * len(ks), np.uint32).reshape(len(ks), m) if m else np.zeros((len(ks), 0), np.uint32)
    for x in ptrs:
        L.orc_free(x)
    return p, q, w, s, list(wk)


def digest_term(p, q, w, s, w0) -> int:
    return int(lib().orc_digest_term(p, q, w, s, w0))


# BLOSUM62 diagonal (blosum.rs:8-30: C 9, S 4, T 5, A 4, G 6, P 7, D 6, E 5, Q 5, N 6, H 8, R 5,
# K 5, M 5, I 4, L 4, V 4, W 11, Y 7, F 6), indexed by residue code; code 20 ('*', unknown) -> 0
B62_DIAG = np.array([9, 4, 5, 4, 6, 7, 6, 5, 5, 6, 8, 5, 5, 5, 4, 4, 4, 11, 7, 6, 0], dtype=np.int64)


def residue_code(b: int) -> int:
    return int(lib().orc_residue_code(b))


def pack(kmer: bytes) -> int:
    return int(lib().orc_pack(kmer, len(kmer)))
