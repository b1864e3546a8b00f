"""Independent NumPy/SciPy restatement (test infrastructure): w = A·Aᵀ over the binary
protein × distinct-k-mer matrix A.  Shares no code with oracle/ (SURVEY.md §4 item 3)."""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

# src/protein.rs:9-13
_ALPHA = b"CSTAGPDEQNHRKMILVWYF*"
LUT = np.full(256, 20, dtype=np.int64)
for _i, _b in enumerate(_ALPHA):
    LUT[_b] = _i


def window_codes(seq: bytes, k: int) -> np.ndarray:
    c = LUT[np.frombuffer(seq, dtype=np.uint8)] if seq else np.zeros(0, np.int64)
    n = len(c) - k + 1
    if n <= 0:
        return np.zeros(0, dtype=np.int64)
    v = np.zeros(n, dtype=np.int64)
    for i in range(k):
        v = v * 21 + c[i:i + n]
    return v


def kmer_sets(res, off, k):
    return [np.unique(window_codes(bytes(res[int(off[p]):int(off[p + 1])]), k)) for p in range(len(off) - 1)]


def pair_weights(res, off, cls, k, require_class_diff=True, min_shared=1):
    sets = kmer_sets(res, off, k)
    n = len(sets)
    allc = np.concatenate(sets) if sets else np.zeros(0, np.int64)
    uniq, inv = np.unique(allc, return_inverse=True)
    rows = np.repeat(np.arange(n), [len(s) for s in sets])
    A = sp.csr_matrix((np.ones(len(allc), dtype=np.int32), (rows, inv)), shape=(n, len(uniq)))
    W = sp.triu(A @ A.T, k=1).tocoo()
    p, q, w = W.row.astype(np.int64), W.col.astype(np.int64), W.data.astype(np.int64)
    keep = w >= min_shared
    if require_class_diff:
        keep &= np.asarray(cls)[p] != np.asarray(cls)[q]
    p, q, w = p[keep], q[keep], w[keep]
    o = np.lexsort((q, p))
    df = np.asarray(A.sum(axis=0)).ravel()
    counters = {
        "distinct": int(len(uniq)),
        "repeat": int((df >= 2).sum()),
        "sum_cdf2": int((df * (df - 1) // 2).sum()),
        "sum_S": int(len(allc)),
    }
    return p[o].astype(np.uint32), q[o].astype(np.uint32), w[o].astype(np.uint32), counters


def hash_order(res, off, k):
    """Literal restatement of main.rs:127-193 for one batch: the df of each k-mer over the
    per-protein sets, then per protein remove_unique_five_mers (protein.rs:151-162: drop windows
    whose k-mer has df == 1, order kept) and modify_hash_five_mer (protein.rs:165-174: first
    occurrence wins).  Returns per-protein lists of codes (ids replaced by their codes) and a
    {code: df} map of the repeat k-mers (five_mer_hash_freq keyed by code)."""
    n = len(off) - 1
    wins = [window_codes(bytes(res[int(off[p]):int(off[p + 1])]), k) for p in range(n)]
    df = {}
    for w in wins:
        for c in set(w.tolist()):
            df[c] = df.get(c, 0) + 1
    out = []
    for w in wins:
        five_mers = [c for c in w.tolist() if df[c] != 1]
        seen, hashed = set(), []
        for c in five_mers:
            if c not in seen:
                seen.add(c)
                hashed.append(c)
        out.append(hashed)
    return out, {c: f for c, f in df.items() if f >= 2}
