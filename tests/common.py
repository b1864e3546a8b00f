"""Shared test helpers (test infrastructure; may use oracle/)."""
from __future__ import annotations

import gzip
import hashlib
import json
import os
import sys

import numpy as np

TESTS = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(TESTS)
GOLDEN = os.path.join(TESTS, "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def golden(name: str) -> str:
    return os.path.join(GOLDEN, name)


def load_json(name: str):
    with open(golden(name)) as f:
        return json.load(f)


def parse_fasta_bytes(data: bytes):
    """Independent pure-Python FASTA reader with the seq_io semantics of kmp_fasta.cpp."""
    ids, seqs, classes = [], [], []
    lines = data.split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()
    cur = None
    for raw in lines:
        line = raw[:-1] if raw.endswith(b"\r") else raw
        if line.startswith(b">"):
            head = line[1:]
            ident = head.split(b" ", 1)[0]
            fields = ident.split(b"|")
            if fields and fields[-1] == b"":
                fields = fields[:-1]
            ids.append(ident.decode())
            classes.append(fields[3])
            cur = []
            seqs.append(cur)
        elif cur is not None:
            cur.append(raw)  # interior terminators stay raw (seq_io seq())
    seqs = [b"\n".join(s) for s in seqs]
    seqs = [s[:-1] if s.endswith(b"\r") else s for s in seqs]  # last line's CR goes
    intern = {}
    cid = np.array([intern.setdefault(c, len(intern)) for c in classes], dtype=np.uint16)
    off = np.zeros(len(seqs) + 1, dtype=np.uint64)
    if seqs:
        off[1:] = np.cumsum([len(s) for s in seqs])
    res = np.frombuffer(b"".join(seqs), dtype=np.uint8).copy()
    return res, off, cid, ids


def uniprot_bytes() -> bytes:
    with gzip.open(golden("uniprot_arg.fasta.gz"), "rb") as f:
        return f.read()


def uniprot():
    return parse_fasta_bytes(uniprot_bytes())


def tiny():
    with open(golden("tiny.fasta"), "rb") as f:
        return parse_fasta_bytes(f.read())


def read_edges_tsv(name: str):
    rows = [tuple(int(x) for x in line.split("\t")) for line in open(golden(name))
            if line.strip() and not line.startswith("#")]
    a = np.array(rows, dtype=np.uint32).reshape(-1, 3)
    return a[:, 0].copy(), a[:, 1].copy(), a[:, 2].copy()


def edges_sha256(p, q, w) -> str:
    a = np.stack([np.asarray(p, np.uint32), np.asarray(q, np.uint32), np.asarray(w, np.uint32)], axis=1)
    return hashlib.sha256(np.ascontiguousarray(a).astype("<u4").tobytes()).hexdigest()


def slice_proteins(res, off, cls, idx):
    """Sub-batch of proteins idx (in the given order)."""
    idx = np.asarray(idx)
    lens = (off[1:] - off[:-1])[idx].astype(np.int64)
    new_off = np.zeros(len(idx) + 1, dtype=np.uint64)
    new_off[1:] = np.cumsum(lens)
    parts = [res[int(off[i]):int(off[i + 1])] for i in idx]
    new_res = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    return new_res.astype(np.uint8), new_off, np.asarray(cls)[idx].astype(np.uint16)


def make_batch(seqs, classes):
    """Proteins from python byte strings + class labels."""
    intern = {}
    cid = np.array([intern.setdefault(c, len(intern)) for c in classes], dtype=np.uint16)
    off = np.zeros(len(seqs) + 1, dtype=np.uint64)
    if seqs:
        off[1:] = np.cumsum([len(s) for s in seqs])
    res = np.frombuffer(b"".join(seqs), dtype=np.uint8).copy()
    return res, off, cid
