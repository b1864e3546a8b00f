"""GPU parity of the edge-side outputs: per-edge shared k-mer lists
(KmerEdge::get_kmers, edge.rs:119-124), the reference's final edge order, the w > 10 candidate
files of align_and_output_pairs (mod.rs:195-319) and the Debug dump of main.rs:234.  The checks
restate the reference's formatting in Python (below); the lists are checked against the oracle's
shared-k-mer sets.  MPHF id values are this build's (parity unpinned for ids)."""
import os

import numpy as np
import pytest

from common import slice_proteins, tiny, uniprot
import uniprot_kmer_based_clustering_amd as K
from uniprot_kmer_based_clustering_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    e = K.KmerPairEngine(0, 4)
    yield e
    e.close()


def load(engine, res, off, cls, ids, k):
    pr = K.Proteins(res, off, cls, ids)
    engine.load(pr)
    engine.build_sets(k)
    return pr


def reference_keys(ed, ids, koff):
    """Rank of each edge in ascending (min shared id, p, q) (combine_edges, one thread)."""
    mins = ids[koff[:-1].astype(np.int64)]
    order = np.lexsort((ed.q, ed.p, mins))
    rk = np.empty(len(order), np.uint64)
    rk[order] = np.arange(len(order), dtype=np.uint64)
    return rk


@pytest.mark.parametrize("k", [5, 7])
def test_edge_kmers_match_oracle(engine, oracle_mod, k):
    for res, off, cls, ids in (tiny(), uniprot()):
        o = oracle_mod.Oracle(res, off, cls, k=k, threads=8)
        load(engine, res, off, cls, ids, k)
        with engine.edge_set() as es:
            ed = es.get()
            codes, coff = es.kmers("codes")
            np.testing.assert_array_equal(np.diff(coff.astype(np.int64)), ed.w.astype(np.int64))
            rng = np.random.default_rng(k)
            pick = rng.choice(len(ed), size=min(len(ed), 3000), replace=False) if len(ed) else []
            for i in pick:
                np.testing.assert_array_equal(codes[coff[i]:coff[i + 1]], o.shared(int(ed.p[i]), int(ed.q[i])))
            idl, ioff = es.kmers("ids")
            np.testing.assert_array_equal(ioff, coff)
            by_id = engine.get_repeat_codes()
            for i in pick:
                seg = idl[ioff[i]:ioff[i + 1]]
                assert np.all(np.diff(seg.astype(np.int64)) > 0)  # ascending ids
                np.testing.assert_array_equal(np.sort(by_id[seg]), codes[coff[i]:coff[i + 1]])
            np.testing.assert_array_equal(es.reference_keys(), reference_keys(ed, idl, ioff))


def test_edge_kmers_all_edges_small(engine, oracle_mod):
    res, off, cls, ids = slice_proteins(*uniprot()[:3], np.arange(400)) + ([],)
    o = oracle_mod.Oracle(res, off, cls, k=5)
    load(engine, res, off, cls, None, 5)
    with engine.edge_set(require_class_diff=False) as es:
        ed = es.get()
        codes, coff = es.kmers("codes")
        for i in range(len(ed)):
            np.testing.assert_array_equal(codes[coff[i]:coff[i + 1]], o.shared(int(ed.p[i]), int(ed.q[i])))


def test_edge_kmers_reject_foreign_edges(engine):
    res, off, cls, ids = uniprot()
    load(engine, res, off, cls, ids, 5)
    with engine.edge_set() as es:
        engine.build_sets(7)
        with pytest.raises(_lib.KmpError) as ei:
            es.kmers("codes")
        assert ei.value.status == _lib.KMP_EINVAL
        with pytest.raises(_lib.KmpError) as ei:
            es.reference_keys()
        assert ei.value.status == _lib.KMP_ESTATE


def expected_candidates(ed, rk, pr, threshold):
    """mod.rs:241-280: for edge_key with w > 10, ">{id}\\n{seq}" of p, then of q, in
    fasta_files/{edge_key}_{id.split_once('|').0}.fasta (the query overwrites on equal names)."""
    files = {}
    for i in range(len(ed)):
        if ed.w[i] <= threshold:
            continue
        for v in (int(ed.p[i]), int(ed.q[i])):
            pid = pr.ids[v]
            seq = bytes(pr.residues[int(pr.offsets[v]):int(pr.offsets[v + 1])])
            files[f"{int(rk[i])}_{pid.split('|', 1)[0]}.fasta"] = b">" + pid.encode() + b"\n" + seq
    return files


HEADER = ("query id\tquery length\tsubject id\tsubject length\tquery alignment start\tquery alignment end\t"
          "subject alignment start\tsubject alignment end\talignment length\tpercent identity\tevalue\tbit score\n")


@pytest.mark.parametrize("threshold", [10, 3])
def test_candidate_files(engine, tmp_path, threshold):
    res, off, cls, ids = uniprot()
    pr = load(engine, res, off, cls, ids, 5)
    # files of an earlier run are removed (the reference's rm -r, mod.rs:202-210)
    for d in ("fasta_files", "db_files"):
        (tmp_path / d / "old").mkdir(parents=True)
        (tmp_path / d / "old" / "stale.fasta").write_text(">x\nA")
        (tmp_path / d / "stale.fasta").write_text(">x\nA")
    with engine.edge_set() as es:
        ed = es.get()
        es.kmers("ids")
        rk = es.reference_keys()
        n = es.write_candidates(pr, str(tmp_path), threshold=threshold, threads=8)
    assert n == int((ed.w > threshold).sum())
    want = expected_candidates(ed, rk, pr, threshold)
    got = sorted(os.listdir(tmp_path / "fasta_files"))
    assert got == sorted(want)
    for name in got[:: max(1, len(got) // 500)]:
        assert (tmp_path / "fasta_files" / name).read_bytes() == want[name], name
    assert (tmp_path / "blastp_output.tsv").read_text() == HEADER
    assert (tmp_path / "db_files").is_dir() and not os.listdir(tmp_path / "db_files")
    # without IDS lists the edge index is the key
    with engine.edge_set() as es:
        out = tmp_path / "plain"
        es.write_candidates(pr, str(out), threshold=threshold)
        want2 = expected_candidates(ed, np.arange(len(ed)), pr, threshold)
        assert sorted(os.listdir(out / "fasta_files")) == sorted(want2)


def rust_debug(ed, ids, koff, rk, n):
    """`{:#?}` of Graph (mod.rs:700-708) as main.rs:234 prints it, restated."""
    order = np.argsort(rk)
    out = ["Graph right now:\n", "Graph {\n"]
    if len(ed) == 0:
        out.append("    Kmers: [],\n")
    else:
        out.append("    Kmers: [\n")
        for i in order:
            seg = ids[koff[i]:koff[i + 1]]
            if len(seg) == 1:
                out.append(f"        Single Kmer {{\n            kmer: {int(seg[0])},\n            size: 2,\n        }},\n")
            else:
                out.append("        Kmer Group {\n            kmer: [\n")
                out.extend(f"                {int(x)},\n" for x in seg)
                out.append("            ],\n            size: 2,\n        },\n")
        out.append("    ],\n")
    deg = np.bincount(np.concatenate([ed.p, ed.q]).astype(np.int64), minlength=n)
    if n == 0:
        out.append("    Proteins: [],\n")
    else:
        out.append("    Proteins: [\n")
        out.extend(f"        Protein {{\n            key: {p},\n            size: {int(deg[p])},\n        }},\n"
                   for p in range(n))
        out.append("    ],\n")
    out.append("}\n")
    return "".join(out)


@pytest.mark.parametrize("which", ["tiny", "uniprot"])
def test_graph_debug_dump(engine, tmp_path, which):
    res, off, cls, ids = tiny() if which == "tiny" else uniprot()
    load(engine, res, off, cls, ids, 5)
    n = len(off) - 1
    with engine.edge_set() as es:
        ed = es.get()
        with pytest.raises(_lib.KmpError):
            es.write_debug(str(tmp_path / "g.txt"), n)  # needs IDS lists
        idl, ioff = es.kmers("ids")
        rk = es.reference_keys()
        es.write_debug(str(tmp_path / "g.txt"), n, threads=8)
    assert (tmp_path / "g.txt").read_text() == rust_debug(ed, idl, ioff, rk, n)
