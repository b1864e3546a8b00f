"""Debug: the engine fixture's call sequence of test_gpu_edges_out (tiny k5, uniprot k5, tiny k7)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
from common import tiny, uniprot
import uniprot_kmer_based_clustering_amd as K
from oracle.oracle import Oracle
e = K.KmerPairEngine(0, 4)
for k in (5, 7):
    for name, (res, off, cls, _) in (("tiny", tiny()), ("uniprot", uniprot())):
        e.load(K.Proteins(res, off, cls))
        e.build_sets(k)
        try:
            got = e.pairs()
        except Exception as ex:
            print(name, k, "ERROR", ex, flush=True)
            continue
        p, q, w = Oracle(res, off, cls, k=k, threads=8).pairs()
        ok = len(got) == len(p) and np.array_equal(got.p, p) and np.array_equal(got.q, q) and np.array_equal(got.w, w)
        print(name, k, len(got), len(p), ok, flush=True)
