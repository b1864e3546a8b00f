import sys, time, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import uniprot_kmer_based_clustering_amd as K
from uniprot_kmer_based_clustering_amd import _lib
for n in (100_000, 300_000, 1_000_000):
    b = K.synth(n, 5, 1)
    with K.KmerPairEngine(0, 16) as e:
        e.load(b)
        for rep in range(2):
            t0 = time.perf_counter()
            got, wk = e.pairs_multi_k((5, 7), score=_lib.KMP_SCORE_BLOSUM)
            dt = time.perf_counter() - t0
            print(n, rep, "edges", len(got), "passes", e.last_passes, "s %.3f" % dt, flush=True)
            del got, wk
