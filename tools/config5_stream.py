"""Config 5 at its stated shape on one GPU: 1,000,000 proteins (seed 5, log-uniform 50-2000),
k = 5 + 7 fused, BLOSUM, streamed (device summary only).  Prints the summary and the time."""
import json, os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import uniprot_kmer_based_clustering_amd as K
from uniprot_kmer_based_clustering_amd import _lib
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
ks = tuple(int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "5,7").split(","))
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
t0 = time.perf_counter()
b = K.synth(n, 5, 1)
print("synth", round(time.perf_counter() - t0, 2), flush=True)
with K.KmerPairEngine(0, 16) as e:
    e.load(b)
    for r in range(reps):
        t0 = time.perf_counter()
        sm = e.pairs_stream(ks, score=_lib.KMP_SCORE_BLOSUM)
        dt = time.perf_counter() - t0
        out = {k: v for k, v in sm.items() if not k.startswith("seg_")}
        out.update(n=n, ks=ks, seconds=dt)
        print(json.dumps(out), flush=True)
