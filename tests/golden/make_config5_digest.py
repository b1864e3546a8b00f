"""Generates tests/golden/config5_1m_k5k7_blosum_digest.json: the oracle's summary (counters,
digest, per-row-segment digests; oracle/kmp_oracle.c orc_stream) of config 5 at its stated shape
(1,000,000 synthetic proteins, seed 5, log-uniform lengths 50-2000, k = 5 + 7,
BLOSUM score, class filter on, min_shared 1).  The oracle restates the reference's posting-list
expansion row by row; at this size it runs ~14 min on 8 threads (~20 GB of host memory), so the
GPU test compares against this fixture instead of running it live.

    python tests/golden/make_config5_digest.py [N] [threads]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
import uniprot_kmer_based_clustering_amd as K  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    b = K.synth(n, 5, 1)
    orcs = []
    for k in (5, 7):
        t0 = time.time()
        orcs.append(O.Oracle(b.residues, b.offsets, b.class_id, k=k, threads=threads))
        print("oracle build k", k, round(time.time() - t0, 1), "s", flush=True)
    t0 = time.time()
    d = O.stream(orcs, threads=threads)
    d["meta"] = {"n": n, "seed": 5, "law": "log-uniform 50-2000", "ks": [5, 7], "score": "blosum",
                 "require_class_diff": True, "min_shared": 1, "oracle_seconds": round(time.time() - t0, 1),
                 "threads": threads,
                 "counters_k5": orcs[0].counters(), "counters_k7": orcs[1].counters()}
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), f"config5_{n // 1000}k_k5k7_blosum_digest.json"
                       if n != 1_000_000 else "config5_1m_k5k7_blosum_digest.json")
    json.dump(d, open(out, "w"), indent=1)
    print(out, {k: v for k, v in d.items() if not k.startswith("seg") and k != "meta"})


if __name__ == "__main__":
    main()
