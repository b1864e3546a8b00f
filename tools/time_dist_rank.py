"""Per-rank compute of the multi-GPU row split, emulated on one GPU: for G = 1, 2, 4, 8 every
rank's step (kmp_dev_pairs_rows over its kmp_row_split rows, graph-captured after its second
call) is timed in turn on its own DevicePipeline; the slowest rank bounds the step.  The gather
to rank 0 (point-to-point over xGMI) is not included.  Diagnostic tool:
python tools/time_dist_rank.py [config3|config1]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import load_batch, CONFIGS  # noqa: E402
from uniprot_kmer_based_clustering_amd.device import DevicePipeline  # noqa: E402
from uniprot_kmer_based_clustering_amd.dist import row_ranges  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "config3"
    k = CONFIGS[name][3]
    b = load_batch(name)
    out = {"config": name, "n": b.n, "ranks": {}}
    full = DevicePipeline(b, k, "cuda:0")
    for _ in range(3):
        full.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        full.step()
    torch.cuda.synchronize()
    out["single_gpu_ms"] = (time.perf_counter() - t0) / 20 * 1e3
    for g in (1, 2, 4, 8):
        per = []
        for r, (lo, hi) in enumerate(row_ranges(b.n, g)):
            pipe = DevicePipeline(b, k, "cuda:0")
            for _ in range(3):
                m = pipe.rows(lo, hi)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                m = pipe.rows(lo, hi)
            torch.cuda.synchronize()
            per.append({"rows": [lo, hi], "ms": (time.perf_counter() - t0) / 10 * 1e3, "edges": m})
            del pipe
        out["ranks"][g] = {"max_ms": max(x["ms"] for x in per), "per_rank": per}
        print(g, out["ranks"][g]["max_ms"], [round(x["ms"], 3) for x in per], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
