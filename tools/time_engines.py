"""Times one full step of each engine (build sets + pairs, canonical edges resident on the
GPU) on a synthetic config, HIP events + wall clock.  Diagnostic tool."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import uniprot_kmer_based_clustering_amd as K  # noqa: E402
from uniprot_kmer_based_clustering_amd.device import DevicePipeline  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    engines = sys.argv[3].split(",") if len(sys.argv) > 3 else ["residues", "postings", "tiles"]
    b = K.synth(n, 3)
    pipe = DevicePipeline(b, 7, "cuda:0")
    for eng in engines:
        pipe.step(engine=eng)
        torch.cuda.synchronize()
        t = []
        for _ in range(reps):
            t0 = time.perf_counter()
            m = pipe.step(engine=eng)
            torch.cuda.synchronize()
            t.append((time.perf_counter() - t0) * 1e3)
        post = eng in ("postings", "residues")
        print(f"engine={eng} n={n} edges={m} median_ms={np.median(t):.3f} min_ms={min(t):.3f} "
              f"stats={pipe.postings_stats.as_dict() if post else ''}")
        if post:
            pipe.set_stage_timing(True)
            pipe.step(engine=eng)
            print("  stages_ms", {k: round(v, 3) for k, v in pipe.postings_stats.stages().items()})
            pipe.set_stage_timing(False)


if __name__ == "__main__":
    main()
