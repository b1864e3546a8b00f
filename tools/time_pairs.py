"""Times the pair kernel alone (HIP events on torch's stream) on a bench config, repeated.
Diagnostic tool: KMP_PAIR_ABLATE=<mode> selects an ablated kernel (see kmp_kernels.hip)."""
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
    b = K.synth(n, 3)
    pipe = DevicePipeline(b, 7, "cuda:0")
    pipe.build_sets()
    pipe.filter()
    plan = pipe.plan()
    pipe.pairs()
    torch.cuda.synchronize()
    t = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        pipe.pairs()
        e1.record()
        torch.cuda.synchronize()
        t.append(e0.elapsed_time(e1))
    items = plan.items.astype(np.int64)
    d = plan.dense_off.astype(np.int64)
    cols = np.maximum(items[:, 2], items[:, 0] + 1)
    col_visits = int(np.sum(np.maximum(0, items[:, 3] - cols)))
    kmer_visits = int(np.sum(d[items[:, 3]] - d[np.minimum(cols, items[:, 3])]))
    print(f"ablate={os.environ.get('KMP_PAIR_ABLATE', '0')} window={pipe.col_window} items={len(items)} col_visits={col_visits} "
          f"kmer_visits={kmer_visits} median_ms={np.median(t):.3f} min_ms={min(t):.3f}")


if __name__ == "__main__":
    main()
