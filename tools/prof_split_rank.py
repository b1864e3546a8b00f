"""One rank's k-mer split phases in a loop, for a rocprofv3 kernel trace (diagnostic).

  python tools/prof_split_rank.py [config3|config1] G [rank] [reps]

Learns the capacities like tools/time_dist_rank.py, then runs rank `rank` of G's
kmp_dev_split_expand and kmp_dev_split_edges `reps` times each, so the kernel statistics of the
trace are that rank's per-step kernels (exchanges excluded: the received keys are the
concatenation of every rank's send region for this rank, built once)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import load_batch, CONFIGS  # noqa: E402
from uniprot_kmer_based_clustering_amd import _lib  # noqa: E402
from uniprot_kmer_based_clustering_amd.device import DevicePipeline  # noqa: E402
from uniprot_kmer_based_clustering_amd.dist import row_ranges  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "config3"
    g = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    rank = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    k = CONFIGS[name][3]
    b = load_batch(name)
    pipes = [DevicePipeline(b, k, "cuda:0") for _ in range(g)]
    cap = max(4096, pipes[0].total // 4 // (g * g))
    learn = None
    for _ in range(4):
        sends = [torch.empty(g * cap, dtype=torch.int64, device="cuda:0") for _ in range(g)]
        flags = [torch.zeros(_lib.KMP_SPLIT_FLAGS, dtype=torch.int32, device="cuda:0") for _ in range(g)]
        stats = [torch.zeros(8, dtype=torch.int64, device="cuda:0") for _ in range(g)]
        for r in range(g):
            pipes[r].split_expand(r, g, cap, sends[r], flags[r], stats[r], learn=learn)
        fl = torch.stack(flags).max(dim=0).values.cpu().tolist()
        if not fl[_lib.KMP_SPLIT_RERUN] and not fl[_lib.KMP_SPLIT_HEAVY]:
            break
        learn = fl
        cap = max(cap, fl[_lib.KMP_SPLIT_MAX_PART] * 17 // 16 + 1024)
    recv = torch.cat([sends[r][rank * cap:(rank + 1) * cap] for r in range(g)])
    lo, hi = row_ranges(b.n, g)[rank]
    p = pipes[rank]
    for _ in range(reps):
        p.split_expand(rank, g, cap, sends[rank], flags[rank], stats[rank])
    for _ in range(reps):
        p.split_edges(recv, lo, hi)
    torch.cuda.synchronize()
    print(f"{name} G={g} rank={rank} rows=[{lo},{hi}) edges={p.n_edges} reps={reps}", flush=True)


if __name__ == "__main__":
    main()
