"""One rank's k-mer split phases in a loop, for a rocprofv3 kernel trace (diagnostic).

  python tools/prof_split_rank.py [config3|config1] G [rank] [reps] [kmer|sharded]

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
    mode = sys.argv[5] if len(sys.argv) > 5 else "kmer"
    k = CONFIGS[name][3]
    b = load_batch(name)
    if mode == "sharded":
        return sharded(b, name, k, g, rank, reps)
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


def sharded(b, name, k, g, rank, reps):
    """The sharded start's phases of rank `rank`: keys, group over the keys it would receive, edges."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from time_dist_rank import sharded_ranks  # noqa: F401  (same capacity learning)
    from uniprot_kmer_based_clustering_amd.device import ShardPipeline
    pipes = [ShardPipeline(b.residues, b.offsets, b.class_id, k, r, g, "cuda:0") for r in range(g)]
    kcap = int(pipes[0].span.key_cap)
    cap = max(4096, pipes[0].total // 4 // (g * g))
    learn = None
    for _ in range(6):
        ksend = [torch.empty(g * kcap, dtype=torch.int64, device="cuda:0") for _ in range(g)]
        sends = [torch.empty(g * cap, dtype=torch.int64, device="cuda:0") for _ in range(g)]
        flags = [torch.zeros(_lib.KMP_SPLIT_FLAGS, dtype=torch.int32, device="cuda:0") for _ in range(g)]
        stats = [torch.zeros(8, dtype=torch.int64, device="cuda:0") for _ in range(g)]
        for r in range(g):
            pipes[r].split_keys(r, g, kcap, ksend[r], flags[r])
        krecv = [torch.cat([ksend[r][d * kcap:(d + 1) * kcap] for r in range(g)]) for d in range(g)]
        for d in range(g):
            pipes[d].split_group(krecv[d], kcap, d, g, cap, sends[d], flags[d], stats[d], learn=learn)
        fl = torch.stack(flags).max(dim=0).values.cpu().tolist()
        if not fl[_lib.KMP_SPLIT_RERUN] and not fl[_lib.KMP_SPLIT_HEAVY]:
            break
        learn = fl
        cap = max(cap, fl[_lib.KMP_SPLIT_MAX_PART] * 17 // 16 + 1024)
        kcap = max(kcap, fl[_lib.KMP_SPLIT_MAX_KEYS] * 33 // 32 + 1024)
    recv = torch.cat([sends[r][rank * cap:(rank + 1) * cap] for r in range(g)])
    lo, hi = row_ranges(b.n, g)[rank]
    p = pipes[rank]
    for _ in range(reps):
        p.split_keys(rank, g, kcap, ksend[rank], flags[rank])
    for _ in range(reps):
        p.split_group(krecv[rank], kcap, rank, g, cap, sends[rank], flags[rank], stats[rank])
    for _ in range(reps):
        p.split_edges(recv, lo, hi)
    torch.cuda.synchronize()
    print(f"{name} G={g} rank={rank} rows=[{lo},{hi}) edges={p.n_edges} reps={reps} (sharded)", flush=True)


if __name__ == "__main__":
    main()
