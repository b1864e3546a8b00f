"""Benchmark of the k-mer pair path (BASELINE.json metric: protein pairs/sec + edges/sec,
100k x 300 aa synthetic proteins, k = 7, 1/2/4/8 MI355X).

One step = one pass of the hot path over the resident batch: per-protein k-mer sets
(extract + sort + dedup), repeat filter, pair planning, the tiled pair kernel over the whole
N x N upper triangle, and the canonical (p, q) edge sort — from packed residues resident in
HBM to the canonical edge list resident in HBM (rank 0).  Inputs are synthetic (SURVEY.md §8d,
config 3: N = 100,000, seed 3, len ~ N(300, 30^2), k = 7).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

CONFIGS = {
    # name: (N, seed, length law, k)
    "config3": (100_000, 3, 0, 7),
    "config2": (10_000, 2, 0, 7),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="config3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="oracle threads (0: min(16, cores))")
    return ap.parse_args()


def cpu_baseline(proteins, k, threads):
    """The reference algorithm restated in C (oracle/, posting-list expansion + class filter +
    per-pair collapse), timed on this host over the full workload."""
    from oracle.oracle import Oracle
    t0 = time.perf_counter()
    o = Oracle(proteins.residues, proteins.offsets, proteins.class_id, k=k, threads=threads)
    p, _, _ = o.pairs()
    dt = time.perf_counter() - t0
    n = proteins.n
    return {"value": n * (n - 1) / 2 / dt, "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": f"full workload ({n} proteins, k={k}): windows, sets, df, Σ C(df,2) "
                      f"posting-list expansion, class filter, per-pair collapse; {dt:.2f} s",
            "seconds": dt, "edges": int(len(p))}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import uniprot_kmer_based_clustering_amd as K
    from uniprot_kmer_based_clustering_amd.device import DevicePipeline
    from uniprot_kmer_based_clustering_amd.dist import distributed_step

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            print("run N>1 under torch.distributed.run (one process per GPU)", file=sys.stderr)
            sys.exit(2)
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    n, seed, law, k = CONFIGS[args.config]
    proteins = K.synth(n, seed, law)
    pipe = DevicePipeline(proteins, k, f"cuda:{local}")
    torch.cuda.synchronize()

    ev_pairs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                for _ in range(args.steps)]

    def one_step(i=None):
        timers = {"pairs": ev_pairs[i]} if i is not None else None
        if world > 1:
            return distributed_step(pipe, rank, world, timers=timers)
        pipe.build_sets()
        pipe.filter()
        pipe.plan()
        if timers:
            timers["pairs"][0].record()
        m = pipe.pairs()
        if timers:
            timers["pairs"][1].record()
        pipe.sort(m)
        return m

    for _ in range(args.warmup):
        one_step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        n_edges = one_step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    pair_ms = float(np.mean([a.elapsed_time(b) for a, b in ev_pairs]))
    ms = dt / args.steps * 1e3
    pairs_total = n * (n - 1) / 2
    rep_len = pipe.rep_len_host.astype(np.int64)
    set_len = pipe.set_len[:n].cpu().numpy().astype(np.int64)
    # algorithmic bytes of this rank's pair launches (4·(S_p + S_q) per pair
    # over the sets the kernel intersects, the repeat-filtered K(p)); rank share by item cost
    b_alg_all = 4.0 * (n - 1) * rep_len.sum()
    share = 1.0 / world
    achieved = b_alg_all * share / (pair_ms * 1e-3) / 1e9

    out = None
    if rank == 0:
        out = {
            "metric": "protein pairs/sec (+ edges/sec), 100k x 300aa synthetic, k=7",
            "value": pairs_total / (dt / args.steps),
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (SURVEY.md §8d generator, seeded; random families)",
            "config": {"workload": f"{args.config}: N={n}, seed={seed}, len~N(300,30^2), k={k}",
                       "proteins": n, "k": k, "pairs": int(pairs_total), "edges": int(n_edges),
                       "parallelism": f"pair-space tiles x{world}"},
            "edges_per_s": n_edges / (dt / args.steps),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "kernel": "pair_kernel", "kernel_ms": pair_ms,
                         "alg_bytes_per_launch": b_alg_all * share,
                         "alg_bytes_unfiltered_sets": 4.0 * (n - 1) * set_len.sum() * share},
        }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        out["cpu_baseline"] = cpu_baseline(proteins, k, threads)
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
