"""Benchmark of the k-mer pair path (BASELINE.json metric: protein pairs/sec + edges/sec,
100k x 300 aa synthetic proteins, k = 7, 1/2/4/8 MI355X).

One step = one pass of the hot path over the resident batch, packed residues in HBM ->
canonical (p, q, w) edge list in HBM: k-mer windows (radix-21 codes), the grouping of equal
k-mers (the reference's df pass), duplicate-window removal (K(p) dedup), the Σ C(df,2)
(k-mer, pair) incidence expansion with the AMR class filter, and the per-pair reduction to
w = |K(p) ∩ K(q)| in canonical order (Graph::new + remove_uninteresting_edges + combine_edges).
Inputs are synthetic (N = 100,000, seed 3, len ~ N(300, 30^2), k = 7).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--engine residues|postings|tiles]
  N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N [--split kmer|rows]

N > 1 (config 4): one process per GPU over RCCL, the k-mer split (dist.kmer_split_step): each rank
groups and expands its share of the k-mers, one all-to-all moves the pair keys to their row
owners, each rank reduces its rows.  The step ends with every rank holding the canonical edges of
its row range in HBM (rank order = canonical order); the gather of all of them onto one GPU is
timed apart (gather_ms) and is not part of the step.
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

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)

CONFIGS = {
    # name: (N, seed, length law, k); N = 0: the reference's own dataset (uniprot_arg.fasta)
    "config3": (100_000, 3, 0, 7),
    "config2": (10_000, 2, 0, 7),
    "config1": (0, 0, 0, 5),
    "config5": (1_000_000, 5, 1, 7),
}
WORKLOADS = {
    "config3": "config3: N=100000, seed=3, len~N(300,30^2), k=7",
    "config2": "config2: N=10000, seed=2, len~N(300,30^2), k=7",
    "config1": "config1: uniprot_arg.fasta (the reference's dataset, 10619 proteins), k=5",
    "config5": "config5 at k=7: N=1000000, seed=5, len log-uniform 50-2000, k=7, BLOSUM scores, row passes",
}


def load_batch(name):
    """The config's batch: synthetic (SURVEY.md §8d generator) or the reference's FASTA through
    the library's own ingest (kmp_read_fasta)."""
    import gzip
    import tempfile

    import uniprot_kmer_based_clustering_amd as K
    n, seed, law, _ = CONFIGS[name]
    if n:
        return K.synth(n, seed, law)
    with gzip.open(os.path.join(ROOT, "tests", "golden", "uniprot_arg.fasta.gz"), "rb") as f:
        raw = f.read()
    with tempfile.NamedTemporaryFile(suffix=".fasta") as t:
        t.write(raw)
        t.flush()
        return K.read_fasta(t.name)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="config3", choices=sorted(CONFIGS))
    ap.add_argument("--engine", default="residues", choices=["residues", "postings", "tiles"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="oracle threads (0: min(16, cores))")
    ap.add_argument("--score", default="blosum", choices=["blosum", "count"], help="config5: edge score")
    ap.add_argument("--split", default="kmer", choices=["kmer", "rows"], help="multi-GPU flow (N > 1)")
    return ap.parse_args()


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(proteins, k, threads):
    """The reference algorithm restated in C (oracle/: windows, per-protein sort + dedup, df,
    Σ C(df,2) posting-list expansion, class filter, per-pair collapse), timed on this host over
    the full workload: once single-threaded (the reference's threads = 1, run.sh's plumbing
    config) and once on `threads` cores.  `value` is the multi-core run."""
    from oracle.oracle import Oracle
    n = proteins.n
    runs = {}
    for t in (1, threads):
        t0 = time.perf_counter()
        o = Oracle(proteins.residues, proteins.offsets, proteins.class_id, k=k, threads=t)
        p, _, _ = o.pairs()
        runs[t] = (time.perf_counter() - t0, int(len(p)))
    dt, ne = runs[threads]
    return {"value": n * (n - 1) / 2 / dt, "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": f"full workload ({n} proteins, k={k}): windows, K(p) sort+dedup, df, Σ C(df,2) "
                      f"posting-list expansion, class filter, per-pair collapse; one run per thread count",
            "seconds": dt, "edges": ne,
            "single_thread": {"value": n * (n - 1) / 2 / runs[1][0], "seconds": runs[1][0], "cores": 1},
            "nproc": os.cpu_count(), "cpu_model": cpu_model()}


# names of the six stage-timing slots (kmp_postings_stats.stage_ms) per tail
STAGE_NAMES = {
    "rows": ("keys_level1", "buckets_level2", "group_expand", "pair_partition", "pair_sort_rle", "emit"),
}
STAGE_NAMES_DEFAULT = ("keys", "code_sort", "count", "write", "pair_sort", "rle_emit")


def stage_bytes(n_res, slots, n_inc, n_edges, n_uniq, tail="sort", n_win=None):
    """Algorithmic HBM bytes of each postings stage (one read of every input, one write of
    every output).  The six timing slots of the p-shard tail are keys, bucket sort,
    group + expand (pair keys written to their row ranges), -, row-range reduce (+ offsets),
    compaction.  'rows' (the default residue step): level-1 partition (residues in, one u64 key
    per window out), level-2 partition (keys in and out), group + expand (keys in, pair keys out),
    pair-key row-block histogram (pair keys in), scatter + LDS sort + run-length encode (pair keys
    in, runs out), emit (runs in, edges out)."""
    if tail == "rows":
        return {
            "keys_level1": n_res + 8 * n_win,
            "buckets_level2": 16 * n_win,
            "group_expand": 8 * n_win + 8 * n_inc,
            "pair_partition": 8 * n_inc,
            "pair_sort_rle": 8 * n_inc + 12 * n_uniq,
            "emit": 12 * n_uniq + 12 * n_edges,
        }
    if tail == "fused":
        return {
            "keys": n_res + 8 * slots,
            "code_sort": 16 * slots,
            "count": 8 * slots + 8 * n_inc,                 # keys in, pair keys out to the shards
            "write": 0,                                     # padding of the shard tails
            "pair_sort": 16 * n_inc,
            "rle_emit": 8 * n_inc + 12 * n_uniq + 12 * n_edges,
        }
    if tail == "pshard":
        return {
            "keys": n_res + 8 * slots,
            "code_sort": 16 * slots,
            "count": 8 * slots + 8 * n_inc,
            "write": 0,
            "pair_sort": 8 * n_inc + 12 * n_edges,
            "rle_emit": 24 * n_edges,
        }
    return {
        "keys": n_res + 8 * slots,                      # residues in, one u64 key per slot out
        "code_sort": 16 * slots,                        # keys read once + written once
        "count": 8 * slots + 8 * n_inc,                 # bucketed: keys in, pair keys out
        "write": 16 * n_inc,                            # shard gather (bucketed) / write pass (flat)
        "pair_sort": 16 * n_inc,                        # pair keys read once + written once
        "rle_emit": 8 * n_inc + 12 * n_uniq + 12 * n_edges,
    }


def pmc_traffic(stage: str):
    """HBM bytes per step of `stage` from the newest committed PMC table (profiles/r*_pmc_traffic.json,
    made by tools/pmc_traffic.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of
    this bench on config 3, FETCH_SIZE doubled per the gfx950 note in MI355X_MICROARCH.md)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
    if not files:
        return None, None
    st = json.load(open(files[-1]))["stages"].get(stage)
    return (st["bytes"] if st else None), os.path.relpath(files[-1], ROOT)


def bench_config5(args):
    """Config 5's batch at k = 7 through the C ABI (kmp_build_sets + kmp_pairs with BLOSUM scores):
    1,000,000 proteins of log-uniform lengths 50-2,000 (~5.3e8 windows) do not fit one call, so the
    library runs bounded-memory row passes.  One step = sets built from the resident
    residues + every pass + the canonical edge list and its scores copied into the edge set's host
    arrays (the C ABI hands edges to the caller: this line is PCIe-inclusive).  The k = 5 + 7 union at this size does not fit one GPU."""
    import uniprot_kmer_based_clustering_amd as K
    from uniprot_kmer_based_clustering_amd import _lib
    n, seed, law, k = CONFIGS["config5"]
    score = _lib.KMP_SCORE_BLOSUM if args.score == "blosum" else _lib.KMP_SCORE_COUNT
    proteins = K.synth(n, seed, law)
    with K.KmerPairEngine(0, 16) as e:
        e.load(proteins)

        def one_step():
            e.build_sets(k)
            with e.edge_set(score=score) as es:
                return len(es)
        for _ in range(args.warmup):
            one_step()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            n_edges = one_step()
        dt = time.perf_counter() - t0
        passes = e.last_passes
        c = e.counters()
    ms = dt / args.steps * 1e3
    pairs_total = n * (n - 1) / 2
    out = {"metric": "protein pairs/sec (+ edges/sec), 100k x 300aa synthetic, k=7",
           "value": pairs_total / (dt / args.steps), "unit": "pairs/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "strong",
           "vs_baseline": None, "dtype": "u32",
           "data": "synthetic (SURVEY.md §8d generator, seeded; log-uniform lengths 50-2000)",
           "config": {"workload": WORKLOADS["config5"], "proteins": n, "k": k, "pairs": int(pairs_total),
                      "edges": int(n_edges), "passes": passes, "score": args.score, "engine": "C ABI kmp_pairs",
                      "edges_in": "host (PCIe-inclusive)"},
           "edges_per_s": n_edges / (dt / args.steps),
           "counters": c,
           "roofline": None,
           "roofline_note": "per-stage roofline on the config3 line; this line times whole C-ABI calls"}
    if not args.no_cpu_baseline:
        from oracle.oracle import Oracle
        t0 = time.perf_counter()
        o = Oracle(proteins.residues, proteins.offsets, proteins.class_id, k=k, threads=16)
        p, _, _ = o.pairs()
        cdt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": pairs_total / cdt, "unit": "pairs/s", "cores": 16, "kind": "port",
                               "sample": f"full workload ({n} proteins, k={k}), 16 threads, no scores",
                               "seconds": cdt, "edges": int(len(p)), "nproc": os.cpu_count(),
                               "cpu_model": cpu_model()}
    print(json.dumps(out))


def main():
    args = parse()
    if args.config == "config5":
        if args.gpus != 1:
            print("config5 is a single-GPU line", file=sys.stderr)
            sys.exit(2)
        return bench_config5(args)
    import torch
    import torch.distributed as dist

    import uniprot_kmer_based_clustering_amd as K
    from uniprot_kmer_based_clustering_amd import _lib
    from uniprot_kmer_based_clustering_amd.device import DevicePipeline
    from uniprot_kmer_based_clustering_amd.dist import distributed_step, kmer_split_step

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world == 1 and args.gpus > 1:
        print("run N>1 under torch.distributed.run (one process per GPU)", file=sys.stderr)
        sys.exit(2)
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    _, seed, law, k = CONFIGS[args.config]
    proteins = load_batch(args.config)
    n = proteins.n
    pipe = DevicePipeline(proteins, k, f"cuda:{local}")
    torch.cuda.synchronize()
    postings = args.engine in ("residues", "postings")

    def one_step(timings=None, gather=False):
        if world > 1 and args.split == "kmer":
            return kmer_split_step(pipe, rank, world, gather=gather, timings=timings)
        if world > 1:
            return distributed_step(pipe, rank, world)
        return pipe.step(engine=args.engine)

    stage_sum = None
    if postings and world == 1:
        pipe.set_stage_timing(True)  # before the warm-up: the timed steps replay the same graph
    for _ in range(args.warmup):
        one_step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        n_edges = one_step()
        if postings and world == 1:
            st = np.array(pipe.postings_stats.stage_ms[:], dtype=np.float64)
            stage_sum = st if stage_sum is None else stage_sum + st
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if postings and world == 1:
        pipe.set_stage_timing(False)
    rank_info = None
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        # untimed: the edge total over the ranks, per-rank phase times, and the gather to rank 0
        ne = torch.tensor([n_edges], dtype=torch.int64, device=f"cuda:{local}")
        if args.split == "kmer":
            dist.all_reduce(ne)
            stt = pipe._split_state.bufs[3].clone()
            dist.all_reduce(stt)  # every rank's k-mers' statistics: the batch's
            split_stats = [int(x) for x in stt.tolist()]
            tims = []
            for _ in range(5):
                kmer_split_step(pipe, rank, world, timings=tims)
            ph = torch.tensor(np.mean(np.array(tims), axis=0), dtype=torch.float64, device=f"cuda:{local}")
            lo, hi = (int(x) for x in _lib.row_split(n, world)[rank:rank + 2])
            mine = torch.tensor([rank, lo, hi, n_edges, *ph.tolist()], dtype=torch.float64, device=f"cuda:{local}")
            allv = [torch.zeros_like(mine) for _ in range(world)]
            dist.all_gather(allv, mine)
            rank_info = [dict(zip(("rank", "row_lo", "row_hi", "edges", "expand_ms", "exchange_ms", "edges_ms"),
                                  [int(v) if i < 4 else v for i, v in enumerate(x.tolist())])) for x in allv]
            dist.barrier()
            torch.cuda.synchronize()
            g0 = time.perf_counter()
            tot = kmer_split_step(pipe, rank, world, gather=True)
            torch.cuda.synchronize()
            gather_ms = (time.perf_counter() - g0) * 1e3
            if rank == 0:
                assert tot == int(ne.item()), (tot, int(ne.item()))
        n_edges = int(ne.item())

    ms = dt / args.steps * 1e3
    pairs_total = n * (n - 1) / 2
    out = None
    if rank == 0:
        out = {
            "metric": "protein pairs/sec (+ edges/sec), 100k x 300aa synthetic, k=7",
            # config1 / config2 lines are extra workloads of the same metric (named in config)
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
            "data": ("synthetic (SURVEY.md §8d generator, seeded; protein families, 15 AMR classes)"
                     if CONFIGS[args.config][0] else "uniprot_arg.fasta (the reference's dataset)"),
            "config": {"workload": WORKLOADS[args.config],
                       "proteins": n, "k": k, "pairs": int(pairs_total), "edges": int(n_edges),
                       "engine": args.engine,
                       "parallelism": ("single GPU" if world == 1 else
                                       f"k-mer split x{world} (all-to-all of pair keys)" if args.split == "kmer"
                                       else f"row split x{world}")},
            "edges_per_s": n_edges / (dt / args.steps),
        }
        if rank_info is not None:
            # roofline of the whole multi-GPU step: its algorithmic bytes (the single-GPU stage
            # model over all ranks' work plus the pair keys crossing the links) against N x peak
            lens = np.diff(np.asarray(proteins.offsets, dtype=np.int64))
            n_win = int(np.maximum(lens - k + 1, 0).sum())
            n_inc = split_stats[6]
            byts = sum(stage_bytes(int(proteins.offsets[-1]), 0, n_inc, n_edges, n_edges, "rows", n_win).values())
            ach = byts / (ms * 1e-3) / 1e9
            out["roofline"] = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
                               "frac": ach / (HBM_PEAK_GBS * world), "traffic": None,
                               "kernel": f"whole step over {world} GPUs", "alg_bytes_per_step": byts,
                               "incidences": n_inc, "exchange_bytes": 8 * n_inc}
            out["ranks"] = rank_info
            out["gather_ms"] = gather_ms
            out["edges_layout"] = "row-sharded across ranks (rank order = canonical); gather_ms = step + gather"
        if args.engine in ("residues", "postings"):
            out["config"]["layout"] = pipe.last_layout()
            out["config"]["heavy_path"] = pipe.last_heavy()
            out["config"]["row_overflow_blocks"] = pipe.overflow_blocks()
        if stage_sum is not None:
            ps = pipe.postings_stats.as_dict()
            slots = int(_lib.lib().kmp_set_capacity(n, int(proteins.offsets[-1])))
            tail = pipe.last_tail()
            lens = np.diff(np.asarray(proteins.offsets, dtype=np.int64))
            n_win = int(np.maximum(lens - k + 1, 0).sum())  # windows = keys of the residue path
            byts = stage_bytes(int(proteins.offsets[-1]), slots, ps["incidences"], n_edges, ps["pairs"], tail,
                               n_win)
            names = STAGE_NAMES.get(tail, STAGE_NAMES_DEFAULT)
            stage_ms = dict(zip(names, (stage_sum / args.steps).tolist()))
            stages = {s: {"ms": stage_ms[s], "alg_bytes": byts[s],
                          "GBs": byts[s] / (stage_ms[s] * 1e-3) / 1e9 if stage_ms[s] > 0 else None}
                      for s in stage_ms}
            dom = max(stage_ms, key=stage_ms.get)
            ach = stages[dom]["GBs"]
            traffic, source = (pmc_traffic(dom) if args.config == "config3" and args.engine == "residues"
                               else (None, None))
            out["roofline"] = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": ach / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": source,
                               "traffic_over_alg": traffic / byts[dom] if traffic else None, "kernel": dom,
                               "kernel_ms": stage_ms[dom], "alg_bytes_per_launch": byts[dom],
                               "layout": pipe.last_layout(), "tail": tail, "stages": stages,
                               "step_alg_bytes": sum(byts.values()),
                               "step_GBs": sum(byts.values()) / (ms * 1e-3) / 1e9}
            # SURVEY.md §8d model: 4·(S_p + S_q) bytes per pair, i.e. a merge-intersection of every
            # pair's sets; the postings engine never touches non-sharing pairs, so this is an
            # effective figure far above the HBM peak
            b_model = 4.0 * (n - 1) * ps["sum_S"]
            out["roofline"]["pairs_model_GBs"] = b_model / (ms * 1e-3) / 1e9
            out["postings_stats"] = ps
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        out["cpu_baseline"] = cpu_baseline(proteins, k, threads)
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
