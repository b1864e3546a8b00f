"""Benchmark of the k-mer pair path (BASELINE.json metric: protein pairs/sec + edges/sec,
100k x 300 aa synthetic proteins, k = 7, 1/2/4/8 MI355X).

One step = one pass of the hot path over the resident batch, packed residues in HBM ->
canonical (p, q, w) edge list in HBM: k-mer windows (radix-21 codes), the grouping of equal
k-mers (the reference's df pass), duplicate-window removal (K(p) dedup), the Σ C(df,2)
(k-mer, pair) incidence expansion with the AMR class filter, and the per-pair reduction to
w = |K(p) ∩ K(q)| in canonical order (Graph::new + remove_uninteresting_edges + combine_edges).
Inputs are synthetic (N = 100,000, seed 3, len ~ N(300, 30^2), k = 7).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--engine residues|postings|tiles]
  N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N [--split kmer|replicated|rows]
        [--start auto|keys|residues]

N > 1 (config 4): one process per GPU over RCCL, the k-mer split with a sharded start
(dist.sharded_split_step): rank r holds only the residues of its own chunks (about
1/N of the batch).  From 8 GPUs up (--start keys) it keys its windows once and an all-to-all sends
every key to the rank owning its k-mer's bins; below 8 (--start residues) the ranks all-gather the
residue slices (1 B per residue instead of 8 B per key) and every rank keys the whole batch, keeping
its bins.  Each rank groups and expands its k-mers, a second all-to-all moves the pair keys to
their row owners, each rank reduces its rows, and rank 0 gathers every rank's row block behind its
own (rank order = canonical order).  Both exchanges are inside the timed step, which ends with the
canonical list resident on rank 0; the row-sharded step without that gather is
reported as a breakdown.  --split replicated: every rank holds the whole batch and keys every window
(dist.kmer_split_step); --split rows: the row split.

--config config5: config 5 at its stated shape (1M proteins, k = 5 + 7, BLOSUM, streamed row
passes; bench_config5); N > 1 splits its rows over the ranks with no data-path collective.
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
    "config5": "config5: N=1000000, seed=5, len log-uniform 50-2000, k=5+7 combined, BLOSUM scores, streamed row passes",
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


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default 20; config5: 1)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 3; config5: 0)")
    ap.add_argument("--config", default="config3", choices=sorted(CONFIGS))
    ap.add_argument("--engine", default="residues", choices=["residues", "postings", "tiles"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sync", action="store_true",
                    help="one GPU: a synchronous call per step (kmp_dev_pairs_residues) instead of pipelined "
                         "submissions (kmp_dev_pairs_residues_submit / kmp_postings_wait)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="oracle threads of the all-cores run (0: every usable core)")
    ap.add_argument("--score", default="blosum", choices=["blosum", "count"], help="config5: edge score")
    ap.add_argument("--split", default="kmer", choices=["kmer", "replicated", "rows"], help="multi-GPU flow (N > 1)")
    ap.add_argument("--start", default="auto", choices=["auto", "keys", "residues"],
                    help="the sharded start's first exchange (--split kmer, N > 1): the key all-to-all, the "
                         "residue all-gather, or auto (keys from 8 GPUs up)")
    ap.add_argument("--rank-of", default=None, metavar="R/G",
                    help="config5, one GPU: stream only rank R's rows of a G-rank split (kmp_row_split), the "
                         "per-rank share of the N > 1 run, measured alone")
    ap.add_argument("--direct-tail", type=int, default=1, help="config5: fused reduction writes edges in place (A/B)")
    ap.add_argument("--flat-heavy", type=int, default=1, help="config5: passes expand frequent k-mers by rows (A/B)")
    return ap.parse_args(argv)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def usable_cores() -> dict:
    """The host's cores as this process can use them: nproc, the affinity mask, and the cgroup CPU
    quota (cpu.max) when one is set; `all` = the smallest (a box shares its host, so nproc
    overstates what a job gets)."""
    n = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = n
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(-(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    allc = min(n, aff, quota or n)
    return {"nproc": n, "affinity": aff, "cgroup_quota": quota, "all": allc}


def cpu_baseline(proteins, k, threads=0):
    """The reference algorithm restated in C (oracle/: windows, per-protein sort + dedup, df,
    Σ C(df,2) posting-list expansion, class filter, per-pair collapse), timed on this host over
    the full workload: single-threaded (the reference's threads = 1), on 32
    threads (run.sh:16's `threads`) and on every usable host core.  `value` is the all-cores run
    (`threads` overrides it)."""
    from oracle.oracle import Oracle
    n = proteins.n
    cores = usable_cores()
    allc = threads or cores["all"]
    runs = {}
    for t in sorted({1, 32, allc}):
        t0 = time.perf_counter()
        o = Oracle(proteins.residues, proteins.offsets, proteins.class_id, k=k, threads=t)
        p, _, _ = o.pairs()
        runs[t] = (time.perf_counter() - t0, int(len(p)))
    dt, ne = runs[allc]
    per = {str(t): {"value": n * (n - 1) / 2 / v[0], "seconds": v[0], "cores": t} for t, v in runs.items()}
    return {"value": n * (n - 1) / 2 / dt, "unit": "pairs/s", "cores": allc, "kind": "port",
            "sample": f"full workload ({n} proteins, k={k}): windows, K(p) sort+dedup, df, Σ C(df,2) "
                      f"posting-list expansion, class filter, per-pair collapse; runs at 1, 32 (run.sh:16) and "
                      f"{allc} (all usable cores) threads",
            "seconds": dt, "edges": ne, "runs": per,
            "single_thread": per["1"], "threads_32": per["32"],
            "host_cores": cores, "cpu_model": cpu_model()}


# names of the six stage-timing slots (kmp_postings_stats.stage_ms) of the bucketed residue step
STAGE_NAMES = ("keys_level1", "buckets_level2", "group_expand", "pair_partition", "pair_sort_rle", "emit")


def stage_bytes(n_res, n_inc, n_edges, n_uniq, n_win, tail="rows"):
    """Algorithmic HBM bytes of each stage of the residue step (one read of every input, one write
    of every output): level-1 partition (residues in, one u64 key per window out),
    level-2 partition (keys in and out), group + expand (keys in, pair keys out), then the tail.
    Counting tail ("rows"): pair-key row-block histogram (pair keys in), scatter + LDS sort +
    run-length encode (pair keys in, runs out), emit (runs in, edges out).  Fast tail ("fast"):
    scatter into the row-block regions (u64 pair keys in, u32 row-block keys out), then one reduce
    (u32 keys in, edges out); no emit."""
    if tail == "fast":
        return {
            "keys_level1": n_res + 8 * n_win,
            "buckets_level2": 16 * n_win,
            "group_expand": 8 * n_win + 8 * n_inc,
            "pair_partition": 12 * n_inc,
            "pair_sort_rle": 4 * n_inc + 12 * n_edges,
            "emit": 0,
        }
    return {
        "keys_level1": n_res + 8 * n_win,
        "buckets_level2": 16 * n_win,
        "group_expand": 8 * n_win + 8 * n_inc,
        "pair_partition": 8 * n_inc,
        "pair_sort_rle": 8 * n_inc + 12 * n_uniq,
        "emit": 12 * n_uniq + 12 * n_edges,
    }


def pmc_traffic(stage: str):
    """HBM bytes per step of `stage` from the newest committed PMC table (profiles/r*_pmc_traffic.json,
    made by tools/pmc_traffic.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of
    this bench on config 3; FETCH_SIZE divided by its measured factor, 0.5 at 4, 8 and 16 B per lane,
    profiles/r03_pmc_calib.json).  Returns (corrected bytes, raw counter bytes or None, source)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
    if not files:
        return None, None, None
    st = json.load(open(files[-1]))["stages"].get(stage)
    if not st:
        return None, None, os.path.relpath(files[-1], ROOT)
    return st["bytes"], st.get("raw_bytes"), os.path.relpath(files[-1], ROOT)


def config5_cpu_baseline(threads):
    """CPU baseline of config 5: the oracle's restatement of the reference algorithm
    (posting lists, per-row expansion of every k, class filter, per-pair collapse, the BLOSUM score
    summed per pair: oracle/kmp_oracle.c orc_build + orc_stream) on a bounded sample — the SAME
    workload law at N = 100,000 (config 5's lengths, seed 5, k = 5 + 7, BLOSUM), run in full (about
    30 s on 8 threads); pairs/s scales with the pair count since the incidences grow as N^2 too.
    The full 10^6 run took 817 s on 8 threads of this container (tests/golden/
    config5_1m_k5k7_blosum_digest.json)."""
    from oracle import oracle as O
    import uniprot_kmer_based_clustering_amd as K
    n = 100_000
    b = K.synth(n, 5, 1)
    t0 = time.perf_counter()
    orcs = [O.Oracle(b.residues, b.offsets, b.class_id, k=k, threads=threads) for k in (5, 7)]
    d = O.stream(orcs, threads=threads)
    dt = time.perf_counter() - t0
    return {"value": n * (n - 1) / 2 / dt, "unit": "pairs/s", "cores": threads, "kind": "port",
            "host_cores": usable_cores(),
            "sample": f"config-5 law at N={n} (seed 5, log-uniform 50-2000), k=5+7, BLOSUM, full run: "
                      f"{d['n_edges']} edges, {d['incidences']} incidences",
            "seconds": dt, "edges": d["n_edges"], "nproc": os.cpu_count(), "cpu_model": cpu_model(),
            "full_1m_seconds_8_threads_container": 817.4}


def bench_config5(args):
    """Config 5 at its stated shape (BASELINE.json configs[4]): 1,000,000 proteins of log-uniform
    lengths 50-2,000 (~5.3e8 windows), k = 5 and 7 combined in one reduction, BLOSUM score, through
    the C ABI's streamed passes (kmp_pairs_stream).  One step = sets per k built
    from the resident residues + every bounded-memory row pass: grouping + expansion of both k, the
    fused pair reduction, and the device summary of each pass's chunk (counters and digest) — each
    pass's canonical edges are resident in HBM when it is summarised (8.4e10 edges in all: the list
    never exists whole).  N > 1 (torch.distributed.run): each rank streams its kmp_row_split rows on
    its own GPU (kmp_ctx_set_rows), no data-path collective; value = all ranks' pairs / max time."""
    import uniprot_kmer_based_clustering_amd as K
    from uniprot_kmer_based_clustering_amd import _lib
    import torch
    import torch.distributed as dist
    n, seed, law, _ = CONFIGS["config5"]
    ks = (5, 7)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    steps = args.steps if args.steps is not None else 1
    warmup = args.warmup if args.warmup is not None else 0
    score = _lib.KMP_SCORE_BLOSUM if args.score == "blosum" else _lib.KMP_SCORE_COUNT
    proteins = K.synth(n, seed, law)
    lo, hi = (int(x) for x in _lib.row_split(n, world)[rank:rank + 2])
    emulated = None
    if args.rank_of and world == 1:  # one rank's share of a G-rank row split, on this one GPU
        er, eg = (int(x) for x in args.rank_of.split("/"))
        lo, hi = (int(x) for x in _lib.row_split(n, eg)[er:er + 2])
        emulated = {"rank": er, "of": eg, "row_lo": lo, "row_hi": hi}
    with K.KmerPairEngine(local, 16) as e:
        e.load(proteins)
        e.set_direct_tail(bool(args.direct_tail))
        e.set_flat_heavy(bool(args.flat_heavy))
        if world > 1 or emulated:
            e.set_rows(lo, hi)
        for _ in range(warmup):
            e.pairs_stream(ks, score=score)
        if world > 1:
            dist.barrier()
        # a marker kernel between the warm-up and the timed streams (untimed): profiles of this
        # command keep what follows it (tools/pmc_config5.py, tools/trace_after_marker.py)
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            sm = e.pairs_stream(ks, score=score)
        dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        keys = ("n_edges", "sum_w", "sum_score", "n_align", "incidences", "digest", "passes")
        v = torch.tensor([sm[k] & 0x7FFFFFFFFFFFFFFF if k == "digest" else sm[k] for k in keys],
                         dtype=torch.int64, device=f"cuda:{local}")
        allv = [torch.zeros_like(v) for _ in range(world)]
        dist.all_gather(allv, v)
        st = torch.tensor(list(sm["stage_ms"].values()), dtype=torch.float64, device=f"cuda:{local}")
        alls = [torch.zeros_like(st) for _ in range(world)]
        dist.all_gather(alls, st)
        ranks = [dict(zip(keys, [int(x) for x in a.tolist()]), stage_ms=dict(zip(sm["stage_ms"], b.tolist())),
                      row_lo=int(_lib.row_split(n, world)[r]), row_hi=int(_lib.row_split(n, world)[r + 1]))
                 for r, (a, b) in enumerate(zip(allv, alls))]
        tot = {k: sum(r[k] for r in ranks) for k in ("n_edges", "sum_w", "sum_score", "n_align", "incidences", "passes")}
        dist.destroy_process_group()
        if rank != 0:
            return
    else:
        ranks = None
        tot = {k: sm[k] for k in ("n_edges", "sum_w", "sum_score", "n_align", "incidences", "passes")}
    ms = dt / steps * 1e3
    pairs_total = n * (n - 1) / 2
    lens = np.diff(np.asarray(proteins.offsets, dtype=np.int64))
    win = {k: int(np.maximum(lens - k + 1, 0).sum()) for k in ks}
    stg = (ranks[0]["stage_ms"] if ranks else sm["stage_ms"])
    # algorithmic bytes per stage (one read of every input, one write of every output), per rank 0
    # or the single GPU: the expansion re-reads the grouped elements each pass, reads each key's
    # partner element and writes the u32 row-block key; the reduce reads each row-block key once and
    # writes the edges (p q w score w5 w7: 24 B)
    r0 = ranks[0] if ranks else {"incidences": sm["incidences"], "n_edges": sm["n_edges"], "passes": sm["passes"]}
    alg = {"expand_k0": 8 * win[5] * r0["passes"] + 8 * r0["incidences"],
           "reduce": 4 * r0["incidences"] + 24 * r0["n_edges"]}
    stages = {s: {"ms": stg[s], "alg_bytes": alg.get(s),
                  "GBs": alg[s] / (stg[s] * 1e-3) / 1e9 if s in alg and stg[s] > 0 else None} for s in stg}
    dom = max(alg, key=lambda s: stg[s])
    ach = stages[dom]["GBs"]
    # the dominant stage's HBM bytes per step from the newest committed config-5 PMC table
    # (tools/profile.sh traffic5: FETCH_SIZE / WRITE_SIZE passes over one step, corrected)
    traffic, traffic_src = None, None
    import glob
    pmc5 = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_config5.json")))
    if pmc5 and world == 1:
        try:
            traffic = json.load(open(pmc5[-1]))["stages"][dom]["bytes"]
            traffic_src = os.path.relpath(pmc5[-1], ROOT)
        except (OSError, KeyError, ValueError):
            traffic = None
    out = {"metric": "protein pairs/sec (+ edges/sec), config 5: 1M synthetic log-uniform 50-2000, k=5+7 combined, "
                     "BLOSUM-weighted",
           "value": pairs_total / (dt / steps), "unit": "pairs/s", "n_gpus": world, "steps": steps,
           "warmup": warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "strong",
           "vs_baseline": None, "dtype": "u32",
           "data": "synthetic (SURVEY.md §8d generator, seeded; log-uniform lengths 50-2000, 15 AMR classes)",
           "config": {"workload": WORKLOADS["config5"], "proteins": n, "k": list(ks), "pairs": int(pairs_total),
                      "edges": tot["n_edges"], "incidences": tot["incidences"], "passes": tot["passes"],
                      "score": args.score, "engine": "C ABI kmp_pairs_stream (fused k=5+7 reduction)",
                      "parallelism": "single GPU" if world == 1 else f"row split x{world} (kmp_ctx_set_rows per rank)",
                      "edges_in": "device, per pass (summarised on the device; never copied whole)"},
           "edges_per_s": tot["n_edges"] / (dt / steps),
           "incidences_per_s": tot["incidences"] / (dt / steps),
           "summary": {k: tot[k] for k in ("n_edges", "sum_w", "sum_score", "n_align")},
           "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": ach / HBM_PEAK_GBS if ach else None, "traffic": traffic,
                        "traffic_source": traffic_src,
                        "traffic_over_alg": traffic / alg[dom] if traffic else None, "kernel": dom,
                        "kernel_ms": stg[dom], "alg_bytes_per_launch": alg[dom], "stages": stages,
                        "note": "stage times summed over the passes (HIP events on the stream); "
                                "rank 0's when N > 1"}}
    if ranks:
        out["ranks"] = ranks
    if emulated:
        # one rank's rows measured alone: value and edges are that rank's share, not the batch's
        emulated["stage_ms"] = sm["stage_ms"]
        out["emulated_rank"] = emulated
        out["value"] = None
        out["note"] = "per-rank evidence (--rank-of): ms_per_step is one rank's stream of its kmp_row_split rows"
    if world == 1 and not emulated:
        if not ranks and "digest" in sm:
            out["digest"] = str(sm["digest"])
        if not args.no_cpu_baseline:
            out["cpu_baseline"] = config5_cpu_baseline(args.cpu_threads or usable_cores()["all"])
            # no published number: the ratio is to the reference's algorithm restated on
            # this box's host cores (a bounded sample of the same law, pairs/s)
            # vs_baseline stays null (no published number); the ratio to the CPU sample apart
            out["vs_cpu_baseline"] = out["value"] / out["cpu_baseline"]["value"]
    print(json.dumps(out))


def main(argv=None, dist_mod=None):
    """dist_mod (tests): a torch.distributed stand-in whose process group is already up (the GPU
    test of this N > 1 path runs two ranks on one GPU over gloo through host copies)."""
    args = parse(argv)
    if args.config == "config5":
        return bench_config5(args)
    if args.steps is None:
        args.steps = 20
    if args.warmup is None:
        args.warmup = 3
    import torch
    import torch.distributed as dist

    import uniprot_kmer_based_clustering_amd as K
    if dist_mod is not None:
        import uniprot_kmer_based_clustering_amd.dist as D
        dist = D.dist = dist_mod
    from uniprot_kmer_based_clustering_amd import _lib
    from uniprot_kmer_based_clustering_amd.device import DevicePipeline, ShardPipeline
    from uniprot_kmer_based_clustering_amd.dist import distributed_step, kmer_split_step, sharded_split_step, start_mode

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world == 1 and args.gpus > 1:
        print("run N>1 under torch.distributed.run (one process per GPU)", file=sys.stderr)
        sys.exit(2)
    torch.cuda.set_device(local)
    if world > 1 and dist_mod is None:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    _, seed, law, k = CONFIGS[args.config]
    proteins = load_batch(args.config)
    n = proteins.n
    sharded = world > 1 and args.split == "kmer"
    start = start_mode(args.start, world) if sharded else None
    if sharded:
        # the start state of SURVEY.md §8e: this GPU holds its chunks' residues only (plus offsets
        # and class ids); the host batch is generated whole by every rank, and only the slice moves
        pipe = ShardPipeline(proteins.residues, proteins.offsets, proteins.class_id, k, rank, world, f"cuda:{local}")
    else:
        pipe = DevicePipeline(proteins, k, f"cuda:{local}")
    torch.cuda.synchronize()
    postings = args.engine in ("residues", "postings")

    def one_step(timings=None, gather=False):
        if sharded:
            return sharded_split_step(pipe, rank, world, gather=gather, timings=timings, start=start)
        if world > 1 and args.split == "replicated":
            return kmer_split_step(pipe, rank, world, gather=gather, timings=timings)
        if world > 1:
            return distributed_step(pipe, rank, world)
        return pipe.step(engine=args.engine)

    stage_sum = None
    # stage times (the roofline): HIP events on the library's stream between its stages, measured in
    # an untimed pass after the timed steps, with graphs off — event-record nodes of a replayed HIP
    # graph keep the times of the graph's first launch on this stack (tools/pipe_probe.py: identical
    # stage times on every replay), so the timed steps carry no events.  BENCH_NO_STAGE_TIMING=1:
    # no stage pass (the line then carries no measured roofline)
    stage_timing = postings and world == 1 and os.environ.get("BENCH_NO_STAGE_TIMING") != "1"
    stage_steps = 10
    # one GPU, residues engine: the steps go out as pipelined submissions — step i + 1 is queued
    # behind step i, then step i is waited for and its read-back checked (a step that asks for a rerun
    # runs again at its wait) — so the device does not idle between steps while the host checks the
    # last one and launches the next; --sync: one synchronous call per step
    pipelined = world == 1 and args.engine == "residues" and not args.sync

    def run_steps(count, record=None):
        n = 0
        if not pipelined:
            for _ in range(count):
                # N > 1: the step ends with the canonical list on rank 0 (SURVEY.md §8d's clock), so
                # it includes the rank-order gather of every rank's rows
                n = one_step(gather=True)
                if record:
                    record()
            return n
        prev = None
        for _ in range(count):
            t = pipe.submit()
            if prev is not None:
                n = pipe.wait(prev)
                if record:
                    record()
            prev = t
        if prev is not None:
            n = pipe.wait(prev)
            if record:
                record()
        return n

    run_steps(args.warmup)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n_edges = run_steps(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if stage_timing:  # untimed: the stage times, plain launches with events between the stages
        pipe.set_graph(False)
        pipe.set_stage_timing(True)
        pipe.step(engine=args.engine)
        for _ in range(stage_steps):
            pipe.step(engine=args.engine)
            st = np.array(pipe.postings_stats.stage_ms[:], dtype=np.float64)
            stage_sum = st if stage_sum is None else stage_sum + st
        pipe.set_stage_timing(False)
        pipe.set_graph(True)
    sync_ms = None
    if pipelined:  # untimed: the synchronous call's latency per step, for the record
        for _ in range(3):
            pipe.step(engine=args.engine)
        torch.cuda.synchronize()
        s0 = time.perf_counter()
        for _ in range(10):
            pipe.step(engine=args.engine)
        torch.cuda.synchronize()
        sync_ms = (time.perf_counter() - s0) / 10 * 1e3
    rank_info = None
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        # untimed: per-rank phase times and the step without the gather (the breakdown)
        ne = torch.tensor([n_edges], dtype=torch.int64, device=f"cuda:{local}")
        dist.broadcast(ne, 0)  # rank 0 holds the whole list: its count is the total
        if args.split in ("kmer", "replicated"):
            step_fn = (lambda *a_, **kw: sharded_split_step(*a_, start=start, **kw)) if sharded else kmer_split_step
            st_ = pipe._split_state
            stt = st_.bufs[3].clone()
            dist.all_reduce(stt)  # every rank's k-mers' statistics: the batch's
            split_stats = [int(x) for x in stt.tolist()]
            tims = []
            for _ in range(5):
                own_edges = step_fn(pipe, rank, world, timings=tims)  # without the gather: this rank's rows
            ph = torch.tensor(np.mean(np.array(tims), axis=0), dtype=torch.float64, device=f"cuda:{local}")
            lo, hi = (int(x) for x in _lib.row_split(n, world)[rank:rank + 2])
            # bytes this rank sends to the other ranks per step (equal splits: its own region stays)
            # the start exchange: the padded key regions, or the rank's residue slice to every peer;
            # the residue start's pair keys travel in its rebuilt batch's split state
            if start == "residues":
                lo_, hi_, _ = pipe.own_residues()
                kx = (world - 1) * (hi_ - lo_)
                px = (world - 1) * st_.cap * 8
            else:
                kx = (world - 1) * st_.kcap * 8 if sharded else 0
                px = (world - 1) * st_.cap * 8
            res_mb = pipe.res.numel() / 1e6
            mine = torch.tensor([rank, lo, hi, own_edges, kx, px, res_mb, *ph.tolist()], dtype=torch.float64,
                                device=f"cuda:{local}")
            allv = [torch.zeros_like(mine) for _ in range(world)]
            dist.all_gather(allv, mine)
            names = (("rank", "row_lo", "row_hi", "edges", "start_exchange_bytes", "pair_exchange_bytes",
                      "residues_resident_MB") +
                     (("keys_ms", "start_exchange_ms", "group_ms", "pair_exchange_ms", "edges_ms") if sharded else
                      ("expand_ms", "exchange_ms", "edges_ms")))
            rank_info = [dict(zip(names, [int(v) if i < 6 else v for i, v in enumerate(x.tolist())])) for x in allv]
            dist.barrier()
            torch.cuda.synchronize()
            g0 = time.perf_counter()
            for _ in range(5):
                step_fn(pipe, rank, world, gather=False)
            torch.cuda.synchronize()
            dist.barrier()
            t = torch.tensor([(time.perf_counter() - g0) / 5 * 1e3], dtype=torch.float64, device=f"cuda:{local}")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            no_gather_ms = float(t.item())
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
                                       (f"k-mer split x{world}, sharded start (all-to-all of keys, then of pair keys)"
                                        if start == "keys" else
                                        f"k-mer split x{world}, sharded start (all-gather of residue slices, "
                                        "all-to-all of pair keys)")
                                       if args.split == "kmer" else
                                       f"k-mer split x{world}, replicated start (all-to-all of pair keys)"
                                       if args.split == "replicated" else f"row split x{world}")},
            "edges_per_s": n_edges / (dt / args.steps),
        }
        if world == 1:
            out["config"]["steps_issued"] = ("pipelined submissions (two outstanding; each step waited for and "
                                             "its read-back checked)" if pipelined else "one synchronous call per step")
            if sync_ms is not None:
                out["ms_per_step_sync"] = sync_ms
        if rank_info is not None:
            # roofline of the whole multi-GPU step: its algorithmic bytes (the single-GPU stage
            # model over all ranks' work plus the pair keys crossing the links) against N x peak
            lens = np.diff(np.asarray(proteins.offsets, dtype=np.int64))
            n_win = int(np.maximum(lens - k + 1, 0).sum())
            n_inc = split_stats[6]
            byts = sum(stage_bytes(int(proteins.offsets[-1]), n_inc, n_edges, n_edges, n_win).values())
            ach = byts / (ms * 1e-3) / 1e9
            out["roofline"] = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
                               "frac": ach / (HBM_PEAK_GBS * world), "traffic": None,
                               "kernel": f"whole step over {world} GPUs", "alg_bytes_per_step": byts,
                               "incidences": n_inc,
                               # algorithmic exchange bytes: one 8-B key per window (sharded start) and
                               # one 8-B pair key per incidence, the (N-1)/N of them that leave a rank
                               "exchange_bytes": int((8 * n_win * (start == "keys") + 8 * n_inc) * (world - 1) / world
                                                     + (world - 1) * int(proteins.offsets[-1]) * (start == "residues"))}
            out["ranks"] = rank_info
            out["step_without_gather_ms"] = no_gather_ms
            out["gather_ms"] = ms - no_gather_ms
            out["edges_layout"] = ("canonical list on rank 0 at the end of each timed step (the ranks' row blocks "
                                   "gathered in rank order); step_without_gather_ms = the row-sharded step alone")
        if args.engine in ("residues", "postings"):
            out["config"]["layout"] = pipe.last_layout()
            out["config"]["heavy_path"] = pipe.last_heavy()
            out["config"]["row_overflow_blocks"] = pipe.overflow_blocks()
        tail = pipe.last_tail() if args.engine in ("residues", "postings") else None
        if stage_sum is not None and tail in ("rows", "fast"):  # the bucketed step's six stages
            ps = pipe.postings_stats.as_dict()
            lens = np.diff(np.asarray(proteins.offsets, dtype=np.int64))
            n_win = int(np.maximum(lens - k + 1, 0).sum())  # windows = keys of the residue path
            byts = stage_bytes(int(proteins.offsets[-1]), ps["incidences"], n_edges, ps["pairs"], n_win, tail)
            names = STAGE_NAMES
            stage_ms = dict(zip(names, (stage_sum / stage_steps).tolist()))
            stages = {s: {"ms": stage_ms[s], "alg_bytes": byts[s],
                          "GBs": byts[s] / (stage_ms[s] * 1e-3) / 1e9 if stage_ms[s] > 1e-4 else None}
                      for s in stage_ms}
            dom = max(stage_ms, key=stage_ms.get)
            ach = stages[dom]["GBs"]
            traffic, traffic_raw, source = (pmc_traffic(dom) if args.config == "config3" and args.engine == "residues"
                                            else (None, None, None))
            out["roofline"] = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": ach / HBM_PEAK_GBS, "traffic": traffic, "traffic_raw": traffic_raw,
                               "traffic_source": source,
                               "traffic_over_alg": traffic / byts[dom] if traffic else None, "kernel": dom,
                               "kernel_ms": stage_ms[dom], "alg_bytes_per_launch": byts[dom],
                               "layout": pipe.last_layout(), "tail": tail, "stages": stages,
                               "step_alg_bytes": sum(byts.values()),
                               "step_GBs": sum(byts.values()) / (ms * 1e-3) / 1e9,
                               "stage_timing": f"HIP events between the stages, {stage_steps} untimed steps with "
                                               "plain launches after the timed ones (graph event nodes keep "
                                               "their first launch's times on this stack)"}
            # SURVEY.md §8d model: 4·(S_p + S_q) bytes per pair, i.e. a merge-intersection of every
            # pair's sets; the postings engine never touches non-sharing pairs, so this is an
            # effective figure far above the HBM peak
            b_model = 4.0 * (n - 1) * ps["sum_S"]
            out["roofline"]["pairs_model_GBs"] = b_model / (ms * 1e-3) / 1e9
            out["postings_stats"] = ps
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(proteins, k, args.cpu_threads)
        # the reference has no published number: the ratio is to its algorithm
        # restated on this box's host cores, measured in this run
        # vs_baseline stays null: BASELINE.md holds no published number for this metric; the ratio to
        # the reference's algorithm restated on this box's host cores is reported apart
        out["vs_cpu_baseline"] = out["value"] / out["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1 and dist_mod is None:
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
