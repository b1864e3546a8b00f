"""Per-rank device time of the two multi-GPU flows, emulated on one GPU (diagnostic):
  rows   the row split: every rank's kmp_dev_pairs_rows over its kmp_row_split rows;
  kmer   the k-mer split with a replicated start: every rank's kmp_dev_split_expand (every window
         keyed, its share of the bucket hash range kept, pair keys routed by row owner) and
         kmp_dev_split_edges over the keys it would receive;
  sharded  the k-mer split with a sharded start (bench.py --gpus N): every rank holds its residue
         slice, kmp_dev_split_keys (its windows keyed once, sent to the bins' owners),
         kmp_dev_split_group over the keys it would receive, kmp_dev_split_edges.
For G = 2, 4, 8 each rank's stages are timed in turn on its own DevicePipeline (G = 1: the fused
step, which kmer_split_step runs at world 1); the slowest
rank bounds the step.  Exchanges (all-to-all, gather) are not included.  Each phase is reported as
wall time (host clock over back-to-back calls: launches and the edges phase's read-back included)
and device time (HIP events around each call on its stream).
python tools/time_dist_rank.py [config3|config1] [rows|kmer|sharded] [G ...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import load_batch, CONFIGS  # noqa: E402
from uniprot_kmer_based_clustering_amd import _lib  # noqa: E402
from uniprot_kmer_based_clustering_amd.device import DevicePipeline, ShardPipeline  # noqa: E402
from uniprot_kmer_based_clustering_amd.dist import row_ranges  # noqa: E402


def timed(fn, reps=10):
    """(wall ms per call, device ms per call): wall = host clock over reps back-to-back calls;
    device = HIP events recorded around each call on the stream its kernels run on."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps * 1e3
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return wall, sum(a.elapsed_time(b) for a, b in ev) / reps


def kmer_ranks(b, k, g):
    if g == 1:  # dist.kmer_split_step at world 1: nothing to exchange, the fused step
        pipe = DevicePipeline(b, k, "cuda:0")
        w, d = timed(lambda: pipe.step())
        return [{"rows": [0, b.n], "fused_step": True, "ms": w, "dev_ms": d, "send_MB": 0.0, "sent_keys": 0,
                 "edges": pipe.n_edges}]
    pipes = [DevicePipeline(b, k, "cuda:0") for _ in range(g)]
    cap = max(4096, pipes[0].total // 4 // (g * g))
    learn = None
    for _ in range(4):  # learn the capacities
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
    recvs = [torch.cat([sends[r][d * cap:(d + 1) * cap] for r in range(g)]) for d in range(g)]
    per = []
    for r, (lo, hi) in enumerate(row_ranges(b.n, g)):
        t1, d1 = timed(lambda: pipes[r].split_expand(r, g, cap, sends[r], flags[r], stats[r]))
        t2, d2 = timed(lambda: pipes[r].split_edges(recvs[r], lo, hi))
        per.append({"rows": [lo, hi], "expand_ms": t1, "edges_ms": t2, "ms": t1 + t2,
                    "dev_expand_ms": d1, "dev_edges_ms": d2, "dev_ms": d1 + d2,
                    "send_MB": g * cap * 8 / 1e6, "sent_keys": int(stats[r][6].item()), "edges": pipes[r].n_edges})
    return per


def sharded_ranks(b, k, g):
    if g == 1:
        return kmer_ranks(b, k, 1)
    pipes = [ShardPipeline(b.residues, b.offsets, b.class_id, k, r, g, "cuda:0") for r in range(g)]
    kcap = int(pipes[0].span.key_cap)
    cap = max(4096, pipes[0].total // 4 // (g * g))
    learn = None
    for _ in range(6):  # learn the capacities
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
    recvs = [torch.cat([sends[r][d * cap:(d + 1) * cap] for r in range(g)]) for d in range(g)]
    per = []
    for r, (lo, hi) in enumerate(row_ranges(b.n, g)):
        p = pipes[r]
        # the rank's whole step without its exchanges, back to back as in dist.sharded_split_step
        # (keys, group, edges; the host's launches of a phase overlap the GPU's work of the one
        # before, and the step ends with the edges phase's synchronisation); device time from
        # events around the sequence, the phases split at events between them
        def seq(ev=None):
            if ev:
                ev[0].record()
            p.split_keys(r, g, kcap, ksend[r], flags[r])
            if ev:
                ev[1].record()
            p.split_group(krecv[r], kcap, r, g, cap, sends[r], flags[r], stats[r])
            if ev:
                ev[2].record()
            p.split_edges(recvs[r], lo, hi)
            if ev:
                ev[3].record()
        for _ in range(3):
            seq()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            seq()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / 10 * 1e3
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(10)]
        for ev in evs:
            seq(ev)
        torch.cuda.synchronize()
        d0, d1, d2 = (sum(ev[i].elapsed_time(ev[i + 1]) for ev in evs) / len(evs) for i in range(3))
        t0, t1, t2 = d0, d1, wall - d0 - d1
        # bytes this rank sends to the others in each exchange (its own region stays local)
        kbytes = (g - 1) * kcap * 8
        pbytes = (g - 1) * cap * 8
        per.append({"rows": [lo, hi], "keys_ms": t0, "group_ms": t1, "edges_ms": t2, "ms": wall,
                    "dev_keys_ms": d0, "dev_group_ms": d1, "dev_edges_ms": d2, "dev_ms": d0 + d1 + d2,
                    "residue_slice_MB": p.res.numel() / 1e6, "key_exchange_MB": kbytes / 1e6,
                    "pair_exchange_MB": pbytes / 1e6, "key_cap": kcap, "pair_cap": cap,
                    "sent_pair_keys": int(stats[r][6].item()), "edges": p.n_edges})
    return per


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "config3"
    mode = sys.argv[2] if len(sys.argv) > 2 else "kmer"
    k = CONFIGS[name][3]
    b = load_batch(name)
    out = {"config": name, "mode": mode, "n": b.n, "ranks": {}}
    full = DevicePipeline(b, k, "cuda:0")
    out["single_gpu_ms"], out["single_gpu_dev_ms"] = timed(lambda: full.step(), 20)
    print("single", round(out["single_gpu_ms"], 3), "device", round(out["single_gpu_dev_ms"], 3), flush=True)
    del full
    for g in [int(x) for x in sys.argv[3:]] or (1, 2, 4, 8):
        if mode == "kmer":
            per = kmer_ranks(b, k, g)
        elif mode == "sharded":
            per = sharded_ranks(b, k, g)
        else:
            per = []
            for r, (lo, hi) in enumerate(row_ranges(b.n, g)):
                pipe = DevicePipeline(b, k, "cuda:0")
                w, d = timed(lambda: pipe.rows(lo, hi))
                per.append({"rows": [lo, hi], "ms": w, "dev_ms": d, "edges": pipe.n_edges})
                del pipe
        out["ranks"][g] = {"max_ms": max(x["ms"] for x in per), "max_dev_ms": max(x["dev_ms"] for x in per),
                           "per_rank": per}
        print(g, "wall", round(out["ranks"][g]["max_ms"], 3), [round(x["ms"], 3) for x in per],
              "device", round(out["ranks"][g]["max_dev_ms"], 3), [round(x["dev_ms"], 3) for x in per], flush=True)
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
