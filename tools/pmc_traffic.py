"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; KiB per
dispatch).  gfx950 correction: FETCH_SIZE counts half of the bytes read, WRITE_SIZE all of them
— measured at 4, 8 and 16 B per lane against a known byte count (tools/pmc_calib.hip,
profiles/r03_pmc_calib.json; MI355X_MICROARCH.md §HBM states it for 16 B) — so reads are divided
by the calibrated factor (0.5) and writes taken as is.  Both raw and corrected bytes are written.
Usage: python tools/pmc_traffic.py FETCH.csv WRITE.csv [out.json]"""
import collections
import csv
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402


def load(path):
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        out[(short(r["Kernel_Name"]), int(r["Grid_Size"]))].append(float(r["Counter_Value"]) * 1024.0)
    return out


def calib():
    """(read factor, write factor) from the committed calibration (8-B-per-lane lines; every width
    measured the same)"""
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "r03_pmc_calib.json")
    try:
        c = json.load(open(path))
        return c["read"]["8"]["FETCH_SIZE_factor"], c["write"]["8"]["WRITE_SIZE_factor"]
    except (OSError, KeyError, ValueError):
        return 0.5, 1.0


def main():
    fetch, write = load(sys.argv[1]), load(sys.argv[2])
    rf, wf = calib()
    rows = []
    for key in sorted(set(fetch) | set(write), key=lambda k: -(sum(fetch.get(k, [0])) + sum(write.get(k, [0])))):
        f, w = fetch.get(key, []), write.get(key, [])
        n = max(len(f), len(w))
        fraw = sum(f) / max(1, len(f))
        wraw = sum(w) / max(1, len(w))
        fb, wb = fraw / rf, wraw / wf
        rows.append({"kernel": key[0], "grid": key[1], "dispatches": n, "read_bytes": fb, "write_bytes": wb,
                     "bytes": fb + wb, "raw_read_bytes": fraw, "raw_write_bytes": wraw, "raw_bytes": fraw + wraw})
    print(f"{'kernel':<52} {'grid':>10} {'disp':>5} {'read MB':>9} {'write MB':>9}")
    for r in rows[:20]:
        print(f"{r['kernel'][:52]:<52} {r['grid']:>10} {r['dispatches']:>5} {r['read_bytes']/1e6:>9.1f} "
              f"{r['write_bytes']/1e6:>9.1f}")
    # per-step traffic of the residue step's stages (bench.py STAGE_NAMES["rows"]); one
    # level-1 scatter dispatch per step
    calls = max([r["dispatches"] for r in rows if r["kernel"].split("<")[0] in
                 ("bp_scatter1_kernel", "bp_scatter1l_kernel", "bp_scatter1p_kernel")] or [1])
    # the fast tail (round 4): the capped scatter is the pair partition, the reduce writes the edges
    # (its emit share is in pair_sort_rle); the counting tail as before
    by_kernel = {
        "chunk_first_kernel": "keys_level1", "bp_hist1_kernel": "keys_level1", "bp_colscan_kernel": "keys_level1",
        "bp_scatter1_kernel": "keys_level1", "bp_scatter1l_kernel": "keys_level1", "bp_h1t_kernel": "keys_level1",
        "chunk_desc_kernel": "keys_level1", "bp_scatter1p_kernel": "keys_level1",
        "pt_scatter_capped_kernel": "pair_partition", "pt_reduce_fast_kernel": "pair_sort_rle",
        "pt_reduce_dense_kernel": "pair_sort_rle",
        "bp_scatter2g_kernel": "buckets_level2", "bp_colsum_kernel": "keys_level1", "bp_colprefix_kernel": "keys_level1",
        "bp_hist2_kernel": "buckets_level2", "bp_scan2_kernel": "buckets_level2",
        "bp_scatter2_kernel": "buckets_level2", "bp_scatter2c_kernel": "buckets_level2",
        "bp_cur_clear_kernel": "buckets_level2", "step_clear_kernel": "keys_level1", "step_pack_kernel": "emit",
        "pt_hist_kernel": "pair_partition", "pt_colscan_kernel": "pair_partition",
        "pt_scatter_kernel": "pair_sort_rle", "pt_reduce_kernel": "pair_sort_rle",
        "pt_offsets_kernel": "emit", "pt_emit_kernel": "emit", "fused_pack_kernel": "emit",
    }

    def stage(r):
        k = r["kernel"].removeprefix("void ").split("<")[0]
        if "bucket_small_kernel" in k or "bucket_large_kernel" in k:
            return "group_expand"
        return by_kernel.get(k)

    stages = collections.defaultdict(lambda: {"read_bytes": 0.0, "write_bytes": 0.0, "raw_bytes": 0.0})
    for r in rows:
        st = stage(r)
        if st:
            per_step = r["dispatches"] / calls
            stages[st]["read_bytes"] += r["read_bytes"] * per_step
            stages[st]["write_bytes"] += r["write_bytes"] * per_step
            stages[st]["raw_bytes"] += r["raw_bytes"] * per_step
    for st in stages.values():
        st["bytes"] = st["read_bytes"] + st["write_bytes"]
    print("per-step stage traffic (MB):", {k: round(v["bytes"] / 1e6, 1) for k, v in stages.items()})
    if len(sys.argv) > 3:
        json.dump({"calls": calls, "correction": f"FETCH_SIZE / {rf:.4f}, WRITE_SIZE / {wf:.4f} "
                   "(profiles/r03_pmc_calib.json); KiB counters; raw_* uncorrected",
                   "stages": stages, "kernels": rows}, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
