"""Config-5 HBM traffic of the fused reduce and the expansion stages from two rocprofv3 PMC passes
(FETCH_SIZE, WRITE_SIZE) over one bench step (`bench.py --config config5`), summed over every
dispatch of the step (58 passes), with the gfx950 correction of tools/pmc_traffic.py.
Usage: python tools/pmc_config5.py FETCH.csv WRITE.csv out.json"""
import collections
import csv
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_traffic import calib  # noqa: E402
from prof_summary import short  # noqa: E402

STAGE = {  # bench_config5's stage names
    "pt_hist_kernel": "reduce", "pt_tscan_kernel": "reduce", "pt_scatter_kernel": "reduce",
    "pt_split_kernel": "reduce", "pt_window_count_kernel": "reduce", "pt_reduce_count_kernel": "reduce",
    "pt_reduce_write_kernel": "reduce", "pt_reduce_scored_kernel": "reduce", "pt_emit_kernel": "reduce",
    "heavy_flat_kernel": "expand", "heavy_rows_kernel": "expand", "bucket_small_kernel": "expand", "bucket_large_kernel": "expand",
    "edge_digest_kernel": "summary",
}


def load(path):
    """Per kernel, the counter summed over the dispatches after the last marker kernel (torch's
    spin_kernel, which bench.py launches between the warm-up and the timed stream), or over every
    dispatch of a run without one."""
    rows = list(csv.DictReader(open(path)))
    marks = [int(r["Dispatch_Id"]) for r in rows if "spin_kernel" in r["Kernel_Name"]]
    after = max(marks) if marks else -1
    out = collections.defaultdict(float)
    for r in rows:
        if int(r["Dispatch_Id"]) <= after or "spin_kernel" in r["Kernel_Name"]:
            continue
        out[short(r["Kernel_Name"]).removeprefix("void ").split("<")[0]] += float(r["Counter_Value"]) * 1024.0
    return out


def main():
    fetch, write = load(sys.argv[1]), load(sys.argv[2])
    rf, wf = calib()
    kernels, stages = {}, collections.defaultdict(lambda: {"read_bytes": 0.0, "write_bytes": 0.0, "bytes": 0.0})
    for k in sorted(set(fetch) | set(write)):
        rb, wb = fetch.get(k, 0.0) / rf, write.get(k, 0.0) / wf
        kernels[k] = {"read_bytes": rb, "write_bytes": wb, "bytes": rb + wb}
        st = STAGE.get(k.split("(")[0])
        if st:
            for f, v in (("read_bytes", rb), ("write_bytes", wb), ("bytes", rb + wb)):
                stages[st][f] += v
    out = {"config": "config5", "per": "one bench step (every pass)", "correction": f"FETCH_SIZE / {rf}, WRITE_SIZE / {wf}",
           "stages": stages, "kernels": kernels}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    for st, v in stages.items():
        print(st, {f: round(x / 1e9, 2) for f, x in v.items()}, "GB")


if __name__ == "__main__":
    main()
