"""Condenses a rocprofv3 --stats kernel_stats.csv into a short table (kernel names shortened,
template noise dropped).  Usage: python tools/prof_summary.py run_kernel_stats.csv [steps]
(or the results.db rocprofv3 writes without --output-format csv)"""
import csv
import re
import sqlite3
import sys


def short(name: str) -> str:
    n = re.sub(r"ROCPRIM_\d+_NS::", "", name)
    m = re.search(r"detail::(radix_sort_onesweep_\w+|scan_impl|partition_impl|transform_impl|"
                  r"run_length_encode\w*|trivial_runs\w*|reduce_by_key\w*|init_lookback_scan_state_kernel|"
                  r"radix_sort_\w+)", n)
    if "trampoline_kernel" in n and m:
        return "rocprim::" + m.group(1)
    if "init_lookback" in n:
        return "rocprim::init_lookback_scan_state_kernel"
    n = n.replace("(anonymous namespace)::", "")
    n = n.replace("void ", "")
    depth = 0
    for i, ch in enumerate(n):  # the parameter list: the first '(' outside template brackets
        depth += (ch == "<") - (ch == ">")
        if ch == "(" and depth == 0:
            return n[:i][:90]
    return n[:90]


def main():
    path = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 0
    if path.endswith(".db"):  # rocprofv3's default output: the kernels view of its database
        db = sqlite3.connect(path)
        q = "select name, count(*), sum(end - start) from kernels group by name"
        rows = [{"Name": n, "Calls": c, "TotalDurationNs": t} for n, c, t in db.execute(q)]
    else:
        rows = list(csv.DictReader(open(path)))
    agg = {}
    for r in rows:
        k = short(r["Name"])
        c, t = agg.get(k, (0, 0.0))
        agg[k] = (c + int(r["Calls"]), t + float(r["TotalDurationNs"]))
    tot = sum(t for _, t in agg.values())
    print(f"{'kernel':<72} {'calls':>6} {'total_ms':>9} {'avg_us':>9} {'%':>6}" +
          (f" {'ms/step':>8}" if steps else ""))
    for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
        line = f"{k:<72} {c:>6} {t / 1e6:>9.3f} {t / c / 1e3:>9.1f} {100 * t / tot:>6.2f}"
        if steps:
            line += f" {t / 1e6 / steps:>8.3f}"
        print(line)


if __name__ == "__main__":
    main()
