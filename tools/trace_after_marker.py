"""Kernel summary of the dispatches after the last marker kernel (torch's spin_kernel, which
bench.py --config config5 launches between its warm-up and timed streams) in a rocprofv3
--kernel-trace CSV, so the summary describes the timed step alone.
Usage: python tools/trace_after_marker.py run_kernel_trace.csv"""
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"]]
    rows = rows[marks[-1] + 1:] if marks else rows
    agg = {}
    for r in rows:
        k = short(r["Kernel_Name"])
        c, t = agg.get(k, (0, 0.0))
        agg[k] = (c + 1, t + int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = sum(t for _, t in agg.values())
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e6 if rows else 0.0
    print(f"# {len(rows)} dispatches after the marker; first start to last end {span:.1f} ms; kernel time {tot / 1e6:.1f} ms")
    print(f"{'kernel':<72} {'calls':>6} {'total_ms':>9} {'avg_us':>9} {'%':>6}")
    for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"{k:<72} {c:>6} {t / 1e6:>9.3f} {t / c / 1e3:>9.1f} {100 * t / tot:>6.2f}")


if __name__ == "__main__":
    main()
