"""Prints the last N kernels of a rocprofv3 kernel trace with their durations and the idle gap
before each (us).  Usage: python tools/trace_gaps.py <run_kernel_trace.csv> [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
prev = None
busy = gaps = 0.0
for r in rows[-n:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev is not None else 0.0
    prev = e
    busy += (e - s) / 1000
    gaps += max(gap, 0.0)
    print(f"{gap:8.1f} {(e - s) / 1000:8.1f}  {r['Kernel_Name'].replace('(anonymous namespace)::', '')[:90]}")
print(f"busy {busy:.1f} us, gaps {gaps:.1f} us")
