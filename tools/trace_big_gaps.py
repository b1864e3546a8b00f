"""The largest idle gaps between kernels after the last marker kernel (torch's spin_kernel) of a
rocprofv3 --kernel-trace CSV: where a step waits on the host.
Usage: python tools/trace_big_gaps.py run_kernel_trace.csv [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"]]
rows = rows[marks[-1] + 1:] if marks else rows
n = int(sys.argv[2]) if len(sys.argv) > 2 else 15
gaps = []
for a, b in zip(rows, rows[1:]):
    g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e6
    gaps.append((g, a["Kernel_Name"][:60], b["Kernel_Name"][:60]))
print(f"total gap {sum(max(g, 0) for g, _, _ in gaps):.1f} ms over {len(gaps)} intervals")
for g, a, b in sorted(gaps, reverse=True)[:n]:
    print(f"{g:9.2f} ms  after {a}  before {b}")
