"""Per-wave SQ counters per kernel from rocprofv3 --pmc passes (each pass carries SQ_WAVES).
Usage: python tools/sq_summary.py PASS_DIR [PASS_DIR ...]"""
import collections
import csv
import glob
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402


def main():
    for d in sys.argv[1:]:
        print(f"# {d}")
        for f in glob.glob(f"{d}/**/run_counter_collection.csv", recursive=True):
            agg = collections.defaultdict(list)
            for r in csv.DictReader(open(f)):
                agg[(short(r["Kernel_Name"])[-60:], r["Counter_Name"])].append(float(r["Counter_Value"]))
            for n in sorted({k[0] for k in agg}):
                w = sum(agg[(n, "SQ_WAVES")]) / max(1, len(agg[(n, "SQ_WAVES")]))
                per = {c: round(sum(v) / len(v) / max(w, 1), 1) for (m, c), v in agg.items() if m == n and c != "SQ_WAVES"}
                print(n, per, "waves", w)


if __name__ == "__main__":
    main()
