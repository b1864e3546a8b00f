"""Per-access-width FETCH_SIZE / WRITE_SIZE factors from tools/pmc_calib under two rocprofv3 PMC
passes: factor = counter bytes (KiB x 1024) / bytes the kernel moves.  tools/pmc_traffic.py divides
each kernel's counters by the factor of its access width.
Usage: python tools/pmc_calib.py FETCH_counter_collection.csv WRITE_counter_collection.csv BYTES out.json"""
import collections
import csv
import json
import sys


def per_kernel(path):
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("void ", "").split("(")[0]
        out[name].append(float(r["Counter_Value"]) * 1024.0)
    return out


def main():
    fetch, write = per_kernel(sys.argv[1]), per_kernel(sys.argv[2])
    nbytes = float(sys.argv[3])
    res = {"bytes_per_dispatch": nbytes, "read": {}, "write": {}}
    for name, vals in fetch.items():
        if name.startswith("read_kernel"):
            width = {"unsigned int": 4, "uint2": 8, "uint4": 16}[name[name.index("<") + 1:-1]]
            res["read"][width] = {"FETCH_SIZE_factor": sorted(vals)[len(vals) // 2] / nbytes,
                                  "dispatches": len(vals)}
    for name, vals in write.items():
        if name.startswith("write_kernel"):
            width = {"unsigned int": 4, "uint2": 8, "uint4": 16}[name[name.index("<") + 1:-1]]
            res["write"][width] = {"WRITE_SIZE_factor": sorted(vals)[len(vals) // 2] / nbytes,
                                   "dispatches": len(vals)}
    print(json.dumps(res, indent=1))
    json.dump(res, open(sys.argv[4], "w"), indent=1)


if __name__ == "__main__":
    main()
