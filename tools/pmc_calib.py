"""Per-access-width FETCH_SIZE / WRITE_SIZE factors from tools/pmc_calib under two rocprofv3 PMC
passes: factor = counter bytes (KiB x 1024) / bytes the kernel moves.  tools/pmc_traffic.py divides
each kernel's counters by the factor of its access width.
Usage: python tools/pmc_calib.py FETCH_counter_collection.csv WRITE_counter_collection.csv BYTES out.json"""
import collections
import csv
import json
import sys


def width_of(name):
    """access width of a calibration kernel: read_kernel<unsigned int> / <HIP_vector_type<unsigned int, 2u>> / 4u"""
    if "2u>" in name:
        return 8
    if "4u>" in name:
        return 16
    return 4


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
            width = width_of(name)
            res["read"][width] = {"FETCH_SIZE_factor": sorted(vals)[len(vals) // 2] / nbytes,
                                  "dispatches": len(vals)}
    for name, vals in write.items():
        if name.startswith("write_kernel"):
            width = width_of(name)
            res["write"][width] = {"WRITE_SIZE_factor": sorted(vals)[len(vals) // 2] / nbytes,
                                   "dispatches": len(vals)}
    print(json.dumps(res, indent=1))
    json.dump(res, open(sys.argv[4], "w"), indent=1)


if __name__ == "__main__":
    main()
