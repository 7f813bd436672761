"""Summarise rocprofv3 --pmc CSVs: per-kernel average counter value per dispatch."""
import collections
import csv
import glob
import sys

def summary(paths, kernel="cl_exec_kernel"):
    agg = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for p in paths:
        for r in csv.DictReader(open(p)):
            if kernel not in r["Kernel_Name"]:
                continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r["Dispatch_Id"])
    return {k: agg[k] / len(disp[k]) for k in agg}

if __name__ == "__main__":
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    kern = sys.argv[2] if len(sys.argv) > 2 else "cl_exec_kernel"
    s = summary(glob.glob(f"{root}/*/p_counter_collection.csv"), kern)
    for k in sorted(s):
        print(f"{k:28s} {s[k]:16.1f}")
