"""Summarises tools/pmc_profile.sh output: per-dispatch counters of one kernel,
averaged over its dispatches."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(outdir, kernel="fast2d_search"):
    vals = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(outdir, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and "search_v" in r["Kernel_Name"] or (
                    kernel in r["Kernel_Name"] and kernel.endswith("_v2") is False):
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in sorted(vals):
        v = vals[k]
        print(f"{k:40s} {sum(v) / len(v):16.4g}   (n={len(v)})")


if __name__ == "__main__":
    main(*sys.argv[1:])
