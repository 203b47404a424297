"""Sums rocprofv3 counter CSVs (one dir per pass) for one kernel name substring."""
import collections
import csv
import glob
import sys

root, kernel = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "fast2d"
tot = collections.defaultdict(float)
for f in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if kernel in r.get("Kernel_Name", ""):
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(tot.items()):
    print(f"{k:40s} {v:.4e}")
