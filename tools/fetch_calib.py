"""Joins tools/fetch_calib's known byte counts with a rocprofv3 FETCH_SIZE
pass over it: FETCH_SIZE x 1024 per dispatch against the bytes the dispatch
read and the distinct 32 / 64 / 128-byte units it touched.

    python tools/fetch_calib.py calib.json pmc_dir/run_counter_collection.csv [out.json]

The measured dispatches are the Stream / Scatter kernels in dispatch order
(every other one is the cache-flushing read before it); their positions in
that sequence are the "index" fields fetch_calib prints.
"""
import csv
import json
import sys


def main():
    calib = json.load(open(sys.argv[1]))
    rows = {}
    for r in csv.DictReader(open(sys.argv[2])):
        if r["Counter_Name"] != "FETCH_SIZE":
            continue
        name = r["Kernel_Name"]
        if "Stream" in name or "Scatter" in name:
            rows[int(r["Dispatch_Id"])] = rows.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    seq = [rows[k] for k in sorted(rows)]
    out = []
    for d in calib["dispatches"]:
        fetch = seq[d["index"]] * 1024.0
        e = {"pattern": d["name"], "bytes_read": d["bytes_read"], "fetch_size_bytes": fetch,
             "distinct_32B": d["u32"], "distinct_64B": d["u64"], "distinct_128B": d["u128"],
             "fetch_per_128B_line": fetch / (d["u128"] * 128.0),
             "fetch_per_64B_sector": fetch / (d["u64"] * 64.0),
             "fetch_per_32B_sector": fetch / (d["u32"] * 32.0)}
        out.append(e)
        print(f"{d['name']:14s} read {d['bytes_read'] / 2**20:9.1f} MiB  FETCH {fetch / 2**20:9.1f} MiB"
              f"  per 128B line {e['fetch_per_128B_line']:.3f}  per 64B {e['fetch_per_64B_sector']:.3f}"
              f"  per 32B {e['fetch_per_32B_sector']:.3f}")
    if len(sys.argv) > 3:
        json.dump({"source": sys.argv[2], "dispatches": out}, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
