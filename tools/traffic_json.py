"""Writes profiles/<round>/traffic_<workload>.json from a FETCH_SIZE pass
(rocprofv3 --pmc FETCH_SIZE, its own pass, no tracing) of the C2/C3 bench leg:
HBM-side bytes per fast2d_search_v4 launch = FETCH_SIZE (KB) x 1024 x 2 (the
gfx950 x2 correction of MI355X_MICROARCH.md's HBM/rocprofv3 section).

    python tools/traffic_json.py PMC_DIR OUT_JSON KERNEL_TAG LAUNCH_MS [c3 NODES CHUNK SUBMAPS]
"""
import collections
import csv
import glob
import json
import sys


def main():
    pmc, out, tag, launch_ms = sys.argv[1], sys.argv[2], sys.argv[3], float(sys.argv[4])
    per = collections.defaultdict(float)
    launches = set()
    for f in glob.glob(f"{pmc}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            # The search's own symbol (the tie-enumeration launches are the
            # kCollect = true instantiation).
            name = r.get("Kernel_Name", "")
            if "fast2d_search_v4" in name and "true>" not in name.split(",")[2] and \
                    r["Counter_Name"] == "FETCH_SIZE":
                per[r.get("Dispatch_Id", "0")] += float(r["Counter_Value"])
                launches.add(r.get("Dispatch_Id", "0"))
    if not per:
        sys.exit("no FETCH_SIZE rows for fast2d_search_v4")
    kb = sum(per.values()) / len(per)
    t = {"kernel": "fast2d_search_v4 (v5: FIFO order, hex planes, scan clusters)", "commit_kernel": tag,
         "workload": "C2 bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 0",
         "nodes": 500, "submaps_per_rank": 50, "min_score": 0.55, "search_depth": 0,
         "launches": len(per), "fetch_size_kb_per_launch": kb, "gfx950_fetch_correction": 2.0,
         "traffic_bytes_per_launch": kb * 1024 * 2.0, "launch_ms": launch_ms,
         "source": f"rocprofv3 --pmc FETCH_SIZE (own pass, no tracing); {pmc}"}
    if len(sys.argv) > 5 and sys.argv[5] == "c3":
        nodes, chunk, submaps = (int(v) for v in sys.argv[6:9])
        del t["submaps_per_rank"]
        t.update({"workload": f"C3 chunk launches: bench.py --workload c3 --c3-submaps {submaps} "
                              f"--no-cpu --steps 1 --warmup 0 (the first {submaps} submaps of the "
                              f"2000 x 1000 queue)",
                  "nodes": nodes, "chunk": chunk, "submaps": submaps})
        t["workload"] = (f"C3 chunk launches: bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 0 "
                         f"--c3-slice {submaps} (the first {submaps} submaps of the 2000 x 1000 queue, "
                         f"{chunk}-submap chunks)")
    json.dump(t, open(out, "w"), indent=1)
    print(json.dumps(t))


if __name__ == "__main__":
    main()
