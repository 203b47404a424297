"""Writes profiles/<round>/traffic_c5.json from the C5 probe's PMC passes
(tools/gpu_measure.sh c5: rocprofv3 --pmc, one counter group per pass, no
tracing): HBM-side bytes per fast3d_search dispatch = FETCH_SIZE (KB) x 1024
x 2 (the gfx950 correction, MI355X_MICROARCH.md), plus the texture-path and
L2 counters per dispatch, tied to bench.py's KERNEL3D_TAG.

    python tools/traffic3d_json.py PMC3D_DIR OUT_JSON KERNEL3D_TAG [PROBE_JSON]

PROBE_JSON (the probe's own output in the same session) adds the traffic
per algorithmic byte, so bench.py can scale it to launches of another size
(the C5 step's groups differ in size).
"""
import collections
import csv
import glob
import json
import sys


def main():
    pmc, out, tag = sys.argv[1:4]
    probe = json.load(open(sys.argv[4])) if len(sys.argv) > 4 else None
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{pmc}/p*/**/*counter_collection.csv", recursive=True):
        pass_id = f.split("/p", 1)[1].split("/", 1)[0] if "/p" in f else "0"
        for r in csv.DictReader(open(f)):
            if "fast3d_search" not in r.get("Kernel_Name", ""):
                continue
            per[(pass_id, r.get("Dispatch_Id", "0"))][r["Counter_Name"]] += float(r["Counter_Value"])
    if not per:
        sys.exit(f"no fast3d_search counters under {pmc}")
    sums, counts = collections.defaultdict(float), collections.defaultdict(int)
    for (_, _), cs in per.items():
        for k, v in cs.items():
            sums[k] += v
            counts[k] += 1
    avg = {k: sums[k] / counts[k] for k in sums}  # per dispatch, each counter over its own pass
    kb = avg.get("FETCH_SIZE")
    t = {"kernel": "fast3d_search (octet child levels, root cell lists)", "commit_kernel": tag,
         "workload": "C5 probe (tools/probe_c5.py): 500 nodes x 200 submaps, MatchFullSubmap",
         "counters_per_dispatch": avg, "gfx950_fetch_correction": 2.0,
         "traffic_bytes_per_launch": kb * 1024 * 2.0 if kb else None,
         "source": f"rocprofv3 --pmc passes (own passes, no tracing); {pmc}"}
    if probe and kb:
        launches_per_step = probe["roofline"]["launches"] / max(probe["steps"], 1)
        lookups_per_launch = probe["lookups_per_step"] / launches_per_step
        t["algorithmic_bytes_per_launch"] = lookups_per_launch
        t["traffic_bytes_per_algorithmic_byte"] = t["traffic_bytes_per_launch"] / lookups_per_launch
    json.dump(t, open(out, "w"), indent=1)
    print(json.dumps(t))


if __name__ == "__main__":
    main()
