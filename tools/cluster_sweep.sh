#!/bin/bash
# A/B of the per-level scan cluster sizes (CSM_CLUSTER, log2 per child level)
# on the C2 bench workload; one JSON summary line per setting.
set -e
mkdir -p gpurun_out
for c in "$@"; do
  CSM_CLUSTER="$c" timeout -k 10 120 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 \
    > gpurun_out/sweep.json 2> gpurun_out/sweep.err
  python - "$c" <<'PY'
import json, sys
d = json.load(open("gpurun_out/sweep.json"))
print(json.dumps({"cluster": sys.argv[1], "pairs_per_s": round(d["value"], 1),
                  "kernel_ms": round(d["roofline"]["kernel_ms_avg"], 1),
                  "lookups_per_pair": d["roofline"]["algorithmic_bytes_per_launch"] / 25000,
                  "cands": [round(c) for c in d["search_levels"]["candidates_per_pair"][:9]]}))
PY
done
