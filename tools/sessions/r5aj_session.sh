# Round 5 closing bench: the default bench.py run (no profiler) at HEAD.
set -u
O=gpurun_out/r5aj
mkdir -p $O
date +%T
timeout -k 10 900 python -u bench.py > $O/bench_full.json 2> $O/bench_full.err || { tail -30 $O/bench_full.err; exit 1; }
date +%T
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r5aj/bench_full.json").read().strip().splitlines()[-1])
f = d["fast3d"]
print("c3", round(d["value"], 1), "kernel", round(d["roofline"]["kernel_ms_avg"], 1), "parity", d["parity_sample"]["mismatched_pose"],
      "c5", round(f["value"]), round(f["ms_per_step"], 1), "rt2d", round(d["rt2d"]["cabi_ms_per_scan_match_median"], 4))
PY
