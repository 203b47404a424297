# Round 5 measurement set: the default bench.py run under
# rocprofv3 --kernel-trace --stats (fast2d_search_v4's average duration
# against the bench's own HIP-event kernel_ms_avg, same run).
set -u
O=gpurun_out/r5t
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
date +%T
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_threading_gpu.py \
  > $O/threading.log 2>&1 || { tail -30 $O/threading.log; exit 1; }
tail -1 $O/threading.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 780 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o bench \
  --output-format csv -- python3 $R/bench.py > $R/$O/bench_full.json 2> $R/$O/bench_full.err) \
  || { tail -30 $O/bench_full.err; exit 1; }
date +%T
python3 - <<'PY'
import csv, glob, json
d = json.loads(open("gpurun_out/r5t/bench_full.json").read().strip().splitlines()[-1])
print("value", d["value"], "kernel_ms_avg", d["roofline"]["kernel_ms_avg"], "parity", d["parity_sample"])
for f in glob.glob("gpurun_out/r5t/trace/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "fast2d_search_v4" in r["Name"] or "fast3d_search" in r["Name"]:
            print(r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6, "ms avg")
PY
