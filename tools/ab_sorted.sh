#!/bin/bash
# A/B: batch nodes in pop order (default) vs sorted by (yo, xo) (CSM_SORT_BATCH).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/ab
cd $R
export CSM_AMD_LIB_T=$R/variants/sorted/libcsm_amd.so
CSM_AMD_LIB=$CSM_AMD_LIB_T timeout -k 10 400 python -u -m pytest tests/test_fast2d_gpu.py tests/test_constraint_builder.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/sorted_tests.log 2>&1 || { echo "sorted tests failed"; tail -30 gpurun_out/ab/sorted_tests.log; exit 1; }
tail -1 gpurun_out/ab/sorted_tests.log
CSM_AMD_LIB=$CSM_AMD_LIB_T timeout -k 10 300 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > gpurun_out/ab/sorted.json 2> gpurun_out/ab/sorted.err || { echo "sorted bench failed"; tail -20 gpurun_out/ab/sorted.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > gpurun_out/ab/base.json 2> gpurun_out/ab/base.err || { echo "base bench failed"; tail -20 gpurun_out/ab/base.err; exit 1; }
python - <<'PY'
import json
for k in ("base", "sorted"):
    d = json.load(open(f"gpurun_out/ab/{k}.json"))
    print(k, round(d["value"], 1), "pairs/s", round(d["roofline"]["kernel_ms_avg"], 1), "ms", d["accepted_constraints_per_step"])
PY
echo AB_OK
