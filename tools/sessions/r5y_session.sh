# Round 5: split-list scoring only in quad batches from the overflow stack
# (levels <= 2, raw-scan lists; variants/split) on the GPU:
# (1) the 2D parity tests against the oracle with the split build;
# (2) A/B of one C3 step launch against the HEAD build, twice, the same
# accepted count required.
set -u
O=gpurun_out/r5y
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
date +%T
CSM_AMD_LIB=$R/variants/split/libcsm_amd.so timeout -k 10 500 python -u -m pytest -x -v --timeout 200 \
  --timeout-method thread -m gpu tests/test_fast2d_gpu.py tests/test_c3_gpu.py tests/test_c3_ties.py \
  tests/test_ties_walk.py tests/test_golden.py > $O/split_tests.log 2>&1 || { tail -40 $O/split_tests.log; exit 1; }
tail -2 $O/split_tests.log
date +%T
run() {  # label, lib
  CSM_AMD_LIB=$2 timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$1', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
}
for k in 1 2; do
  run base $R/cartographer-1_amd/libcsm_amd.so
  run split $R/variants/split/libcsm_amd.so
done
date +%T
