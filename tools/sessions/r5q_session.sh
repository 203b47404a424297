# Round 5: prefilter planes (SubmapDesc::pre_mask, CSM_PREFILTER = child
# levels): 2D parity tests with the prefilter at child levels 1 and 3, then
# one C3 step per setting (A/B twice, same accepted count required) and a
# CSM_KPROF pass with each setting.
set -u
O=gpurun_out/r5q
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
date +%T
CSM_PREFILTER=1,3 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_fast2d_gpu.py tests/test_c3_gpu.py tests/test_c3_ties.py tests/test_ties_walk.py > $O/tests_pre13.log 2>&1 \
  || { tail -40 $O/tests_pre13.log; exit 1; }
tail -1 $O/tests_pre13.log
date +%T
run() {  # label, then env assignments
  local label=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$label', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'], [round(x) for x in d['search_levels']['candidates_per_pair']])" | tee -a $O/ab_summary.txt
}
for k in 1 2; do
  run base CSM_NONE=1
  run pre1 CSM_PREFILTER=1
  run pre3 CSM_PREFILTER=3
  run pre13 CSM_PREFILTER=1,3
done
run pre2 CSM_PREFILTER=2
run pre123 CSM_PREFILTER=1,2,3
date +%T
for v in "base CSM_NONE=1" "pre13 CSM_PREFILTER=1,3"; do
  set -- $v
  env $2 CSM_PROFILE2D=1 CSM_AMD_LIB=$R/variants/kprof5/libcsm_amd.so timeout -k 10 300 python -u bench.py --no-cpu --no-rt --no-3d \
    --steps 1 --warmup 0 --c3-slice 16 > $O/kprof_$1.json 2> $O/kprof_$1.err || { tail -20 $O/kprof_$1.err; exit 1; }
  echo "$1"; grep "lines per gather" $O/kprof_$1.err | tail -2
done
date +%T
