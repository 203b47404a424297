# Round 5: out-of-range lanes of fast2d_search's gathers. A CSM_KPROF pass
# counts, per gather instruction and child level, the active lanes and those
# whose entry is off the plane or past the node's list (issued at the
# out-of-range offset); then one C3 step with CSM_MASK_OOB=1 (those lanes
# skip the load) against HEAD, A/B twice, the same accepted count required.
set -u
O=gpurun_out/r5s
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
date +%T
CSM_PROFILE2D=1 CSM_AMD_LIB=$R/variants/kprof5/libcsm_amd.so timeout -k 10 300 python -u bench.py --no-cpu --no-rt --no-3d \
  --steps 1 --warmup 0 --c3-slice 16 > $O/kprof.json 2> $O/kprof.err || { tail -20 $O/kprof.err; exit 1; }
grep "per gather" $O/kprof.err | tail -4
run() {  # label, lib
  CSM_AMD_LIB=$2 timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$1', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
}
for k in 1 2; do
  run base $R/cartographer-1_amd/libcsm_amd.so
  run maskoob $R/variants/maskoob/libcsm_amd.so
done
date +%T
# Coalescing defaults (3 leaders, whole-grid share) confirmed against the
# round-5 alternatives, and the concurrent-results check.
drun() {
  local label=$1; shift
  env "$@" timeout -k 10 240 ./tools/dropin_threads 2000 0.55 > $O/d.json 2> $O/d.err || { tail -5 $O/d.err; exit 1; }
  echo "$label $(tail -1 $O/d.json)" | tee -a $O/dropin_summary.txt
}
drun default CSM_NONE=1
drun leaders2-share0 CSM_COALESCE_LEADERS=2 CSM_COALESCE_SHARE=0
drun leaders4 CSM_COALESCE_LEADERS=4
drun leaders2 CSM_COALESCE_LEADERS=2
drun default-again CSM_NONE=1
timeout -k 10 240 ./tools/dropin_threads 0 0.55 --check > $O/check.json 2>&1 || { cat $O/check.json; exit 1; }
tail -1 $O/check.json | tee -a $O/dropin_summary.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_threading_gpu.py > $O/threading.log 2>&1 || { tail -30 $O/threading.log; exit 1; }
tail -1 $O/threading.log
date +%T
