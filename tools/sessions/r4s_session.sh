# Round 4: C3 one-step sweeps of the search knobs with queue spreading on
# (rotations per item, hex levels, list room, workgroups per CU).
set -u
O=gpurun_out/r4s
mkdir -p $O
run() {
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$*', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
}
run CSM_NONE=1
run CSM_ROT_CHUNK=1
run CSM_ROT_CHUNK=3
run CSM_HEX_LEVELS=8
run CSM_HEX_LEVELS=8,6,4
run CSM_CAPC_PCT=60
run CSM_WG_PER_CU=5
run CSM_NONE=1
bash tools/gpu_measure.sh gpurun_out/r4s c3trace || exit 1
ls -la gpurun_out/r4s/c3trace
timeout -k 10 300 python -u -m pytest tests/test_threading_gpu.py -m gpu -q --timeout 250 --timeout-method thread > $O/tests_threads.log 2>&1 || { tail -30 $O/tests_threads.log; exit 1; }
tail -1 $O/tests_threads.log
