# Tie sorts on the parallel introsort: the 2D parity tests, a C3 step with
# the per-phase tie profile, then 3 C3 steps (r3ba: 12,421-12,441 pairs/s).
set -u
O=gpurun_out/r3bb
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_fast2d_gpu.py tests/test_c3_gpu.py tests/test_golden.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
CSM_PROFILE2D=1 timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/c3p.json 2> $O/c3_tie_profile.err || { tail -20 $O/c3_tie_profile.err; exit 1; }
grep "ties (ms)" $O/c3_tie_profile.err | grep -v "0 need" | tee $O/tie_summary.txt
C3_PROFILE=1 timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 3 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('3 steps', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), round(d['ms_per_step'], 1), d['accepted_constraints'], d['errors_per_step'], d['tied_pairs_rank0'])" | tee -a $O/ab_summary.txt
grep "host phases" $O/ab.err | tee -a $O/ab_summary.txt
