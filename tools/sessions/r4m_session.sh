# Round 4: FIFO ring in (child row, parent, column) order (CSM_PUSH_ROWS=1):
# parity, then C3 one-step A/B.
set -u
O=gpurun_out/r4m
mkdir -p $O
CSM_PUSH_ROWS=1 timeout -k 10 400 python -u -m pytest tests/test_fast2d_gpu.py tests/test_c3_ties.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests_rows.log 2>&1 \
  || { tail -60 $O/tests_rows.log; exit 1; }
tail -1 $O/tests_rows.log
for pr in 0 1 0 1; do
  CSM_PUSH_ROWS=$pr timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('push_rows=$pr', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
done
