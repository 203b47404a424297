# Round 4: C3 queue placement A/B: each chunk's 4 submaps spread over all 8
# XCD queues (CSM_QUEUE_SPREAD=1) vs submap % 8; 8-submap chunks.
set -u
O=gpurun_out/r4o
mkdir -p $O
CSM_QUEUE_SPREAD=1 timeout -k 10 400 python -u -m pytest tests/test_fast2d_gpu.py tests/test_c3_ties.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests_spread.log 2>&1 \
  || { tail -60 $O/tests_spread.log; exit 1; }
tail -1 $O/tests_spread.log
for v in "0 4" "1 4" "0 4" "1 4" "0 8" "1 8"; do
  set -- $v
  CSM_QUEUE_SPREAD=$1 timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 --c3-chunk $2 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('spread=$1 chunk=$2', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
done
