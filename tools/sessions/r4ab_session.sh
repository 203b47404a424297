# Round 4: C3 queue placement within a submap's queues: alternating pairs vs
# contiguous node blocks (CSM_QUEUE_SPLIT=block), one step each.
set -u
O=gpurun_out/r4ab
mkdir -p $O
CSM_QUEUE_SPLIT=block timeout -k 10 400 python -u -m pytest tests/test_c3_ties.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in alt block alt block; do
  CSM_QUEUE_SPLIT=$v timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('split=$v', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
done
