# C3 with 1 vs 2 host workers per rank (each its own context / stream, so a
# chunk's tie resolution and records overlap the next chunk's search): 3 steps
# each, alternating.
set -u
O=gpurun_out/r3ba
mkdir -p $O
for w in 1 2 1 2; do
  C3_PROFILE=1 timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 3 --warmup 1 --c3-workers $w > $O/ab.json 2> $O/ab_w$w.err || { tail -20 $O/ab_w$w.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('workers $w', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), round(d['ms_per_step'], 1), d['accepted_constraints'], d['errors_per_step'], d['tied_pairs_rank0'])" | tee -a $O/ab_summary.txt
  grep "host phases" $O/ab_w$w.err | tee -a $O/ab_summary.txt
done
