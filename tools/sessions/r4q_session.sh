# Round 4: C3 chunk 8 / 16 with 1 and 2 host workers (queue spreading on).
set -u
O=gpurun_out/r4q
mkdir -p $O
for v in "8 1" "8 2" "16 1" "16 2" "4 1"; do
  set -- $v
  timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 --c3-chunk $1 --c3-workers $2 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('chunk=$1 workers=$2', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
done
