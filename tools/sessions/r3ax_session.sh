# C3 with the next chunk's pyramids built on a second context during the
# search: one step x2 (one step at the previous host loop: 12,660-12,725
# pairs/s, profiles/r3ap, r3au), then the 2-rank rehearsal.
set -u
O=gpurun_out/r3ax
mkdir -p $O
for k in 1 2; do
  C3_PROFILE=1 timeout -k 10 120 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('prefetch', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), round(d['ms_per_step'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
  grep "host phases" $O/ab.err | tee -a $O/ab_summary.txt
done
bash tools/gpu_measure.sh $O gloo2 || exit 1
python3 -c "
import json; d=json.loads([l for l in open('$O/rehearsal_2rank.json') if l.startswith('{')][-1]); print('2 ranks', d['value'], d['chunks'], d['chunks_claimed'], d['chunks_max_rank'], d['errors_per_step'], d['accepted_constraints'])" | tee -a $O/ab_summary.txt
