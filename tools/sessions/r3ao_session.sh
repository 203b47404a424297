# Hybrid order (levels <= 2 depth-first) as the default: full GPU suite, C2 step.
set -u
O=gpurun_out/r3ao
mkdir -p $O
bash tools/gpu_measure.sh $O tests || exit 1
tail -2 $O/gpu_tests.log
timeout -k 10 150 python -u bench.py --workload c2 --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/c2.json').read().strip().splitlines()[-1])
print('c2', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints_per_step'], d['errors_per_step'])" | tee $O/c2_summary.txt
