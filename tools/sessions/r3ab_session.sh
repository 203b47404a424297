# Stats out of the batch loop's LDS atomics: C3 one step x2; phase profile (KPROF build).
set -u
O=gpurun_out/r3ab
mkdir -p $O
for k in 1 2; do
  timeout -k 10 120 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('default', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'], [round(x) for x in d['search_levels']['candidates_per_pair']])" | tee -a $O/ab_summary.txt
done
CSM_PROFILE2D=1 CSM_AMD_LIB=$PWD/variants/kprof/libcsm_amd.so timeout -k 10 120 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/kprof.json 2> $O/kprof.err || { tail -20 $O/kprof.err; exit 1; }
grep "phases" $O/kprof.err | tail -2 | tee -a $O/ab_summary.txt
