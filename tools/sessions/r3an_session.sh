# Hybrid order: levels <= L depth-first through the overflow stack, C3 one step.
set -u
O=gpurun_out/r3an
mkdir -p $O
for lib in cartographer-1_amd variants/lifo1 variants/lifo2 variants/lifo3 cartographer-1_amd; do
  CSM_AMD_LIB=$PWD/$lib/libcsm_amd.so timeout -k 10 120 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 \
    > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$lib', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'], d['stack_high_water'])" | tee -a $O/ab_summary.txt
done
