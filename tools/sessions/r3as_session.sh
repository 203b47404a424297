# Overflow-stack bottom in LDS: 128 entries (default) vs 1 (variants/d0, the
# previous all-global stack) vs 256 (variants/d256); C3 one step each.
set -u
O=gpurun_out/r3as
mkdir -p $O
for lib in cartographer-1_amd variants/d0 variants/d256 cartographer-1_amd variants/d0; do
  CSM_PROFILE2D=1 CSM_AMD_LIB=$PWD/$lib/libcsm_amd.so timeout -k 10 120 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 \
    > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$lib', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
  grep -m1 "fast2d launch" $O/ab.err | tee -a $O/ab_summary.txt
done
