# Overflow-stack bottom in LDS at 6 workgroups per CU: 64 entries with the
# list room cut to 70% of npad, against the all-global stack (variants/d0).
set -u
O=gpurun_out/r3at
mkdir -p $O
run() {
  env $2 CSM_PROFILE2D=1 CSM_AMD_LIB=$PWD/$1/libcsm_amd.so timeout -k 10 120 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 \
    > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$1 [$2]', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
  grep -m1 "fast2d launch" $O/ab.err | tee -a $O/ab_summary.txt
}
run variants/d64 "CSM_CAPC_PCT=70" || exit 1
run variants/d0 "CSM_CAPC_PCT=70" || exit 1
run variants/d0 "" || exit 1
run variants/d64 "CSM_CAPC_PCT=70" || exit 1
