# Occupancy with fuller batches: workgroups per CU (register budget, LDS ring)
# against cluster-list room (CSM_CAPC_PCT), C3 one step.
set -u
O=gpurun_out/r3aa
mkdir -p $O
run() {  # lib, env
  env $2 CSM_PROFILE2D=1 CSM_AMD_LIB=$PWD/$1/libcsm_amd.so timeout -k 10 120 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 \
    > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$1 [$2]', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
  grep -m1 "fast2d launch" $O/ab.err | tee -a $O/ab_summary.txt
}
run cartographer-1_amd "" || exit 1
run cartographer-1_amd "CSM_CAPC_PCT=40" || exit 1
run variants/w7 "CSM_CAPC_PCT=50" || exit 1
run variants/w7 "CSM_CAPC_PCT=40" || exit 1
run variants/w7r128 "CSM_CAPC_PCT=40" || exit 1
run variants/w8r128 "CSM_CAPC_PCT=35" || exit 1
run variants/w8r128 "CSM_CAPC_PCT=30" || exit 1
run cartographer-1_amd "" || exit 1
