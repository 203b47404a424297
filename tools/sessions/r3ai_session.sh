# Gathers in flight per lane (quad / hex unroll) and one rotation per item,
# C3 one step each.
set -u
O=gpurun_out/r3ai
mkdir -p $O
run() {  # lib, env
  env $2 CSM_AMD_LIB=$PWD/$1/libcsm_amd.so timeout -k 10 120 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 \
    > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$1 [$2]', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
}
run cartographer-1_amd "" || exit 1
run variants/q4h4 "" || exit 1
run variants/q16h4 "" || exit 1
run variants/q8h2 "" || exit 1
run variants/q8h8 "" || exit 1
run cartographer-1_amd "CSM_ROT_CHUNK=1" || exit 1
run cartographer-1_amd "" || exit 1
