# Round 5: last knob checks on C3 with the flattened lanes: y-fastest child
# order (CSM_XFAST=0), power-of-two batches (CSM_POW2_BATCH=1), and 6 quad
# gathers in flight (CSM_U_QUAD=6, 568.3 vs 569.3-570.3 ms in r5be), as
# variant builds (variants/g_*). One C3 step each, HEAD interleaved.
set -u
O=gpurun_out/r5bj
mkdir -p $O
run() {  # label, lib ('' = in-tree), then env assignments
  local label=$1 lib=$2; shift 2
  env ${lib:+CSM_AMD_LIB=$lib} "$@" timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$label', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
}
run head ''
run xfast0 variants/g_xfast0/libcsm_amd.so
run pow2 variants/g_pow2/libcsm_amd.so
run uq6 variants/g_uq6/libcsm_amd.so
run head2 ''
run uq6b variants/g_uq6/libcsm_amd.so
run head3 ''
run uq6c variants/g_uq6/libcsm_amd.so
