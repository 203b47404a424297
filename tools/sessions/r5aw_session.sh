# Round 5: more workgroups per CU on C3. Variant libraries built with a
# smaller register budget (CSM_V4_WAVES 7 / 8: 72 / 64 VGPRs, 22 / 26
# spilled) and per-rotation tables sized for 2 rotations (static LDS 9296 ->
# 8288 B); the LDS then allows 7 per CU at capc 640 (CSM_CAPC_PCT=58) or 8
# at one rotation per item. One C3 step each.
set -u
O=gpurun_out/r5aw
mkdir -p $O
run() {  # label, lib ('' = in-tree), then env assignments
  local label=$1 lib=$2; shift 2
  env ${lib:+CSM_AMD_LIB=$lib} CSM_PROFILE2D=1 "$@" timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  grep -m1 "fast2d launch" $O/ab.err | tee -a $O/ab_summary.txt
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$label', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
}
W8=variants/w8/libcsm_amd.so
W7=variants/w7/libcsm_amd.so
run head ''
run w8_r2 $W8
run w8_r1 $W8 CSM_ROT_CHUNK=1
run w8_r1_6 $W8 CSM_ROT_CHUNK=1 CSM_WG_PER_CU=6
run w7_c58 $W7 CSM_CAPC_PCT=58
run w7_r1 $W7 CSM_ROT_CHUNK=1
run head_r1 '' CSM_ROT_CHUNK=1
run head_c58 '' CSM_CAPC_PCT=58
