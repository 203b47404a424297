# Round 5: quad planes in 128-byte tiles of 8 x 4 entries (CSM_QUAD_TILED=1,
# variants/tiled, built from tools/experiments/r5bg_quad_tiled.patch with
# EXTRA=-DCSM_QUAD_TILED=1; hex planes unchanged), so a batch's 2 x 2 / 4 x 4 sibling
# blocks read one line per scan entry. 2D parity tests on the variant, then
# one C3 step each, A/B/A/B.
set -u
O=gpurun_out/r5bg
mkdir -p $O
T=variants/tiled/libcsm_amd.so
CSM_AMD_LIB=$T timeout -k 10 600 python -u -m pytest tests/test_fast2d_gpu.py tests/test_c3_gpu.py tests/test_c3_ties.py tests/test_ties_walk.py \
  -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_tiled.log 2>&1 || { tail -30 $O/tests_tiled.log; exit 1; }
tail -2 $O/tests_tiled.log
run() {  # label, lib ('' = in-tree), then env assignments
  local label=$1 lib=$2; shift 2
  env ${lib:+CSM_AMD_LIB=$lib} "$@" timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$label', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
}
run head ''
run tiled $T
run head2 ''
run tiled2 $T
