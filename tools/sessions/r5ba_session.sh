# Round 5: flattened scoring lanes (CSM_FLAT_LANES=1, variants/flat): the
# 256 threads take (node, chunk) pairs instead of 4 waves x nodes-mod-pow2
# lanes. 2D parity tests on the variant, then one C3 step each, A/B/A.
set -u
O=gpurun_out/r5ba
mkdir -p $O
F=variants/flat/libcsm_amd.so
CSM_AMD_LIB=$F timeout -k 10 600 python -u -m pytest tests/test_fast2d_gpu.py tests/test_c3_gpu.py tests/test_c3_ties.py tests/test_ties_walk.py \
  -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_flat.log 2>&1 || { tail -30 $O/tests_flat.log; exit 1; }
tail -2 $O/tests_flat.log
run() {  # label, lib ('' = in-tree), then env assignments
  local label=$1 lib=$2; shift 2
  env ${lib:+CSM_AMD_LIB=$lib} "$@" timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$label', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'], d.get('parity_sample'))" | tee -a $O/ab_summary.txt
}
run head ''
run flat $F
run head2 ''
run flat2 $F
