# Round 4: 4-bit hex bounds. variants/q17 (-DCSM_HEX_Q17): 16-byte hex
# planes with values rounded up to multiples of 17 (the pruning cost alone);
# variants/hex8 (-DCSM_HEX8=1): the 8-byte nibble planes (pruning cost plus
# half the hex bytes). One C3 step each, alternating; then the 2D parity
# tests on the hex8 build.
set -u
O=gpurun_out/r4ae
mkdir -p $O
run() {
  local label=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$label', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'], d['roofline'].get('algorithmic_bytes_per_launch'))" | tee -a $O/ab_summary.txt
}
for k in 1 2; do
  run lib=default CSM_QUEUE_SPREAD=1
  run lib=q17 CSM_AMD_LIB=$PWD/variants/q17/libcsm_amd.so
  run lib=hex8 CSM_AMD_LIB=$PWD/variants/hex8/libcsm_amd.so
done
CSM_AMD_LIB=$PWD/variants/hex8/libcsm_amd.so timeout -k 10 600 python -u -m pytest tests/test_fast2d_gpu.py tests/test_c3_ties.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_hex8.log 2>&1 || { tail -30 $O/tests_hex8.log; exit 1; }
tail -2 $O/tests_hex8.log
