# Round 4: 8-byte hex entries in 4 x 4 tiles (one 128-byte line per tile,
# variants/hex8t: -DCSM_HEX8=1 -DCSM_HEX_TILE=1) against untiled 8-byte
# entries (variants/hex8) and the default; one C3 step each, alternating;
# then the 2D parity tests on the tiled build.
set -u
O=gpurun_out/r4ag
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
  run lib=hex8t CSM_AMD_LIB=$PWD/variants/hex8t/libcsm_amd.so
  run lib=hex8 CSM_AMD_LIB=$PWD/variants/hex8/libcsm_amd.so
done
CSM_AMD_LIB=$PWD/variants/hex8t/libcsm_amd.so timeout -k 10 600 python -u -m pytest tests/test_fast2d_gpu.py tests/test_c3_ties.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_hex8t.log 2>&1 || { tail -30 $O/tests_hex8t.log; exit 1; }
tail -2 $O/tests_hex8t.log
