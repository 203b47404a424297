# Polyphase planes in 2-D 128-byte tiles (default) vs rows (variants/rows),
# C3 one step, alternating; then the 2D parity tests at the default.
set -u
O=gpurun_out/r3al
mkdir -p $O
for k in 1 2; do
  for lib in cartographer-1_amd variants/rows; do
    CSM_AMD_LIB=$PWD/$lib/libcsm_amd.so timeout -k 10 120 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 \
      > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$lib', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
  done
done
timeout -k 10 400 python -u -m pytest tests/test_fast2d_gpu.py tests/test_golden.py tests/test_c3_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
