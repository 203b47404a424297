# x-fastest lane order A/B (variants/x0 = previous order), then the GPU tests
# touched this round (2D search parity, sharded builders with claiming).
set -u
O=gpurun_out/r3s
mkdir -p $O
for k in 1 2 3; do
  for lib in cartographer-1_amd/libcsm_amd.so variants/x0/libcsm_amd.so; do
    CSM_AMD_LIB=$PWD/$lib timeout -k 10 150 python -u bench.py --workload c2 --no-cpu --no-rt --no-3d --steps 1 --warmup 1 \
      > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$lib', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints_per_step'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
  done
done
timeout -k 10 400 python -u -m pytest tests/test_fast2d_gpu.py tests/test_distributed.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
