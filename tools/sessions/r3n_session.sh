set -u
mkdir -p gpurun_out/r3n
timeout -k 10 400 python -u -m pytest tests/test_fast2d_gpu.py tests/test_golden.py tests/test_c3_gpu.py tests/test_constraint_builder.py tests/test_pbstream.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3n/tests.log 2>&1 || { tail -60 gpurun_out/r3n/tests.log; exit 1; }
tail -2 gpurun_out/r3n/tests.log
bash tools/ab_kernel.sh gpurun_out/r3n ""
