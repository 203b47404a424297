set -u
mkdir -p gpurun_out/r3b
timeout -k 10 400 python -u -m pytest tests/test_fast2d_gpu.py tests/test_golden.py tests/test_c3_gpu.py tests/test_fast3d_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3b/tests.log 2>&1 || { tail -40 gpurun_out/r3b/tests.log; exit 1; }
tail -3 gpurun_out/r3b/tests.log
bash tools/ab_kernel.sh gpurun_out/r3b 4 5
