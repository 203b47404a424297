set -u
mkdir -p gpurun_out/r3l
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3l/tests.log 2>&1 || { tail -40 gpurun_out/r3l/tests.log; exit 1; }
tail -2 gpurun_out/r3l/tests.log
bash tools/ab_kernel.sh gpurun_out/r3l "CSM_PROFILE2D=1" "CSM_PROFILE2D=1 CSM_SEARCH_KERNEL=4"
grep -m1 "fast2d launch" gpurun_out/r3l/ab_0.err
