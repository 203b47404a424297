set -u
mkdir -p gpurun_out/r3i
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3i/tests.log 2>&1 || { tail -40 gpurun_out/r3i/tests.log; exit 1; }
tail -2 gpurun_out/r3i/tests.log
bash tools/ab_kernel.sh gpurun_out/r3i "" "CSM_ROT_CHUNK=3" "CSM_ROT_CHUNK=4" "CSM_ROT_CHUNK=1" "CSM_CLUSTER=0,1,1,2,3,3,3,3,3" "CSM_CLUSTER=0,1,2,2,2,3,3,3,3" "CSM_CLUSTER=0,1,1,1,2,3,3,3,3"
