set -u
mkdir -p gpurun_out/r3a
bash tools/gpu_measure.sh gpurun_out/r3a tests || exit 1
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --c3-slice 8 --cpu-pairs 64 --steps3d 1 > gpurun_out/r3a/bench_small.json 2> gpurun_out/r3a/bench_small.err || { tail -30 gpurun_out/r3a/bench_small.err; exit 1; }
