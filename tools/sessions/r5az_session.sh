# Round 5 closing bench: the default bench.py run at HEAD, reading the
# traffic and gather-roofline files of profiles/r5ay.
set -u
bash tools/gpu_measure.sh gpurun_out/r5az bench || exit 1
tail -c 600 gpurun_out/r5az/bench_full.json
