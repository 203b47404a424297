# Round 4 closing set, part 1: every GPU test, then the default bench.py run.
set -u
bash tools/gpu_measure.sh gpurun_out/r4z3 tests bench
