# Round 4 closing set, part 2: C3 kernel trace and FETCH pass, C2 trace and
# PMC passes, C5 probe + trace + PMC (the files bench.py and DESIGN.md cite).
set -u
bash tools/gpu_measure.sh gpurun_out/r4z c3trace c3pmc trace pmc c5
