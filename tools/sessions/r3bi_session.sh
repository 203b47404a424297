# Measurement set at the final HEAD: C3 kernel trace and FETCH pass, C2 kernel
# trace and PMC passes (the traffic files bench.py reads).
set -u
O=gpurun_out/r3bi
mkdir -p $O
bash tools/gpu_measure.sh $O c3trace c3pmc trace pmc || exit 1
ls $O
