# Round 4 final HEAD: GPU tests, the default bench run and the C3 kernel
# trace, after the CSM_HEX8 / cache-policy build options went in (off).
set -u
bash tools/gpu_measure.sh gpurun_out/r4af tests bench c3trace
