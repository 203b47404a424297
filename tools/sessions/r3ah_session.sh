# PMC (instructions, TA/TD busy) of the C3 chunk launches: tiled-quad kernel
# (in-tree) against the previous kernel (variants/prev).
set -u
O=gpurun_out/r3ah
mkdir -p $O
R=$PWD
for lib in cartographer-1_amd variants/prev; do
  tag=$(basename $lib)
  (cd /tmp && export TMPDIR=/tmp && CSM_AMD_LIB=$R/$lib/libcsm_amd.so timeout -s KILL 150 rocprofv3 --pmc TA_BUFFER_READ_WAVEFRONTS_sum TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE \
    -d $R/$O/$tag -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 0 --c3-slice 8 \
    > $R/$O/$tag.log 2>&1) || { echo "pmc $tag failed"; tail -5 $O/$tag.log; exit 1; }
  python3 tools/pmc_sum.py $O/$tag fast2d_search_v4 | tee $O/$tag.summary.txt
done
