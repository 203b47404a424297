# Closing measurement set at the hybrid-order kernel (levels <= 2 depth-first, best read every batch): C3 FETCH pass + kernel
# trace, C2 trace + PMC passes, then the default bench reading both traffic files.
set -u
O=gpurun_out/r3ar
mkdir -p $O profiles/r3ar
bash tools/gpu_measure.sh $O c3pmc c3trace trace pmc || exit 1
cp $O/traffic_c3.json $O/traffic_c2.json profiles/r3ar/ || exit 1
bash tools/gpu_measure.sh $O bench || exit 1
tail -c 400 $O/bench_full.json
bash tools/gpu_measure.sh $O tests || exit 1
tail -2 $O/gpu_tests.log
