# Closing measurement set at the full-batch kernel: C3 FETCH pass + kernel
# trace, C2 trace + PMC passes, then the default bench reading both traffic files.
set -u
O=gpurun_out/r3ae
mkdir -p $O profiles/r3ae
bash tools/gpu_measure.sh $O c3pmc c3trace trace pmc || exit 1
cp $O/traffic_c3.json $O/traffic_c2.json profiles/r3ae/ || exit 1
bash tools/gpu_measure.sh $O bench || exit 1
tail -c 400 $O/bench_full.json
