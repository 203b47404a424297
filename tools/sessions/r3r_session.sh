# Closing measurement set: C3 FETCH pass + kernel trace, then the default bench
# (full C3 queue) reading that traffic file.
set -u
O=gpurun_out/r3r
mkdir -p $O profiles/r3r
bash tools/gpu_measure.sh $O c3pmc c3trace || exit 1
cp $O/traffic_c3.json profiles/r3r/ || exit 1
bash tools/gpu_measure.sh $O bench || exit 1
tail -c 1500 $O/bench_full.json
