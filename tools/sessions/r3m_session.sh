set -u
O=gpurun_out/r3c
bash tools/gpu_measure.sh $O c3pmc pmc || exit 1
mkdir -p profiles/r3c && cp $O/traffic_c3.json $O/traffic_c2.json profiles/r3c/
bash tools/gpu_measure.sh $O c3trace trace bench || exit 1
