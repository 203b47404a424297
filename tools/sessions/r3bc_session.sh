# Checkpoint at HEAD (parallel tie sorts; search kernel as r3ar): the default
# bench, then every GPU test.
set -u
O=gpurun_out/r3bc
mkdir -p $O
bash tools/gpu_measure.sh $O bench || exit 1
tail -c 300 $O/bench_full.json
bash tools/gpu_measure.sh $O tests || exit 1
tail -2 $O/gpu_tests.log
