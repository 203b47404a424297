set -u
O=gpurun_out/r3o
mkdir -p $O
bash tools/gpu_measure.sh $O tests || exit 1
tail -2 $O/gpu_tests.log
bash tools/gpu_measure.sh $O c3pmc c3trace || exit 1
