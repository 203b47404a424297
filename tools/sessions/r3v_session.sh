# Full GPU tests at the current tree, then the 2-rank rehearsal of the
# default (C3) bench over the TCP transport (both ranks on the one GPU).
set -u
O=gpurun_out/r3v
mkdir -p $O
bash tools/gpu_measure.sh $O tests gloo2 || exit 1
tail -2 $O/gpu_tests.log
tail -c 600 $O/rehearsal_2rank.json
