# Checkpoint at HEAD (v4/v5 for clouds up to 16,448 points): smoke, every GPU
# test, then the default bench.
set -u
O=gpurun_out/r3be
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_measure.sh $O tests || exit 1
tail -2 $O/gpu_tests.log
bash tools/gpu_measure.sh $O bench || exit 1
tail -c 400 $O/bench_full.json
