# Last check of the shipped in-tree libraries: smoke and every GPU test.
set -u
O=gpurun_out/r3bm
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_measure.sh $O tests || exit 1
tail -2 $O/gpu_tests.log
