# Final checkpoint: smoke, every GPU test, and the 2-rank rehearsal of the
# scaling path (gloo + the TCP csm_comm, both ranks on the one GPU).
set -u
O=gpurun_out/r3bh
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_measure.sh $O tests || exit 1
tail -2 $O/gpu_tests.log
bash tools/gpu_measure.sh $O gloo2 || exit 1
tail -c 600 $O/rehearsal_2rank.json
