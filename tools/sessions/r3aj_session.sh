# Round-end rehearsal at HEAD: build() check is CPU-side; smoke() and the
# whole GPU suite on the box.
set -u
O=gpurun_out/r3aj
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_measure.sh $O tests || exit 1
tail -2 $O/gpu_tests.log
