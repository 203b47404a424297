# Round 5: every GPU test at the final HEAD (flattened scoring lanes),
# with the slowest tests' durations, then smoke().
set -u
O=gpurun_out/r5bi
mkdir -p $O
date +%T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread --durations=30 \
  > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -36 $O/gputests.log
date +%T
timeout -k 10 60 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
