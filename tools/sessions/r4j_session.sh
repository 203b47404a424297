# Round 4: asynchronous 3D grid / matcher creates (ready events instead of a
# synchronize per create): 3D parity tests, C5 with builds inside the step.
set -u
O=gpurun_out/r4j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fast3d_gpu.py tests/test_constraint_builder_3d.py tests/test_grids.py tests/test_ceres3d.py tests/test_threading_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/probe_c5.py > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5.json')); print({k: d[k] for k in ('value','value_search_only','ms_per_step','build_ms_per_step','search_ms_per_step','kernel_ms_per_step','tied_pairs_per_step','accepted_per_step','errors_per_step')})"
