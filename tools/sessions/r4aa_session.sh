# Round 4: 3D node clouds staged in Morton order (CSM_F3_MORTON): parity and
# C5 A/B.
set -u
O=gpurun_out/r4aa
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fast3d_gpu.py tests/test_constraint_builder_3d.py tests/test_golden.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for m in 0 1 0 1; do
  CSM_F3_MORTON=$m timeout -k 10 300 python -u tools/probe_c5.py > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c5.json')); print('morton=$m', {k: round(d[k],1) for k in ('value','value_search_only','ms_per_step','kernel_ms_per_step','accepted_per_step','errors_per_step')})" | tee -a $O/ab_summary.txt
done
