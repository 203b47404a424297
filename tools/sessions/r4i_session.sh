# Round 4: single-phase staged RTCSM2D scorer; C1 A/B with kernel traces;
# C3 one-step A/B of batch nodes sorted by (rotation, level, y, x).
set -u
O=gpurun_out/r4i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_rt2d_gpu.py tests/test_golden.py -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for k in 1 2; do
  CSM_PROFILE_RT2D=1 CSM_RT2D_KERNEL=$k timeout -k 10 120 python -u tools/rt2d_probe.py > $O/rt2d_k$k.json 2> $O/rt2d_k$k.err \
    || { tail -20 $O/rt2d_k$k.err; exit 1; }
  echo "kernel=$k $(cat $O/rt2d_k$k.json)"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c1 -- python3 tools/rt2d_probe.py > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" | xargs cat | cut -c1-160
CSM_SORT_BATCH=1 timeout -k 10 400 python -u -m pytest tests/test_fast2d_gpu.py tests/test_c3_ties.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests_sort.log 2>&1 \
  || { tail -60 $O/tests_sort.log; exit 1; }
tail -1 $O/tests_sort.log
for sb in 0 1 0 1; do
  CSM_SORT_BATCH=$sb timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('sort=$sb', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
done
timeout -k 10 400 python -u -m pytest tests/test_threading_gpu.py tests/test_constraint_builder.py tests/test_distributed.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests_arena.log 2>&1 \
  || { tail -60 $O/tests_arena.log; exit 1; }
tail -1 $O/tests_arena.log
timeout -k 10 400 python -u bench.py --workload c2 --no-cpu --no-3d --steps 5 > $O/bench_c2.json 2> $O/bench_c2.err \
  || { tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c2.json').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d['dropin']))"

timeout -k 10 600 python -u -m pytest tests/test_fast3d_gpu.py tests/test_constraint_builder_3d.py tests/test_grids.py tests/test_ceres3d.py tests/test_threading_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests3d.log 2>&1 \
  || { tail -60 $O/tests3d.log; exit 1; }
tail -1 $O/tests3d.log
timeout -k 10 300 python -u tools/probe_c5.py > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5.json')); print({k: d[k] for k in ('value','value_search_only','ms_per_step','build_ms_per_step','search_ms_per_step','kernel_ms_per_step','tied_pairs_per_step','accepted_per_step','errors_per_step')})"
