# Round 4: C3 tie fixture and threading tests, the drop-in's threaded
# single-call leg (C2 world).
set -u
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_c3_ties.py tests/test_threading_gpu.py tests/test_constraint_builder.py tests/test_constraint_builder_3d.py -v --timeout 300 \
  --timeout-method thread > $O/new_tests.log 2>&1 || { tail -40 $O/new_tests.log; exit 1; }
tail -3 $O/new_tests.log
timeout -k 10 400 python -u bench.py --workload c2 --no-cpu --no-3d --steps 1 --warmup 1 \
  > $O/bench_c2.json 2> $O/bench_c2.err || { tail -30 $O/bench_c2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c2.json').read().splitlines()[-1]); print(json.dumps(d['dropin'])); print(d['value'], json.dumps(d['rt2d']))"
