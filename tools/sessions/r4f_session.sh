# Round 4: RTCSM2D fused path (parity + C1 timing A/B), C5 with pooled builds
# and 3D tie counts, the LDS-DMA gather microbenchmark.
set -u
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_rt2d_gpu.py tests/test_golden.py tests/test_search_space.py \
  tests/test_constraint_builder_3d.py tests/test_threading_gpu.py tests/test_c3_ties.py -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for f in 0 1; do
  CSM_RT2D_FUSED=$f timeout -k 10 120 python -u tools/rt2d_probe.py > $O/rt2d_fused$f.json 2> $O/rt2d_fused$f.err \
    || { tail -20 $O/rt2d_fused$f.err; exit 1; }
  echo "fused=$f $(cat $O/rt2d_fused$f.json)"
done
timeout -k 10 300 python -u tools/probe_c5.py > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5.json')); print({k: d[k] for k in ('value','value_search_only','ms_per_step','build_ms_per_step','release_ms_per_step','search_ms_per_step','kernel_ms_per_step','tied_pairs_per_step','ties_unresolved_per_step','ties_by_branch_last_step','accepted_per_step')})"
hipcc -O3 --offload-arch=gfx950 tools/gather_lds_bench.hip -o tools/gather_lds_bench && timeout -k 10 120 ./tools/gather_lds_bench > $O/gather_lds.txt 2>&1 || { cat $O/gather_lds.txt; exit 1; }
cat $O/gather_lds.txt
timeout -k 10 400 python -u bench.py --workload c2 --no-cpu --no-3d --steps 5 > $O/bench_c2.json 2> $O/bench_c2.err \
  || { tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c2.json').read().strip().splitlines()[-1]); print(json.dumps({k: v for k, v in d.items() if 'dropin' in k or k in ('value','rt2d')})[:3000])"
