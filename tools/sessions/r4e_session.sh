# Round 4: 3D exact-tie resolution (tests + C5 timing and tie counts), and the
# LDS-DMA gather microbenchmark.
set -u
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests \
  -m gpu -v --timeout 300 --timeout-method thread > $O/tests3d.log 2>&1 \
  || { tail -60 $O/tests3d.log; exit 1; }
tail -3 $O/tests3d.log
timeout -k 10 300 python -u tools/probe_c5.py > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5.json')); print({k: d[k] for k in ('value','value_search_only','ms_per_step','build_ms_per_step','search_ms_per_step','kernel_ms_per_step','tied_pairs_per_step','ties_unresolved_per_step','ties_by_branch_last_step','accepted_per_step')})"
hipcc -O3 --offload-arch=gfx950 tools/gather_lds_bench.hip -o tools/gather_lds_bench && timeout -k 10 120 ./tools/gather_lds_bench > $O/gather_lds.txt 2>&1 || { cat $O/gather_lds.txt; exit 1; }
cat $O/gather_lds.txt
