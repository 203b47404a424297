# Round 4: gathers in flight per lane (CSM_U_QUAD 6/8/12, CSM_U_HEX 2/4/6
# builds) on one C3 step; SSE staging of HybridGrid cell lists: 3D tests, C5.
set -u
O=gpurun_out/r4t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fast3d_gpu.py tests/test_constraint_builder_3d.py tests/test_grids.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests3d.log 2>&1 \
  || { tail -60 $O/tests3d.log; exit 1; }
tail -1 $O/tests3d.log
timeout -k 10 300 python -u tools/probe_c5.py > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5.json')); print({k: d[k] for k in ('value','value_search_only','ms_per_step','build_ms_per_step','search_ms_per_step','kernel_ms_per_step','accepted_per_step','errors_per_step')})"
for lib in cartographer-1_amd variants/uq6 variants/uq12 variants/uh2 variants/uh6 cartographer-1_amd; do
  CSM_AMD_LIB=$PWD/$lib/libcsm_amd.so timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$lib', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
done
