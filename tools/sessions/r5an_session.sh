# Round 5: pruning at a witnessed tie sum in the main searches (2D and 3D)
# and the collect pass abandoning a pair whose record overflowed: the tie and
# parity tests, FindsConstraints' 3D inputs timed (tools/probe_ties3d.py),
# and one C3 step against the previous library (variants/pretie).
set -u
O=gpurun_out/r5an
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
timeout -k 10 300 python -u tools/probe_ties3d.py > $O/ties3d.txt 2> $O/ties3d.err || { tail -20 $O/ties3d.err; exit 1; }
cat $O/ties3d.txt
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu --durations=12 tests/test_ties_walk.py \
  tests/test_c3_ties.py tests/test_fast3d_gpu.py tests/test_fast2d_gpu.py tests/test_golden.py tests/test_c3_gpu.py \
  tests/test_constraint_builder.py tests/test_constraint_builder_3d.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -16 $O/tests.log
run() {  # label, lib
  CSM_AMD_LIB=$2 timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$1', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'], d['tied_pairs_rank0'], d['ties_by_branch_rank0'])" | tee -a $O/ab_summary.txt
}
run pretie $R/variants/pretie/libcsm_amd.so
run tieprune $R/cartographer-1_amd/libcsm_amd.so
