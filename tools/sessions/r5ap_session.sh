# Round 5 (r5ao again, the tie sum read once per combine): the tie witness read every 8th batch instead of every batch
# (2D main search): one C3 step against the library before the tie pruning,
# twice, and FindsConstraints' 3D inputs and the tie tests again.
set -u
O=gpurun_out/r5ap
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
run() {  # label, lib
  CSM_AMD_LIB=$2 timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$1', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'], d['tied_pairs_rank0'], d['ties_by_branch_rank0'])" | tee -a $O/ab_summary.txt
}
for k in 1 2; do
  run pretie $R/variants/pretie/libcsm_amd.so
  run tieprune8h $R/cartographer-1_amd/libcsm_amd.so
done
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ties_walk.py \
  tests/test_c3_ties.py tests/test_fast2d_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
