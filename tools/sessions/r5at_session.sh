# Round 5 (r5ar again, ties detected from the combine's own leaf keys, no global load): HEAD's
# library, the tie-pruning build, and the same source with CSM_TIE_PRUNE=0
# (the witness never read); one C3 step each, three rounds.
set -u
O=gpurun_out/r5at
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
run() {  # label, lib
  CSM_AMD_LIB=$2 timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$1', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
}
for k in 1 2 3; do
  run head $R/variants/pretie/libcsm_amd.so
  run tieprune $R/cartographer-1_amd/libcsm_amd.so
  run tie0 $R/variants/tie0/libcsm_amd.so
done
c5() {  # label, lib
  CSM_AMD_LIB=$2 timeout -k 10 200 python -u tools/probe_c5.py --c5-dropin-calls 0 > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/c5.json').read().strip().splitlines()[-1])
print('c5 $1', round(d['ms_per_step'], 1), 'kernel', round(d['kernel_ms_per_step'], 1), d['accepted_per_step'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
}
for k in 1 2; do
  c5 head $R/variants/pretie/libcsm_amd.so
  c5 tieprune $R/cartographer-1_amd/libcsm_amd.so
done
timeout -k 10 300 python -u tools/probe_ties3d.py > $O/ties3d.txt 2> $O/ties3d.err || { tail -20 $O/ties3d.err; exit 1; }
cat $O/ties3d.txt
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ties_walk.py \
  tests/test_c3_ties.py tests/test_fast3d_gpu.py tests/test_fast2d_gpu.py tests/test_golden.py tests/test_c3_gpu.py \
  tests/test_constraint_builder.py tests/test_constraint_builder_3d.py tests/test_threading_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
