# Round 5: fast3d_search with point-major scoring lanes (CSM_F3_POINT_MAJOR=1,
# variants/pm3, built from tools/experiments/r5bc_f3_point_major.patch with
# EXTRA=-DCSM_F3_POINT_MAJOR=1): 3D parity tests on the variant, then C5 A/B.
set -u
O=gpurun_out/r5bc
mkdir -p $O
P=variants/pm3/libcsm_amd.so
CSM_AMD_LIB=$P timeout -k 10 600 python -u -m pytest tests/test_fast3d_gpu.py tests/test_ties_walk.py tests/test_constraint_builder_3d.py \
  -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_pm3.log 2>&1 || { tail -30 $O/tests_pm3.log; exit 1; }
tail -2 $O/tests_pm3.log
ab() {  # label, lib ('' = in-tree)
  local label=$1 lib=$2; shift 2
  env ${lib:+CSM_AMD_LIB=$lib} timeout -k 10 200 python -u tools/probe_c5.py "$@" > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$label', round(d['ms_per_step'], 1), 'kernel', round(d['kernel_ms_per_step'], 1), d['accepted_per_step'])" | tee -a $O/c5_ab.txt
}
# Kernel alone: one group, one search stream (the search launch runs by itself).
for r in 1 2; do
  ab head1g '' --c5-groups 1 --c5-search-streams 1 --c5-dropin-calls 0
  ab pm3_1g $P --c5-groups 1 --c5-search-streams 1 --c5-dropin-calls 0
done
ab head '' --c5-dropin-calls 0
ab pm3 $P --c5-dropin-calls 0
