# Round 5: C5 step with the grids' host staging spread over the host pool
# (csm_hybrid_grid_create_batch), against HEAD's serial staging, and the
# first group's size (the step's start waits for its build).
set -u
O=gpurun_out/r5al
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
ab() {
  local label=$1 lib=$2; shift 2
  CSM_AMD_LIB=$lib timeout -k 10 200 python -u tools/probe_c5.py "$@" > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$label', round(d['ms_per_step'], 1), 'build', round(d['build_ms_per_step'], 1), 'search', round(d['search_ms_per_step'], 1),
      'kernel', round(d['kernel_ms_per_step'], 1), d['accepted_per_step'], d['errors_per_step'], d['c5_group_sizes'][:3])" | tee -a $O/c5_ab.txt
}
L=$R/cartographer-1_amd/libcsm_amd.so
for k in 1 2; do
  ab serial $R/variants/c5serial/libcsm_amd.so --c5-dropin-calls 0
  ab pool $L --c5-dropin-calls 0
done
ab pool-first3 $L --c5-dropin-calls 0 --c5-first-group 3
ab pool-first2 $L --c5-dropin-calls 0 --c5-first-group 2
ab pool-first3-g14 $L --c5-dropin-calls 0 --c5-first-group 3 --c5-groups 14
ab pool-first4-g12 $L --c5-dropin-calls 0 --c5-first-group 4
