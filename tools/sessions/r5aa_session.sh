# Round 5: C5 step with per-create staging slots (csm_hybrid_grid_create no
# longer waits for the previous create's upload, which sat behind the
# running search kernel): HEAD's library against the new one, and group
# counts; one C5 leg each (tools/probe_c5.py), the same accepted count
# required.
set -u
O=gpurun_out/r5aa
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
ab() {
  local label=$1 lib=$2; shift 2
  CSM_AMD_LIB=$lib timeout -k 10 200 python -u tools/probe_c5.py "$@" > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$label', round(d['ms_per_step'], 1), 'build', round(d['build_ms_per_step'], 1), 'search', round(d['search_ms_per_step'], 1),
      'kernel', round(d['kernel_ms_per_step'], 1), d['accepted_per_step'], d['errors_per_step'], d['c5_group_sizes'], d.get('c5_search_streams'))" | tee -a $O/c5_ab.txt
}
date +%T
for k in 1 2; do
  ab head $R/variants/c5base/libcsm_amd.so
  ab slots $R/cartographer-1_amd/libcsm_amd.so
done
ab slots-g16-f4 $R/cartographer-1_amd/libcsm_amd.so --c5-groups 16 --c5-first-group 4
ab slots-g24-f4 $R/cartographer-1_amd/libcsm_amd.so --c5-groups 24 --c5-first-group 4
ab slots-g8-f6 $R/cartographer-1_amd/libcsm_amd.so --c5-groups 8 --c5-first-group 6
date +%T
