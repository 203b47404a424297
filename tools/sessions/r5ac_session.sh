# Round 5: C5 step with every 3D create's staging in its own slot (grid cell
# lists and pyramid job lists, StageRing): HEAD's library against the new
# one (one C5 leg each, tools/probe_c5.py, the same accepted count
# required), then the new one's host timeline (CSM_C5_TRACE=1).
set -u
O=gpurun_out/r5ac
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
for k in 1 2 3; do
  ab head $R/variants/c5base/libcsm_amd.so
  ab rings $R/cartographer-1_amd/libcsm_amd.so
done
ab rings-g16-f4 $R/cartographer-1_amd/libcsm_amd.so --c5-groups 16 --c5-first-group 4
ab rings-g24-f4 $R/cartographer-1_amd/libcsm_amd.so --c5-groups 24 --c5-first-group 4
CSM_PROFILE3D_BUILD=1 CSM_C5_TRACE=1 timeout -k 10 200 python -u tools/probe_c5.py --steps3d 2 > $O/trace.json 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
grep "c5 trace" $O/trace.err | tail -1
grep "create_batch" $O/trace.err | tail -12
date +%T
