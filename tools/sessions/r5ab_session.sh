# Round 5: host timeline of the C5 step (CSM_C5_TRACE=1: when each group's
# build is issued and returns, when each search call starts and returns),
# HEAD's library and the staging-slot one.
set -u
O=gpurun_out/r5ab
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
for v in slots; do
  lib=$R/cartographer-1_amd/libcsm_amd.so
  [ $v = head ] && lib=$R/variants/c5base/libcsm_amd.so
  CSM_PROFILE3D_BUILD=1 CSM_C5_TRACE=1 CSM_AMD_LIB=$lib timeout -k 10 200 python -u tools/probe_c5.py --steps3d 2 > $O/$v.json 2> $O/$v.err || { tail -20 $O/$v.err; exit 1; }
  echo "$v"; grep "c5 trace" $O/$v.err | tail -1
done
