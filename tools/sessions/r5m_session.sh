# Round 5: C5 at HEAD — the probe (builds pipelined against the searches),
# its kernel trace, and PMC passes of fast3d_search (FETCH, L2, TA/TD) ->
# profiles/r5m/traffic_c5.json (bench.py fast3d.roofline.traffic, KERNEL3D_TAG).
set -u
O=gpurun_out/r5m
mkdir -p $O
# Host phases of csm_fast3d_match_batch (CSM_PROFILE3D prints per call).
CSM_PROFILE3D=1 timeout -k 10 300 python -u tools/probe_c5.py > $O/c5prof.json 2> $O/c5prof.err || { tail -20 $O/c5prof.err; exit 1; }
bash tools/gpu_measure.sh $O c5 || exit 1
TAG3=$(python3 -c "import sys; sys.path.insert(0,'.'); import bench; print(bench.KERNEL3D_TAG)")
python3 tools/traffic3d_json.py $O/pmc3d $O/traffic_c5.json $TAG3 $O/c5.json || exit 1
# C5 step shape A/B: first-group size and batched matcher creation.
ab() {
  local label=$1; shift
  timeout -k 10 200 python -u tools/probe_c5.py "$@" > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$label', round(d['ms_per_step'], 1), 'build', round(d['build_ms_per_step'], 1), 'search', round(d['search_ms_per_step'], 1),
      'kernel', round(d['kernel_ms_per_step'], 1), d['accepted_per_step'], d['c5_group_sizes'])" | tee -a $O/c5_ab.txt
}
ab base
ab batch --c5-create batch
ab first10 --c5-first-group 10
ab first10-batch --c5-first-group 10 --c5-create batch
ab g8-first10 --c5-groups 8 --c5-first-group 10
ab g8-first10-batch --c5-groups 8 --c5-first-group 10 --c5-create batch
ab g2 --c5-groups 2
