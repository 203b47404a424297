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
python3 tools/traffic3d_json.py $O/pmc3d $O/traffic_c5.json $TAG3 || exit 1
