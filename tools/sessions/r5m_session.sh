# Round 5: C5 at HEAD — the probe (builds pipelined against the searches),
# its kernel trace, and PMC passes of fast3d_search (FETCH, L2, TA/TD) ->
# profiles/r5m/traffic_c5.json (bench.py fast3d.roofline.traffic, KERNEL3D_TAG).
set -u
O=gpurun_out/r5m
bash tools/gpu_measure.sh $O c5 || exit 1
TAG3=$(python3 -c "import sys; sys.path.insert(0,'.'); import bench; print(bench.KERNEL3D_TAG)")
python3 tools/traffic3d_json.py $O/pmc3d $O/traffic_c5.json $TAG3 || exit 1
