# Round 5: C5 PMC set at HEAD again, the probe runs without the single-call
# leg (tools/gpu_measure.sh c5 now passes --c5-dropin-calls 0; r5ay's
# per-dispatch averages included its ~1000 small dispatches)
# -> traffic_c5.json (bench.py TRAFFIC3D_FILE, KERNEL3D_TAG f3-octet-tieprune).
set -u
O=gpurun_out/r5bd
mkdir -p $O
TAG3=$(python3 -c "import sys; sys.path.insert(0,'.'); import bench; print(bench.KERNEL3D_TAG)")
bash tools/gpu_measure.sh $O c5 || exit 1
python3 tools/traffic3d_json.py $O/pmc3d $O/traffic_c5.json $TAG3 $O/c5.json || exit 1
