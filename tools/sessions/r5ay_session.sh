# Round 5 closing measurement set at HEAD (tie pruning; bench.py KERNEL_TAG
# v5-tieprune, KERNEL3D_TAG f3-octet-tieprune):
#  1. FETCH_SIZE passes of fast2d_search_v4 on the C3 slice and on C2
#     -> traffic_c3.json, traffic_c2.json;
#  2. the C3 gather roofline: a CSM_KPROF pass (variants/kprof5, lines per
#     gather) and a TD/TA pass on the same slice -> gather_c3.json;
#  3. C5: probe, kernel trace, PMC passes of fast3d_search -> traffic_c5.json
#     (superseded by r5bd: these passes averaged over the single-call leg's
#     small dispatches too);
#  (the default bench.py run reading those files: r5az_session.sh).
set -u
O=gpurun_out/r5ay
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
TAG=$(python3 -c "import sys; sys.path.insert(0,'.'); import bench; print(bench.KERNEL_TAG)")
TAG3=$(python3 -c "import sys; sys.path.insert(0,'.'); import bench; print(bench.KERNEL3D_TAG)")
date +%T
bash tools/gpu_measure.sh $O c3pmc || exit 1
mkdir -p $O/c2pmc
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $R/$O/c2pmc/p0 -o run \
  --output-format csv -- python3 $R/bench.py --workload c2 --no-cpu --no-rt --no-3d --steps 1 --warmup 0 \
  > $R/$O/c2pmc/p0.json 2> $R/$O/c2pmc/p0.log) || { echo "c2 pmc pass failed"; tail -5 $O/c2pmc/p0.log; exit 1; }
python3 tools/traffic_json.py $O/c2pmc $O/traffic_c2.json $TAG 0 || exit 1
date +%T
CSM_PROFILE2D=1 CSM_AMD_LIB=$R/variants/kprof5/libcsm_amd.so timeout -k 10 300 python -u bench.py --no-cpu --no-rt --no-3d \
  --steps 1 --warmup 0 --c3-slice 16 > $O/kprof.json 2> $O/kprof.err || { tail -20 $O/kprof.err; exit 1; }
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc TD_TD_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum \
  -d $R/$O/pmc_td -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 0 \
  --c3-slice 16 > $R/$O/pmc_td.json 2> $R/$O/pmc_td.log) || { echo "pmc pass failed"; tail -5 $O/pmc_td.log; exit 1; }
python3 tools/gather_roofline.py $O/kprof.err $O/pmc_td $O/gather_c3.json $TAG || exit 1
date +%T
bash tools/gpu_measure.sh $O c5 || exit 1
python3 tools/traffic3d_json.py $O/pmc3d $O/traffic_c5.json $TAG3 $O/c5.json || exit 1
date +%T
