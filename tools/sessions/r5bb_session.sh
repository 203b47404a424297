# Round 5: flattened scoring lanes as the default (bench.py KERNEL_TAG
# v5-flat): every GPU test and smoke(), then the 2D PMC set at HEAD
# (C3/C2 FETCH_SIZE, the C3 gather roofline from a CSM_KPROF pass of
# variants/kprof5 and a TD/TA pass) -> traffic_c3.json, traffic_c2.json,
# gather_c3.json.
set -u
O=gpurun_out/r5bb
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
TAG=$(python3 -c "import sys; sys.path.insert(0,'.'); import bench; print(bench.KERNEL_TAG)")
date +%T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread --durations=30 \
  > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 60 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
date +%T
bash tools/gpu_measure.sh $O c3pmc || exit 1
mkdir -p $O/c2pmc
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $R/$O/c2pmc/p0 -o run \
  --output-format csv -- python3 $R/bench.py --workload c2 --no-cpu --no-rt --no-3d --steps 1 --warmup 0 \
  > $R/$O/c2pmc/p0.json 2> $R/$O/c2pmc/p0.log) || { echo "c2 pmc pass failed"; tail -5 $O/c2pmc/p0.log; exit 1; }
python3 tools/traffic_json.py $O/c2pmc $O/traffic_c2.json $TAG 0 || exit 1
CSM_PROFILE2D=1 CSM_AMD_LIB=$R/variants/kprof5/libcsm_amd.so timeout -k 10 300 python -u bench.py --no-cpu --no-rt --no-3d \
  --steps 1 --warmup 0 --c3-slice 16 > $O/kprof.json 2> $O/kprof.err || { tail -20 $O/kprof.err; exit 1; }
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc TD_TD_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum \
  -d $R/$O/pmc_td -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 0 \
  --c3-slice 16 > $R/$O/pmc_td.json 2> $R/$O/pmc_td.log) || { echo "pmc pass failed"; tail -5 $O/pmc_td.log; exit 1; }
python3 tools/gather_roofline.py $O/kprof.err $O/pmc_td $O/gather_c3.json $TAG || exit 1
date +%T
