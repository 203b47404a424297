# Round 5: the gather roofline of the tiled-quad variant (r5bg): a CSM_KPROF
# pass (variants/kprof_tiled: lines per gather by child level) and a TD/TA
# pass (variants/tiled) on the C3 slice -> gather_c3_tiled.json, to set
# against profiles/r5bb/gather_c3.json (row-major planes).
set -u
O=gpurun_out/r5bh
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
CSM_PROFILE2D=1 CSM_AMD_LIB=$R/variants/kprof_tiled/libcsm_amd.so timeout -k 10 300 python -u bench.py --no-cpu --no-rt --no-3d \
  --steps 1 --warmup 0 --c3-slice 16 > $O/kprof.json 2> $O/kprof.err || { tail -20 $O/kprof.err; exit 1; }
(cd /tmp && export TMPDIR=/tmp && CSM_AMD_LIB=$R/variants/tiled/libcsm_amd.so timeout -s KILL 240 rocprofv3 --pmc TD_TD_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum \
  -d $R/$O/pmc_td -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 0 \
  --c3-slice 16 > $R/$O/pmc_td.json 2> $R/$O/pmc_td.log) || { echo "pmc pass failed"; tail -5 $O/pmc_td.log; exit 1; }
python3 tools/gather_roofline.py $O/kprof.err $O/pmc_td $O/gather_c3_tiled.json tiled-quad || exit 1
