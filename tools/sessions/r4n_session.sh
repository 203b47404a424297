# Round 4: RTCSM2D keys to mapped host memory (no device-to-host copy), 3D
# half-resolution levels from LDS-staged rows: parity, C1 A/B + trace, C5 + trace.
set -u
O=gpurun_out/r4n
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_rt2d_gpu.py tests/test_golden.py tests/test_fast3d_gpu.py tests/test_constraint_builder_3d.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for z in 0 1; do
  CSM_PROFILE_RT2D=1 CSM_RT2D_HOSTKEYS=$z timeout -k 10 120 python -u tools/rt2d_probe.py > $O/rt2d_h$z.json 2> $O/rt2d_h$z.err \
    || { tail -20 $O/rt2d_h$z.err; exit 1; }
  echo "hostkeys=$z $(cat $O/rt2d_h$z.json)"
done
timeout -k 10 300 python -u tools/probe_c5.py > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5.json')); print({k: d[k] for k in ('value','value_search_only','ms_per_step','build_ms_per_step','search_ms_per_step','kernel_ms_per_step','accepted_per_step','errors_per_step')})"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c1 -- python3 tools/rt2d_probe.py > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c5 -- python3 tools/probe_c5.py > $O/trace5.log 2>&1 || { tail -20 $O/trace5.log; exit 1; }
for f in c1 c5; do python3 -c "
import csv
for r in csv.DictReader(open('$O/trace/${f}_kernel_stats.csv')): print(r['Name'][:60], r['Calls'], r['TotalDurationNs'], r['AverageNs'])"; done
timeout -k 10 300 ./tools/dropin_threads 2000 > $O/dropin_cpp.json 2> $O/dropin_cpp.err || { tail -20 $O/dropin_cpp.err; exit 1; }
cat $O/dropin_cpp.json
