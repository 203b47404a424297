# Round 4: 3D level / octet builds from LDS-staged rows (dword loads; 3D grid
# launches): 3D parity tests, C5 with builds inside the step, build kernel trace.
set -u
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fast3d_gpu.py tests/test_constraint_builder_3d.py tests/test_golden.py tests/test_rt2d_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/probe_c5.py > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5.json')); print({k: d[k] for k in ('value','value_search_only','ms_per_step','build_ms_per_step','search_ms_per_step','kernel_ms_per_step','accepted_per_step','errors_per_step')})"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c5 -- python3 tools/probe_c5.py > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('$O/trace/c5_kernel_stats.csv')): print(r['Name'][:60], r['Calls'], r['TotalDurationNs'], r['AverageNs'])"

CSM_PUSH_ROWS=1 timeout -k 10 400 python -u -m pytest tests/test_fast2d_gpu.py tests/test_c3_ties.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests_rows.log 2>&1 \
  || { tail -60 $O/tests_rows.log; exit 1; }
tail -1 $O/tests_rows.log
for pr in 0 1 0 1; do
  CSM_PUSH_ROWS=$pr timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('push_rows=$pr', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
done

timeout -k 10 300 python -u -m pytest tests/test_rt2d_gpu.py tests/test_golden.py -m gpu -q --timeout 200 --timeout-method thread > $O/tests_rt2d.log 2>&1 \
  || { tail -60 $O/tests_rt2d.log; exit 1; }
tail -1 $O/tests_rt2d.log
for z in 0 1; do
  CSM_PROFILE_RT2D=1 CSM_RT2D_ZEROCOPY=$z timeout -k 10 120 python -u tools/rt2d_probe.py > $O/rt2d_z$z.json 2> $O/rt2d_z$z.err \
    || { tail -20 $O/rt2d_z$z.err; exit 1; }
  echo "zerocopy=$z $(cat $O/rt2d_z$z.json)"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c1z -- python3 tools/rt2d_probe.py > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('$O/trace/c1z_kernel_stats.csv')): print(r['Name'][:60], r['Calls'], r['AverageNs'])"
