# Round 4: RTCSM2D result hand-off (mapped host word) and polling wait, host
# phase profile; single-call grid sharing under threads (dropin leg).
set -u
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_rt2d_gpu.py tests/test_threading_gpu.py -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
CSM_RT2D_WAIT=poll timeout -k 10 300 python -u -m pytest tests/test_rt2d_gpu.py -m gpu -q --timeout 200 --timeout-method thread > $O/tests_poll.log 2>&1 \
  || { tail -60 $O/tests_poll.log; exit 1; }
tail -1 $O/tests_poll.log
for v in "0 sync" "1 sync" "1 poll"; do
  set -- $v
  CSM_PROFILE_RT2D=1 CSM_RT2D_HANDOFF=$1 CSM_RT2D_WAIT=$2 timeout -k 10 120 python -u tools/rt2d_probe.py > $O/rt2d_h$1_$2.json 2> $O/rt2d_h$1_$2.err \
    || { tail -20 $O/rt2d_h$1_$2.err; exit 1; }
  echo "handoff=$1 wait=$2 $(cat $O/rt2d_h$1_$2.json)"
  grep "rt2d host" $O/rt2d_h$1_$2.err | tail -2
done
timeout -k 10 400 python -u bench.py --workload c2 --no-cpu --no-3d --steps 5 > $O/bench_c2.json 2> $O/bench_c2.err \
  || { tail -20 $O/bench_c2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c2.json').read().strip().splitlines()[-1]); print(json.dumps(d['dropin']))"
timeout -k 10 120 ./tools/gather_pattern_bench > $O/gather_pattern.txt 2>&1 || { cat $O/gather_pattern.txt; exit 1; }
cat $O/gather_pattern.txt
