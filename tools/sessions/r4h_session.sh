# Round 4: RTCSM2D staged scorer (gathers in LDS segments, one wave adds in
# point order): parity under both scorers, C1 A/B with the host profile.
set -u
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_rt2d_gpu.py tests/test_golden.py -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
CSM_RT2D_KERNEL=1 timeout -k 10 300 python -u -m pytest tests/test_rt2d_gpu.py -m gpu -q --timeout 200 --timeout-method thread > $O/tests_k1.log 2>&1 \
  || { tail -60 $O/tests_k1.log; exit 1; }
tail -1 $O/tests_k1.log
for k in 1 2; do
  CSM_PROFILE_RT2D=1 CSM_RT2D_KERNEL=$k timeout -k 10 120 python -u tools/rt2d_probe.py > $O/rt2d_k$k.json 2> $O/rt2d_k$k.err \
    || { tail -20 $O/rt2d_k$k.err; exit 1; }
  echo "kernel=$k $(cat $O/rt2d_k$k.json)"
  grep "rt2d host" $O/rt2d_k$k.err | head -1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/trace -o c1 -- python3 tools/rt2d_probe.py > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
