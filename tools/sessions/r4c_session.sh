# Round 4: RCCL code paths with 2-3 ranks through the test stand-in; FETCH_SIZE
# calibration on scattered 4 / 16-byte gathers of known byte counts.
set -u
O=gpurun_out/r4c
R=$PWD
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_comm_rccl_gpu.py tests/test_distributed.py -m gpu -v \
  --timeout 200 --timeout-method thread > $O/rccl_tests.log 2>&1 || { tail -40 $O/rccl_tests.log; exit 1; }
tail -3 $O/rccl_tests.log
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $R/$O/calib -o run \
  --output-format csv -- $R/tools/fetch_calib > $R/$O/calib.json 2> $R/$O/calib.err) \
  || { echo "calib pmc failed"; tail -20 $O/calib.err; exit 1; }
python3 tools/fetch_calib.py $O/calib.json $O/calib/run_counter_collection.csv $O/fetch_calibration.json
