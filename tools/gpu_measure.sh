#!/bin/bash
# Round-2 measurement set on one MI355X box. Usage: tools/gpu_measure.sh OUT STAGE...
#   tests   pytest -m gpu (all GPU tests)
#   bench   bench.py defaults (C2 + C1 + voxel + Ceres + C4 + C5, CPU baselines)
#   trace   rocprofv3 --kernel-trace --stats of the C2 leg alone
#   pmc     rocprofv3 --pmc passes on the C2 leg (one counter group per pass)
#   gloo2   2-rank rehearsal (torch.distributed.run, gloo, both ranks on the GPU)
#   c3      bench.py --workload c3 (2000 x 1000 queue, 1 GPU) + CPU baseline
#   c3trace rocprofv3 --kernel-trace --stats of two 16-submap slices of the C3 queue (8 chunk launches)
#   c3pmc   FETCH_SIZE pass on one 16-submap slice of the C3 queue (4 chunk launches)
#   c5      C5 probe (builds inside the step), its kernel trace and PMC passes of fast3d_search
set -u
OUT=$1; shift
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/$OUT
cd $R
for st in "$@"; do
  echo "== $st $(date +%T)"
  case $st in
    tests)
      timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
        > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; } ;;
    bench)
      t0=$(date +%s)
      timeout -k 10 700 python -u bench.py > $OUT/bench_full.json 2> $OUT/bench_full.err \
        || { tail -30 $OUT/bench_full.err; exit 1; }
      echo "bench.py wall seconds: $(( $(date +%s) - t0 ))" | tee $OUT/bench_full.wall ;;
    trace)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$OUT/trace \
        -o c2 --output-format csv -- python3 $R/bench.py --workload c2 --no-cpu --no-rt --no-3d --steps 1 --warmup 1 \
        > $R/$OUT/trace.json 2> $R/$OUT/trace.err) || { tail -20 $OUT/trace.err; exit 1; } ;;
    pmc)
      mkdir -p $OUT/pmc
      i=0
      for g in "TA_TA_BUSY_sum GRBM_GUI_ACTIVE" "TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum" \
               "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
        (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --pmc $g -d $R/$OUT/pmc/p$i -o run \
          --output-format csv -- python3 $R/bench.py --workload c2 --no-cpu --no-rt --no-3d --steps 1 --warmup 0 \
          > $R/$OUT/pmc/p$i.log 2>&1) || { echo "pmc pass $i failed"; tail -5 $OUT/pmc/p$i.log; exit 1; }
        i=$((i+1))
      done
      python3 tools/pmc_sum.py $OUT/pmc fast2d_search_v4 > $OUT/pmc/pmc_c2_summary.txt
      python3 tools/traffic_json.py $OUT/pmc/p3 $OUT/traffic_c2.json $(python3 -c "import sys; sys.path.insert(0,'.'); import bench; print(bench.KERNEL_TAG)") 0 ;;
    gloo2)
      timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --no-cpu --no-rt \
        --steps 1 --warmup 1 > $OUT/rehearsal_2rank.json 2> $OUT/rehearsal_2rank.err \
        || { tail -30 $OUT/rehearsal_2rank.err; exit 1; } ;;
    c3)
      timeout -k 10 1000 python -u bench.py --workload c3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err \
        || { tail -30 $OUT/bench_c3.err; exit 1; } ;;
    c3trace)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$OUT/c3trace \
        -o c3 --output-format csv -- python3 -u $R/bench.py --no-cpu --no-rt --no-3d --steps 2 --warmup 1 --c3-slice 16 \
        > $R/$OUT/c3trace.json 2> $R/$OUT/c3trace.err) || { tail -20 $OUT/c3trace.err; exit 1; } ;;
    c3pmc)
      mkdir -p $OUT/c3pmc
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $R/$OUT/c3pmc/p0 -o run \
        --output-format csv -- python3 $R/bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 0 --c3-slice 16 \
        > $R/$OUT/c3pmc/p0.json 2> $R/$OUT/c3pmc/p0.log) || { echo "c3 pmc pass failed"; tail -5 $OUT/c3pmc/p0.log; exit 1; }
      ms=$(python3 -c "import json,sys; print(json.loads([l for l in open('$OUT/c3pmc/p0.json') if l.startswith('{')][-1])['roofline']['kernel_ms_avg'])" 2>/dev/null || echo 0)
      python3 tools/traffic_json.py $OUT/c3pmc $OUT/traffic_c3.json $(python3 -c "import sys; sys.path.insert(0,'.'); import bench; print(bench.KERNEL_TAG)") $ms c3 2000 4 16 ;;
    c5)
      mkdir -p $OUT/pmc3d
      # --c5-dropin-calls 0: the single-call leg's small dispatches would
      # otherwise dominate the per-dispatch averages of the PMC passes.
      timeout -k 10 300 python -u tools/probe_c5.py --c5-dropin-calls 0 > $OUT/c5.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/c5trace \
        -o c5 --output-format csv -- python3 $R/tools/probe_c5.py --c5-dropin-calls 0 > $R/$OUT/c5trace.json 2> $R/$OUT/c5trace.err) \
        || { tail -20 $OUT/c5trace.err; exit 1; }
      i=0
      for g in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE" \
               "TD_TD_BUSY_sum GRBM_COUNT"; do
        (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc $g -d $R/$OUT/pmc3d/p$i -o run \
          --output-format csv -- python3 $R/tools/probe_c5.py --c5-dropin-calls 0 > $R/$OUT/pmc3d/p$i.json 2> $R/$OUT/pmc3d/p$i.log) \
          || { echo "c5 pmc pass $i failed"; tail -5 $OUT/pmc3d/p$i.log; exit 1; }
        i=$((i+1))
      done
      python3 tools/pmc_sum.py $OUT/pmc3d fast3d_search > $OUT/pmc3d/pmc_c5_summary.txt ;;
  esac
done
echo "== done $(date +%T)"
