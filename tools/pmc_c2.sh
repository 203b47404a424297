#!/bin/bash
# Core PMC passes for the C2 search kernel (one rocprofv3 pass per group; no
# tracing). Usage on the GPU box: tools/pmc_c2.sh OUTDIR
set -u
OUT=$1
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp
export TMPDIR=/tmp
groups=(
 "TA_TA_BUSY_sum GRBM_GUI_ACTIVE"
 "TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum"
 "TCC_HIT_sum TCC_MISS_sum"
 "FETCH_SIZE"
)
mkdir -p $R/$OUT
i=0
for g in "${groups[@]}"; do
  timeout -s KILL 150 rocprofv3 --pmc $g -d $R/$OUT/p$i -o run --output-format csv -- python3 $R/bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 0 > $R/$OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  i=$((i+1))
done
echo done
