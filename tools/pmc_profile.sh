#!/bin/bash
# Collects per-kernel PMC counters for the search kernel, one rocprofv3 pass
# per counter group (counters never combined with tracing, per the pool rules).
# Usage (on the GPU box): tools/pmc_profile.sh OUTDIR [bench args...]
set -u
OUT=$1; shift
cd /tmp
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
groups=(
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
 "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
 "TA_TA_BUSY_sum GRBM_GUI_ACTIVE"
 "TA_BUFFER_READ_WAVEFRONTS_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"
 "TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum"
 "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
 "TCP_TCP_TA_DATA_STALL_CYCLES_sum TD_TC_STALL_sum"
 "TCC_HIT_sum TCC_MISS_sum"
 "FETCH_SIZE"
)
mkdir -p $R/$OUT
i=0
for g in "${groups[@]}"; do
  timeout -k 10 240 rocprofv3 --pmc $g -d $R/$OUT/p$i -o run --output-format csv -- python3 $R/bench.py "$@" > $R/$OUT/p$i.log 2>&1 || echo "pass $i failed"
  i=$((i+1))
done
echo done
