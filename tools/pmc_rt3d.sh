#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, no tracing) over one C4
# RTCSM3D match (tools/probe_rt3d.py). Usage (GPU box): tools/pmc_rt3d.sh OUTDIR SETTING
#   SETTING: probe_rt3d.py's env setting, e.g. CSM_RT3D_V3=- (v4) or CSM_RT3D_V3=1 (v3)
set -u
OUT=$1
SET=$2
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/$OUT
cd /tmp
export TMPDIR=/tmp
groups=(
 "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum"
 "TD_TD_BUSY_sum GRBM_GUI_ACTIVE"
 "TCC_HIT_sum TCC_MISS_sum"
 "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
 "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT"
)
i=0
for g in "${groups[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $g -d $R/$OUT/p$i -o run --output-format csv -- \
    python3 $R/tools/probe_rt3d.py $SET > $R/$OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/$OUT/p$i.log; exit 1; }
  i=$((i+1))
done
python3 $R/tools/pmc_sum.py $R/$OUT rt3d_score > $R/$OUT/summary.txt
echo done
