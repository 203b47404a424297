#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, no tracing) over the
# FastCSM3D C5-share probe. Usage (GPU box): tools/pmc3d.sh OUTDIR
set -u
OUT=$1
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/$OUT
cd /tmp
export TMPDIR=/tmp
groups=(
 "FETCH_SIZE"
 "TCC_HIT_sum TCC_MISS_sum"
 "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
 "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
)
i=0
for g in "${groups[@]}"; do
  timeout -k 10 240 rocprofv3 --pmc $g -d $R/$OUT/p$i -o run --output-format csv -- \
    python3 $R/tools/probe3d.py --nodes 500 --submaps 25 > $R/$OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  i=$((i+1))
done
echo done
