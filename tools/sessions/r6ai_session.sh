#!/bin/bash
# Round 6: octet loads in flight per lane in the tiny build with 32-node
# batches (nu = 25 loads per lane for a 200-point cloud): 4 (variants/i4) and
# 12 (variants/i12, 4 spilled VGPRs) against 8 (HEAD); the C5 probe A/B.
set -u
O=gpurun_out/r6ai
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
date +%T
for v in head i4 i12 head i4 i12; do
  A=""; [ $v != head ] && A=$R/variants/$v/libcsm_amd.so
  CSM_AMD_LIB=$A timeout -k 10 300 python -u tools/probe_c5.py --c5-dropin-calls 0 > $O/c5_$v.json 2> $O/c5_$v.err \
    || { tail -20 $O/c5_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/c5_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value']), round(d['ms_per_step'],1), round(r['kernel_ms_avg'],2), round(d['kernel_ms_per_step'],1), round(r['frac'],3), d['accepted_per_step'], d['errors_per_step'])" | tee -a $O/summary.txt
done
date +%T
