#!/bin/bash
# Round 6: octet row builds storing two adjacent octets per lane (16-byte
# stores on rows that start 16-byte aligned). 3D GPU tests
# (levels byte-identical), the C5 builds apart under a kernel trace
# (--c5-groups 1) at HEAD and the previous build (variants/head6), then the
# default C5 probe A/B.
set -u
O=gpurun_out/r6ay
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
date +%T
timeout -k 10 500 python -u -m pytest tests/test_golden.py tests/test_fast3d_gpu.py -m gpu -v \
  --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in head head6; do
  A=""; [ $v != head ] && A=$R/variants/$v/libcsm_amd.so
  (cd /tmp && export TMPDIR=/tmp && CSM_AMD_LIB=$A timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace_$v -o c5g1 \
    --output-format csv -- python3 $R/tools/probe_c5.py --c5-dropin-calls 0 --c5-groups 1 > $R/$O/c5_g1_$v.json 2> $R/$O/c5_g1_$v.err) \
    || { tail -20 $O/c5_g1_$v.err; exit 1; }
  cp $O/trace_$v/c5g1_kernel_stats.csv $O/stats_$v.csv
done
for v in head6 head head6 head; do
  A=""; [ $v != head ] && A=$R/variants/$v/libcsm_amd.so
  CSM_AMD_LIB=$A timeout -k 10 300 python -u tools/probe_c5.py --c5-dropin-calls 0 > $O/c5_$v.json 2> $O/c5_$v.err \
    || { tail -20 $O/c5_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/c5_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value']), round(d['ms_per_step'],1), round(r['kernel_ms_avg'],2), round(d['kernel_ms_per_step'],1), round(r['frac'],3), d['accepted_per_step'], d['errors_per_step'])" | tee -a $O/summary.txt
done
date +%T
