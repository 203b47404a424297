#!/bin/bash
# Round 6: the tiny-cloud fast3d_search build fixed at 5 workgroups per CU
# and 8 octet loads in flight (0 spills). Every GPU test and smoke() at
# HEAD, then the C5 probe A/B against the previous build (variants/base)
# and the 4- and 12-load variants, and the C++ threaded 3D drop-in.
set -u
O=gpurun_out/r6p
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
date +%T
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread --durations=15 \
  > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -1 $O/gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
date +%T
for v in base head t5i4 t5i12 head base; do
  A=""; [ $v != head ] && A=$R/variants/$v/libcsm_amd.so
  CSM_AMD_LIB=$A timeout -k 10 300 python -u tools/probe_c5.py --c5-dropin-calls 0 > $O/c5_$v.json 2> $O/c5_$v.err \
    || { tail -20 $O/c5_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/c5_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value']), round(d['ms_per_step'],1), round(r['kernel_ms_avg'],2), round(r['frac'],3), d['accepted_per_step'], d['errors_per_step'])" | tee -a $O/summary.txt
done
timeout -k 10 300 tools/dropin_threads3d 4000 8 200 > $O/dropin_head.json 2> $O/dropin_head.err \
  || { cat $O/dropin_head.json; tail -5 $O/dropin_head.err; exit 1; }
echo "dropin $(cat $O/dropin_head.json)" | tee -a $O/summary.txt
date +%T
