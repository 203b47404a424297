#!/bin/bash
# Round 6: root scoring on one wave again (the four-wave split reverted)
# against HEAD (variants/head7, split): KPROF phases of both
# (variants/kprof_ns, variants/kprof3), 3D GPU tests, C5 probe A/B x3.
set -u
O=gpurun_out/r6az
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
date +%T
for k in kprof3 kprof_ns; do
  CSM_PROFILE3D=1 CSM_AMD_LIB=$R/variants/$k/libcsm_amd.so timeout -k 10 300 python -u tools/probe_c5.py \
    --c5-dropin-calls 0 > $O/c5_$k.json 2> $O/c5_$k.err || { tail -20 $O/c5_$k.err; exit 1; }
  echo "$k"; grep "fast3d phases" $O/c5_$k.err | tail -3 | tee $O/phases_$k.txt
done
timeout -k 10 500 python -u -m pytest tests/test_golden.py tests/test_fast3d_gpu.py tests/test_ties_walk.py -m gpu -v \
  --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in head7 head head7 head head7 head; do
  A=""; [ $v != head ] && A=$R/variants/$v/libcsm_amd.so
  CSM_AMD_LIB=$A timeout -k 10 300 python -u tools/probe_c5.py --c5-dropin-calls 0 > $O/c5_$v.json 2> $O/c5_$v.err \
    || { tail -20 $O/c5_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/c5_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value']), round(d['ms_per_step'],1), round(r['kernel_ms_avg'],2), round(d['kernel_ms_per_step'],1), round(r['frac'],3), d['accepted_per_step'], d['errors_per_step'])" | tee -a $O/summary.txt
done
date +%T
