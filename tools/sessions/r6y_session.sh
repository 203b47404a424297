#!/bin/bash
# Round 6: the C5 step's pipeline shape at HEAD: search contexts (2, 3) x
# groups per step (8, 12, 16), the C5 probe per setting.
set -u
O=gpurun_out/r6y
mkdir -p $O
date +%T
for cfg in "2 12" "3 12" "2 16" "3 16" "2 8" "3 8" "2 12" "3 12"; do
  set -- $cfg
  timeout -k 10 300 python -u tools/probe_c5.py --c5-dropin-calls 0 --c5-search-streams $1 --c5-groups $2 \
    > $O/c5_s$1_g$2.json 2> $O/c5_s$1_g$2.err || { tail -20 $O/c5_s$1_g$2.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/c5_s$1_g$2.json').read().strip().splitlines()[-1]); r=d['roofline']; print('streams $1 groups $2', round(d['value']), round(d['ms_per_step'],1), round(r['kernel_ms_avg'],2), round(d['kernel_ms_per_step'],1), round(r['frac'],3), d['accepted_per_step'], d['errors_per_step'])" | tee -a $O/summary.txt
done
date +%T
