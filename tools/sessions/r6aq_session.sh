#!/bin/bash
# Round 6: C5 groups per step (6, 8, 12, 16) with the searches on one
# context, two passes.
set -u
O=gpurun_out/r6aq
mkdir -p $O
date +%T
for g in 6 8 12 16 6 8 12 16; do
  timeout -k 10 300 python -u tools/probe_c5.py --c5-dropin-calls 0 --c5-groups $g > $O/c5_g$g.json 2> $O/c5_g$g.err \
    || { tail -20 $O/c5_g$g.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c5_g$g.json').read().strip().splitlines()[-1]); r=d['roofline']; print('groups $g', round(d['value']), round(d['ms_per_step'],1), round(r['kernel_ms_avg'],2), round(d['kernel_ms_per_step'],1), round(r['frac'],3))" | tee -a $O/summary.txt
done
date +%T
