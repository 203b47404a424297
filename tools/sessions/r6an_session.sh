#!/bin/bash
# Round 6: C5 with one search context against two (the default): step time
# and the per-launch kernel time the roofline divides by (two contexts'
# launches overlap, which stretches each launch's HIP-event duration).
set -u
O=gpurun_out/r6an
mkdir -p $O
date +%T
for s in 1 2 1 2 1 2; do
  timeout -k 10 300 python -u tools/probe_c5.py --c5-dropin-calls 0 --c5-search-streams $s > $O/c5_s$s.json 2> $O/c5_s$s.err \
    || { tail -20 $O/c5_s$s.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c5_s$s.json').read().strip().splitlines()[-1]); r=d['roofline']; print('streams $s', round(d['value']), round(d['ms_per_step'],1), round(r['kernel_ms_avg'],2), round(d['kernel_ms_per_step'],1), round(r['frac'],3))" | tee -a $O/summary.txt
done
date +%T
