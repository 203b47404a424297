#!/bin/bash
# Round 6: C5 with two search contexts whose searches are chained
# (csm_context_set_search_chain: host phases overlap, searches do not)
# against one context (the default) and two unchained.
set -u
O=gpurun_out/r6ap
mkdir -p $O
date +%T
for v in s1 chain s2 s1 chain s2 s1 chain; do
  case $v in s1) A="--c5-search-streams 1";; chain) A="--c5-search-streams 2 --c5-search-chain";; s2) A="--c5-search-streams 2";; esac
  timeout -k 10 300 python -u tools/probe_c5.py --c5-dropin-calls 0 $A > $O/c5_$v.json 2> $O/c5_$v.err \
    || { tail -20 $O/c5_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c5_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value']), round(d['ms_per_step'],1), round(r['kernel_ms_avg'],2), round(d['kernel_ms_per_step'],1), round(r['frac'],3), d['accepted_per_step'], d['errors_per_step'])" | tee -a $O/summary.txt
done
date +%T
