# Round 5: what the split-list build's time goes to (one C3 step each, the
# same accepted count required): HEAD, the split source built with
# CSM_SPLIT=0 (should equal HEAD), with CSM_SPLIT_DECIDE=0 (quad batches keep
# tails but never skip), and the split build.
set -u
O=gpurun_out/r5z
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
date +%T
run() {  # label, lib
  CSM_AMD_LIB=$2 timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$1', round(d['value'], 1), round(r['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'], '%.4g' % (r['achieved'] * r['kernel_ms_avg'] * 1e6))" | tee -a $O/ab_summary.txt
}
for k in 1 2; do
  run base $R/cartographer-1_amd/libcsm_amd.so
  run nosplit $R/variants/nosplit/libcsm_amd.so
  run splitnd $R/variants/splitnd/libcsm_amd.so
  run split $R/variants/split/libcsm_amd.so
done
date +%T
