# Round 5: where the tie-pruning build's extra C3 time comes from: HEAD's
# library, the tie-pruning build, and the same source with CSM_TIE_PRUNE=0
# (the witness never read); one C3 step each, three rounds.
set -u
O=gpurun_out/r5ar
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
run() {  # label, lib
  CSM_AMD_LIB=$2 timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$1', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
}
for k in 1 2 3; do
  run head $R/variants/pretie/libcsm_amd.so
  run tieprune $R/cartographer-1_amd/libcsm_amd.so
  run tie0 $R/variants/tie0/libcsm_amd.so
done
