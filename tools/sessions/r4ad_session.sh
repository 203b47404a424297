# Round 4: (1) hex-level sets on C3 (the default {8, 6} was chosen on C2);
# (2) non-temporal cache policy on the quad / hex gathers (variants/nt*,
# built with -DCSM_CPOL_QUAD=2 / -DCSM_CPOL_HEX=2). One C3 step each, the
# same accepted counts required.
set -u
O=gpurun_out/r4ad
mkdir -p $O
run() {  # label, then env assignments
  local label=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$label', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
}
date +%T
for v in 8,6 8,6,4 8,5 8,6,3 7,5 8,4; do run hex=$v CSM_HEX_LEVELS=$v; done
date +%T
for lib in default variants/ntq variants/nth variants/ntb default; do
  if [ $lib = default ]; then run lib=$lib CSM_QUEUE_SPREAD=1; else run lib=$lib CSM_AMD_LIB=$PWD/$lib/libcsm_amd.so; fi
done
date +%T
