# Round 5: search knobs re-swept on C3 with the flattened scoring lanes
# (small batches now keep the workgroup's lanes busy, which may move the
# optimum): LIFO levels 1/3 (CSM_LIFO_LEVEL), quad gathers in flight 6/12
# (CSM_U_QUAD), hex gathers in flight 3/6 (CSM_U_HEX) as variant builds
# (variants/f_*), hex levels {8,6,4} and 3 rotations per item by env.
# One C3 step each, HEAD repeated.
set -u
O=gpurun_out/r5be
mkdir -p $O
run() {  # label, lib ('' = in-tree), then env assignments
  local label=$1 lib=$2; shift 2
  env ${lib:+CSM_AMD_LIB=$lib} "$@" timeout -k 10 200 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$label', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1), d['accepted_constraints'], d['errors_per_step'])" | tee -a $O/ab_summary.txt
}
run head ''
for v in lifo3 lifo1 uq6 uq12 uh6 uh3; do run $v variants/f_$v/libcsm_amd.so; done
run head2 ''
run hex864 '' CSM_HEX_LEVELS=8,6,4
run rot3 '' CSM_ROT_CHUNK=3
run head3 ''
