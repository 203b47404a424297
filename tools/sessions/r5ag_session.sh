# Round 5: batched HybridGrid builds (csm_hybrid_grid_create_batch): the
# batch-vs-single grid test and the batch-vs-single matcher test, then the
# C5 leg with batched grids against single grid creates (same library,
# --c5-grids), twice each, the same accepted count required.
set -u
O=gpurun_out/r5ag
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_fast3d_gpu.py \
  -k "create_batch" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
ab() {
  local label=$1; shift
  timeout -k 10 200 python -u tools/probe_c5.py "$@" > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$label', round(d['ms_per_step'], 1), 'build', round(d['build_ms_per_step'], 1), 'search', round(d['search_ms_per_step'], 1),
      'kernel', round(d['kernel_ms_per_step'], 1), d['accepted_per_step'], d['errors_per_step'], d['c5_group_sizes'], d.get('c5_search_streams'))" | tee -a $O/c5_ab.txt
}
for k in 1 2; do
  ab grids-single --c5-grids single
  ab grids-batch --c5-grids batch
done
ab batch-g8-f6 --c5-groups 8 --c5-first-group 6
ab batch-g16-f4 --c5-groups 16 --c5-first-group 4
