# Round 5: C5 step shape, second pass: group searches on 1-3 contexts from
# their own host threads (--c5-search-streams), with small first groups and
# batched matcher creation (r5m: g8-first10-batch 302 ms vs 324 base).
set -u
O=gpurun_out/r5n
mkdir -p $O
ab() {
  local label=$1; shift
  timeout -k 10 200 python -u tools/probe_c5.py "$@" > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1])
print('$label', round(d['ms_per_step'], 1), 'build', round(d['build_ms_per_step'], 1), 'search', round(d['search_ms_per_step'], 1),
      'kernel', round(d['kernel_ms_per_step'], 1), d['accepted_per_step'], d['errors_per_step'], d['c5_group_sizes'], d.get('c5_search_streams'))" | tee -a $O/c5_ab.txt
}
date +%T
ab base
ab g8-first10-batch --c5-groups 8 --c5-first-group 10 --c5-create batch
ab g8-first10-batch-s2 --c5-groups 8 --c5-first-group 10 --c5-create batch --c5-search-streams 2
ab g8-first10-batch-s3 --c5-groups 8 --c5-first-group 10 --c5-create batch --c5-search-streams 3
ab g4-batch-s2 --c5-groups 4 --c5-create batch --c5-search-streams 2
ab g12-first6-batch-s2 --c5-groups 12 --c5-first-group 6 --c5-create batch --c5-search-streams 2
ab g16-first4-batch-s2 --c5-groups 16 --c5-first-group 4 --c5-create batch --c5-search-streams 2
date +%T
