# Round 4, first GPU call: every GPU test after the csm_result2d.tie ABI
# change, then the whole C3 queue with its tied pairs logged
# (input of tools/c3_tie_fixture.py).
set -u
O=gpurun_out/r4a
mkdir -p $O
bash tools/gpu_measure.sh $O tests || exit 1
tail -2 $O/gpu_tests.log
timeout -k 10 600 python -u bench.py --no-cpu --no-rt --no-3d --warmup 1 --c3-tie-log $O/c3ties \
  > $O/bench_c3.json 2> $O/bench_c3.err || { tail -30 $O/bench_c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c3.json').read().splitlines()[-1]); print(d['value'], d['tied_pairs_rank0'], d['ties_by_branch_rank0'], d['roofline']['kernel_ms_avg'])"
