# fast3d exact-tail gathers: 3D parity tests, the C5 tie/parity survey over
# the whole C5 queue, then the C5 leg (with a 4-submap C3 slice ahead of it).
set -u
O=gpurun_out/r3bk
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fast3d_gpu.py tests/test_golden.py tests/test_constraint_builder_3d.py -m gpu -v --timeout 300 --timeout-method thread > $O/tests3d.log 2>&1 || { tail -30 $O/tests3d.log; exit 1; }
tail -2 $O/tests3d.log
timeout -k 10 400 python -u tools/tie_stats3d_c5.py 200 > $O/tie_stats3d_c5_full.json 2> $O/tie_stats3d_c5_full.err || { tail -20 $O/tie_stats3d_c5_full.err; exit 1; }
cat $O/tie_stats3d_c5_full.json
timeout -k 10 400 python -u bench.py --no-cpu --no-rt --steps 1 --warmup 0 --c3-slice 4 --steps3d 5 > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/c5.json') if l.startswith('{')][-1])['fast3d']; print(d['value'], d['kernel_ms_per_step'], d['ms_per_step'], d['accepted_per_step'], d['errors_per_step'])"
