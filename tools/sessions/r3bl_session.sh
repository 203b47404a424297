# fast3d with the packed cloud rank-sorted into (z, y, x) order (variant build
# -DCSM_F3_SORT): 3D parity tests, the whole-C5 pose survey and the C5 leg,
# then the C5 leg on the default build for the A/B.
set -u
O=gpurun_out/r3bl
mkdir -p $O
V=$PWD/variants/f3sort/libcsm_amd.so
CSM_AMD_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_fast3d_gpu.py tests/test_golden.py tests/test_constraint_builder_3d.py -m gpu -v --timeout 300 --timeout-method thread > $O/tests3d.log 2>&1 || { tail -30 $O/tests3d.log; exit 1; }
tail -2 $O/tests3d.log
CSM_AMD_LIB=$V timeout -k 10 400 python -u tools/tie_stats3d_c5.py 200 > $O/tie_stats3d_c5_full.json 2> $O/tie_stats3d_c5_full.err || { tail -20 $O/tie_stats3d_c5_full.err; exit 1; }
cat $O/tie_stats3d_c5_full.json
for lib in $V $PWD/cartographer-1_amd/libcsm_amd.so; do
  CSM_AMD_LIB=$lib timeout -k 10 400 python -u bench.py --no-cpu --no-rt --steps 1 --warmup 0 --c3-slice 4 --steps3d 5 > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/c5.json') if l.startswith('{')][-1])['fast3d']; print('$lib', d['value'], d['kernel_ms_per_step'], d['ms_per_step'], d['accepted_per_step'], d['errors_per_step'])" | tee -a $O/ab.txt
done
