set -u
O=gpurun_out/r3p
mkdir -p $O
bash tools/gpu_measure.sh $O tests || exit 1
tail -2 $O/gpu_tests.log
C3_PROFILE=1 timeout -k 10 300 python -u bench.py --no-cpu --no-rt --no-3d --steps 2 --warmup 1 --c3-slice 16 > $O/c3_small.json 2> $O/c3_small.err || { tail -20 $O/c3_small.err; exit 1; }
grep "host phases" $O/c3_small.err
python3 -c "import json; d=json.loads(open('$O/c3_small.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_ms_avg'], d['ms_per_step'])"
bash tools/gpu_measure.sh $O c3pmc c3trace || exit 1
