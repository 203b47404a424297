# Default bench at the final HEAD (bench.py reads profiles/r3bi's traffic files).
set -u
O=gpurun_out/r3bj
mkdir -p $O
bash tools/gpu_measure.sh $O bench || exit 1
python3 -c "import json; d=json.loads([l for l in open('$O/bench_full.json') if l.startswith('{')][-1]); print(d['value'], d['roofline']['frac'], d['roofline']['traffic_frac'], d['roofline']['traffic_source'])"
