# Round 4: C5 with single creates routed through the batch builder (count 1).
set -u
O=gpurun_out/r4y
mkdir -p $O
for k in 1 2; do
CSM_PROFILE3D=1 timeout -k 10 300 python -u tools/probe_c5.py > $O/c5_$k.json 2> $O/c5_$k.err || { tail -20 $O/c5_$k.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5_$k.json')); print({k: d[k] for k in ('value','value_search_only','ms_per_step','build_ms_per_step','search_ms_per_step','kernel_ms_per_step','accepted_per_step','errors_per_step')})"
done
