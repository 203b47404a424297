# Round 4: C5 host phases (CSM_PROFILE3D) with the asynchronous builds.
set -u
O=gpurun_out/r4v
mkdir -p $O
CSM_PROFILE3D=1 timeout -k 10 300 python -u tools/probe_c5.py > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
grep "fast3d host" $O/c5.err | tail -4
python3 -c "import json; d=json.load(open('$O/c5.json')); print({k: d[k] for k in ('value','ms_per_step','build_ms_per_step','search_ms_per_step','kernel_ms_per_step')})"
