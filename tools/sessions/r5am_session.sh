# Round 5: FindsConstraints' 3D inputs (every leaf ties), GPU path against
# the oracle, per call (tools/probe_ties3d.py).
set -u
O=gpurun_out/r5am
mkdir -p $O
CSM_PROFILE3D=1 timeout -k 10 300 python -u tools/probe_ties3d.py > $O/ties3d.txt 2> $O/ties3d.err || { tail -20 $O/ties3d.err; exit 1; }
cat $O/ties3d.txt
grep -v "^fast3d root\|^fast3d phases" $O/ties3d.err | tail -20
