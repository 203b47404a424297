# Round 5: RTCSM2D (C1) host phases per Match (CSM_PROFILE_RT2D=1: window +
# rotation table, grid check, staging, launches, wait), C1 leg alone.
set -u
O=gpurun_out/r5ak
mkdir -p $O
CSM_PROFILE_RT2D=1 timeout -k 10 200 python -u tools/rt2d_probe.py > $O/rt2d.json 2> $O/rt2d.err || { tail -20 $O/rt2d.err; exit 1; }
tail -3 $O/rt2d.err
tail -c 600 $O/rt2d.json
