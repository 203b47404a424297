# Round 4: CSM_KPROF build on one C3 step: distinct lines per gather
# instruction by child level and the workgroups' phase cycles.
set -u
O=gpurun_out/r4w
mkdir -p $O
CSM_PROFILE2D=1 CSM_AMD_LIB=$PWD/variants/kprof/libcsm_amd.so timeout -k 10 300 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 > $O/kprof.json 2> $O/kprof.err || { tail -20 $O/kprof.err; exit 1; }
grep "lines per gather\|fast2d phases" $O/kprof.err | tail -6
