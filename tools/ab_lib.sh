#!/bin/bash
# A/B of two builds of libcsm_amd.so on the C2 bench workload, alternating:
# tools/ab_lib.sh LIB_A LIB_B ROUNDS
set -e
mkdir -p gpurun_out
for k in $(seq 1 $3); do
  for lib in "$1" "$2"; do
    CSM_AMD_LIB=$lib timeout -k 10 120 python -u bench.py --no-cpu --no-rt --no-3d --steps 1 --warmup 1 \
      > gpurun_out/ab.json 2> gpurun_out/ab.err
    python -c "
import json; d=json.load(open('gpurun_out/ab.json'))
print('$lib', round(d['value'], 1), round(d['roofline']['kernel_ms_avg'], 1))"
  done
done
