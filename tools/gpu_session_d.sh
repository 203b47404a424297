#!/bin/bash
# PMC counter groups over the C2 bench (one rocprofv3 pass per group).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
cd $R
bash tools/pmc_profile.sh gpurun_out/pmc_d --no-cpu --no-rt --no-3d --steps 1 --warmup 0
echo ALL_OK
