#!/bin/bash
# Round 6: the C5 PMC set of fast3d_search with the tiny-cloud build
# (KERNEL3D_TAG f3-tiny5-r64: the tiny-cloud build and roots at the lowest
# level with <= 64 candidates), reduced into gpurun_out/r6x/profile/ (committed
# as profiles/r6x/).
set -u
O=gpurun_out/r6x
R=${GRAFT_REPO_ROOT:-$PWD}
P=$O/profile
mkdir -p $O $P
date +%T
bash tools/gpu_measure.sh $O c5 || exit 1
cp $O/c5.json $P/c5.json
python3 tools/profiles.py reduce-pmc $O/pmc3d $P/c5_pmc.csv fast3d_search || exit 1
cp $O/pmc3d/pmc_c5_summary.txt $P/ 2>/dev/null
date +%T
