#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r4q}; mkdir -p $OUT
AB_STEPS=50 bash tools/ab_env.sh ${1:-r4q}/ab_c2 c2 2 "" "TRPO_FUSED=1" || exit 1
AB_STEPS=30 bash tools/ab_env.sh ${1:-r4q}/ab_c3 c3 2 "" "TRPO_FUSED=1" || exit 1
bash tools/pmc_kernels.sh ${1:-r4q}/pmc --steps 1 --warmup 0 || exit 1
