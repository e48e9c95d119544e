#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r4t}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_learn.py -x -v --timeout 300 --timeout-method thread -k "variants or golden or head_bwd2 or fused or learn or graph or chain" > $OUT/pytest_v.log 2>&1
rc=$?; tail -3 $OUT/pytest_v.log; [ $rc -eq 0 ] || exit $rc
AB_STEPS=50 bash tools/ab_env.sh ${1:-r4t}/ab_c2 c2 2 "" "TRPO_HBWD2=0" || exit 1
AB_STEPS=30 bash tools/ab_env.sh ${1:-r4t}/ab_c3 c3 2 "" "TRPO_HBWD2=0" || exit 1
