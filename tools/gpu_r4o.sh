#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r4o}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_learn.py -x -v --timeout 200 --timeout-method thread -k "variants or golden or cg or graph" > $OUT/pytest_v.log 2>&1
rc=$?; tail -3 $OUT/pytest_v.log; [ $rc -eq 0 ] || exit $rc
AB_STEPS=50 bash tools/ab_env.sh ${1:-r4o}/ab_c2 c2 2 "" "TRPO_CG_SMALL=0" "TRPO_HEAD_FWD=1" || exit 1
AB_STEPS=30 bash tools/ab_env.sh ${1:-r4o}/ab_c3 c3 2 "" "TRPO_CG_SMALL=0" "TRPO_HEAD_FWD=1" || exit 1
