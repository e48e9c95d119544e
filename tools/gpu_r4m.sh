#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r4m}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "variants or head_bwd2 or golden or bench_dims" > $OUT/pytest_v.log 2>&1
rc=$?; tail -3 $OUT/pytest_v.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/diag_bign.py > $OUT/diag_bign.txt 2>&1
rc=$?; tail -30 $OUT/diag_bign.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh ${1:-r4m}/ab c4 2 "" "TRPO_PG_SPLITS=512"
