#!/bin/bash
# round 4: parity of the BK 32 row-GEMM variant, then a same-box A/B of split_mfma 5 vs 14 on C4
set -o pipefail
OUT=gpurun_out/${1:-r4b}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "split_mfma" > $OUT/pytest_bk32.log 2>&1
rc=$?; tail -3 $OUT/pytest_bk32.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh ${1:-r4b}/ab c4 2 "TRPO_SPLIT_MFMA=5" "TRPO_SPLIT_MFMA=14"
