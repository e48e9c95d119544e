#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r4l}; mkdir -p $OUT
timeout -k 10 900 python -u tools/diag_bign.py > $OUT/diag_bign.txt 2>&1
rc=$?; tail -30 $OUT/diag_bign.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh ${1:-r4l}/ab c4 2 "" "TRPO_SPLITS=1024" "TRPO_SPLITS=2048"
