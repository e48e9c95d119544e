#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r4g}; mkdir -p $OUT
timeout -k 10 500 python -u tools/diag_bign.py > $OUT/diag_bign.txt 2>&1
rc=$?; cat $OUT/diag_bign.txt | tail -12; [ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh ${1:-r4g}/ab c4 2 "TRPO_HBWD2=1 TRPO_HEAD_FWD=1" "TRPO_HBWD2=0 TRPO_HEAD_FWD=0" "TRPO_HBWD2=1 TRPO_HEAD_FWD=0"
