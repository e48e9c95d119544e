#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r4ae}; mkdir -p $OUT
timeout -k 10 1000 python -u tools/diag_bign.py c5 c5 > $OUT/diag_c5.txt 2>&1
rc=$?; tail -20 $OUT/diag_c5.txt; exit $rc
