#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r4ac}; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests/test_gpu_full_size.py -x -v -s --timeout 800 --timeout-method thread > $OUT/pytest_full.log 2>&1
rc=$?; grep "rel L2\|passed\|failed\|Error" $OUT/pytest_full.log | tail -24; exit $rc
