#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r4s}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_learn.py -x -v -s --timeout 500 --timeout-method thread > $OUT/pytest_learn.log 2>&1
rc=$?; tail -15 $OUT/pytest_learn.log; exit $rc
