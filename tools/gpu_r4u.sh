#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r4u}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "variants or golden or head_bwd2 or graph or bench_dims or saturated" > $OUT/pytest_v.log 2>&1
rc=$?; tail -3 $OUT/pytest_v.log; exit $rc
