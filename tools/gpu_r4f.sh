#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r4f}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "head_bwd2 or rbwd0 or tail or saturated or bench_dims or hbwd2 or head_fwd or golden or many_actions" > $OUT/pytest_hb.log 2>&1
rc=$?; tail -3 $OUT/pytest_hb.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh ${1:-r4f}/ab c4 2 "TRPO_HBWD2=1 TRPO_HEAD_FWD=1" "TRPO_HBWD2=0 TRPO_HEAD_FWD=0" "TRPO_HBWD2=1 TRPO_HEAD_FWD=0"
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt --profile-out $OUT/events_c4.json > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail $OUT/bench_c4.err; exit 1; }
