#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r4i}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "head_bwd2 or hbwd2 or head_fwd or bench_dims or golden or saturated or many_actions" > $OUT/pytest_hb.log 2>&1
rc=$?; tail -3 $OUT/pytest_hb.log; [ $rc -eq 0 ] || exit $rc
for v in "TRPO_HEAD_FWD=1" "TRPO_HEAD_FWD=2" "TRPO_HEAD_FWD=3" "TRPO_HEAD_FWD=4" "TRPO_HEAD_FWD=0"; do
  tag=$(echo $v | tr -d ' =' | tr 'A-Z' 'a-z')
  timeout -k 10 300 env $v python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt --profile-out $OUT/events_$tag.json > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail $OUT/bench_$tag.err; exit 1; }
done
