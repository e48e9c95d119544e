#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r4p}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "variants or golden or bench_dims or saturated or rbwd0 or head_bwd2 or graph" > $OUT/pytest_v.log 2>&1
rc=$?; tail -3 $OUT/pytest_v.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_bigN.py -x -v -s --timeout 500 --timeout-method thread > $OUT/pytest_bign.log 2>&1
rc=$?; grep "rel L2\|passed\|failed" $OUT/pytest_bign.log | tail -20; [ $rc -eq 0 ] || exit $rc
for v in "TRPO_WG_D1H=1" "TRPO_WG_D1H=0"; do
  tag=$(echo $v | tr -d ' =' | tr 'A-Z' 'a-z')
  timeout -k 10 300 env $v python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt --profile-out $OUT/events_$tag.json > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail $OUT/bench_$tag.err; exit 1; }
done
bash tools/ab_env.sh ${1:-r4p}/ab c4 2 "" "TRPO_WG_D1H=0"
