#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r4h}; mkdir -p $OUT
timeout -k 10 700 python -u tools/diag_bign.py > $OUT/diag_bign.txt 2>&1
rc=$?; tail -30 $OUT/diag_bign.txt; [ $rc -eq 0 ] || exit $rc
for v in "TRPO_HBWD2=1 TRPO_HEAD_FWD=1" "TRPO_HBWD2=0 TRPO_HEAD_FWD=0"; do
  tag=$(echo $v | tr -d ' =' | tr 'A-Z' 'a-z')
  timeout -k 10 300 env $v python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt --profile-out $OUT/events_$tag.json > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail $OUT/bench_$tag.err; exit 1; }
done
