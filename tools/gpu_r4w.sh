#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r4w}; mkdir -p $OUT
for v in "TRPO_SPLIT_MFMA=5" "TRPO_SPLIT_MFMA=6" "TRPO_SPLIT_MFMA=5" "TRPO_SPLIT_MFMA=6"; do
  i=$((i+1))
  tag=$(echo $v | tr -d ' =' | tr 'A-Z' 'a-z')_$i
  timeout -k 10 300 env $v python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt --profile-out $OUT/events_$tag.json > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail $OUT/bench_$tag.err; exit 1; }
done
