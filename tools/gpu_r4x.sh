#!/bin/bash
# rbwd0 ablation builds (R0_ABL: 1 no X^T RD_0 phase, 2 no epilogue loads, 3 no k-loop); timing only
set -o pipefail
OUT=gpurun_out/${1:-r4x}; mkdir -p $OUT
for v in "" "TRPO_ENGINE_LIB=trpo_amd/libtrpo_engine_r0abl1.so" "TRPO_ENGINE_LIB=trpo_amd/libtrpo_engine_r0abl2.so" "TRPO_ENGINE_LIB=trpo_amd/libtrpo_engine_r0abl3.so"; do
  i=$((i+1))
  timeout -k 10 300 env $v python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-alt --profile-out $OUT/events_$i.json > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { tail $OUT/bench_$i.err; exit 1; }
done
