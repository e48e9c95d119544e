#!/bin/bash
# C5 line, world-1 RCCL line and the 2-rank rehearsal line (GPU box, repo root). usage: bash tools/gpu_extra.sh <outdir>
set -o pipefail
OUT=gpurun_out/${1:-extra}; mkdir -p $OUT
timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-alt --profile-out $OUT/events_c5.json > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -5 $OUT/bench_c5.err; exit 1; }
tail -1 $OUT/bench_c5.json | cut -c1-200
timeout -k 10 300 python -u bench.py --rccl-world1 --steps 3 --warmup 1 --no-cpu-baseline --no-alt > $OUT/bench_rccl_world1.json 2> $OUT/bench_rccl_world1.err || { tail -5 $OUT/bench_rccl_world1.err; exit 1; }
tail -1 $OUT/bench_rccl_world1.json | cut -c1-200
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --rehearsal --rows 2000000 --steps 2 --warmup 1 --no-cpu-baseline --no-alt > $OUT/bench_2rank_rehearsal.json 2> $OUT/bench_2rank_rehearsal.err || { tail -5 $OUT/bench_2rank_rehearsal.err; exit 1; }
tail -1 $OUT/bench_2rank_rehearsal.json | cut -c1-200
