#!/bin/bash
# Round-4 final evidence in one call (GPU box, repo root): GPU suite, smoke, bench lines (C4 with the CPU baseline,
# C3, C2, C5), rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes over the C4 bench.
# usage: bash tools/gpu_r4final.sh <outdir>
set -o pipefail
NAME=${1:-r4final}
OUT=gpurun_out/$NAME
bash tools/gpu_round.sh $NAME || exit $?
timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-alt > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail $OUT/bench_c5.err; exit 1; }
tail -1 $OUT/bench_c5.json | cut -c1-200
bash tools/prof.sh $NAME --steps 3 --warmup 1 --no-alt || exit $?
echo final done
