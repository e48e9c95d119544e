#!/bin/bash
# Round-4 final evidence in one call (GPU box, repo root): GPU suite, smoke, bench lines, rocprofv3 kernel
# trace + FETCH_SIZE / WRITE_SIZE passes over the C4 bench.  usage: bash tools/gpu_r4final.sh <outdir>
set -o pipefail
NAME=${1:-r4final}
bash tools/gpu_round.sh $NAME || exit $?
bash tools/prof.sh $NAME --steps 3 --warmup 1 --no-alt || exit $?
echo final done
