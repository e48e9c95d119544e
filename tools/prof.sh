#!/bin/bash
# rocprofv3 passes for the committed profiles (run on the GPU box from the repo root).
# usage: bash tools_prof.sh <outdir-name> [bench args...]
set -o pipefail
NAME=$1; shift
ROOTD=$(pwd)
OUT=$ROOTD/gpurun_out/$NAME
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $ROOTD/bench.py --no-cpu-baseline "$@" > $OUT/bench_trace.log 2>&1 || exit 11
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
  python3 $ROOTD/bench.py --no-cpu-baseline "$@" > $OUT/bench_fetch.log 2>&1 || exit 12
timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
  python3 $ROOTD/bench.py --no-cpu-baseline "$@" > $OUT/bench_write.log 2>&1 || exit 13
echo done
