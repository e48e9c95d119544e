#!/bin/bash
# PMC passes over a short bench run (GPU box, repo root): SQ issue/wait/LDS counters and L2 hits.
# usage: bash tools/pmc_chain.sh <outdir-name> [bench args...]
set -o pipefail
NAME=$1; shift
ROOTD=$(pwd)
OUT=$ROOTD/gpurun_out/$NAME
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
  SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES \
  --output-format csv -d $OUT/pmc_sq -o run -- python3 $ROOTD/bench.py --no-cpu-baseline "$@" > $OUT/sq.log 2>&1 || exit 21
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc_tcc -o run -- \
  python3 $ROOTD/bench.py --no-cpu-baseline "$@" > $OUT/tcc.log 2>&1 || exit 22
echo pmc done
