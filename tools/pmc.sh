#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter group). usage: bash tools_pmc.sh <outname> <bench args...>
set -o pipefail
NAME=$1; shift
ROOTD=$(pwd)
OUT=$ROOTD/gpurun_out/$NAME
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for GROUP in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $GROUP --output-format csv -d $OUT/pmc$i -o run -- \
    python3 $ROOTD/bench.py --no-cpu-baseline "$@" > $OUT/bench_pmc$i.log 2>&1 || echo "pass $i failed rc=$?"
done
echo done
