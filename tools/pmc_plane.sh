#!/bin/bash
# SQ / GRBM counter passes over tools/plane_bench (GPU box, repo root).
# usage: bash tools/pmc_plane.sh <outdir-name> [plane_bench args...]; then python tools/pmc_summary.py gpurun_out/<name>
set -o pipefail
NAME=$1; shift
ROOTD=$(pwd)
OUT=$ROOTD/gpurun_out/$NAME
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for GROUP in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVES SQ_INSTS_MFMA" \
             "SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU_FP64"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $GROUP --output-format csv -d $OUT/pmc$i -o run -- \
    $ROOTD/tools/plane_bench "$@" > $OUT/bench_pmc$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -3 $OUT/bench_pmc$i.log; exit 1; }
done
echo done
