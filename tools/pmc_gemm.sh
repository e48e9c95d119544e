#!/bin/bash
# PMC passes over the GEMM micro-bench. usage: bash tools/pmc_gemm.sh <outname> <M> <split mode>
set -o pipefail
NAME=$1; M=$2; MODE=$3
ROOTD=$(pwd)
OUT=$ROOTD/gpurun_out/$NAME
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for GROUP in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVES" \
             "SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_VALU_MFMA_COEXEC_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $GROUP --output-format csv -d $OUT/pmc$i -o run -- \
    $ROOTD/tools/gemm_bench $M 2 $MODE > $OUT/pmc$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
echo done
