#!/bin/bash
# SQ / GRBM counter passes over one C4 bench run, per kernel (GPU box, repo root).
# usage: bash tools/pmc_kernels.sh <outdir-name> [bench args...]; then python tools/pmc_summary.py gpurun_out/<name>
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
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $GROUP --output-format csv -d $OUT/pmc$i -o run -- \
    python3 $ROOTD/bench.py --no-cpu-baseline --no-alt --steps 1 --warmup 0 --profile-steps 1 "$@" \
    > $OUT/bench_pmc$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -3 $OUT/bench_pmc$i.log; }
done
echo done
