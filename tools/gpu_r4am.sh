#!/bin/bash
# head_bwd2 VALU trims: default = packed d / s chains + no per-FMA select; _sel = no per-FMA select only;
# _old = the previous build. Parity of the head kernels, then interleaved C4 benches.
set -o pipefail
OUT=gpurun_out/r4am; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "head_bwd2 or variants" > $OUT/t.log 2>&1 || { tail -20 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
bash tools/ab_bench.sh r4am "" "TRPO_ENGINE_LIB=trpo_amd/libtrpo_engine_sel.so" "TRPO_ENGINE_LIB=trpo_amd/libtrpo_engine_old.so" "" "TRPO_ENGINE_LIB=trpo_amd/libtrpo_engine_sel.so" "TRPO_ENGINE_LIB=trpo_amd/libtrpo_engine_old.so"
