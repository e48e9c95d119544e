#!/bin/bash
# head_bwd2 prefetch depth 1 (default) vs 2 (libtrpo_engine_hb2.so): parity of both, then interleaved C4 benches
set -o pipefail
OUT=gpurun_out/r4aj; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "head_bwd2 or variants" > $OUT/t_d1.log 2>&1 || { tail -20 $OUT/t_d1.log; exit 1; }
tail -1 $OUT/t_d1.log
TRPO_ENGINE_LIB=trpo_amd/libtrpo_engine_hb2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "head_bwd2 or variants" > $OUT/t_d2.log 2>&1 || { tail -20 $OUT/t_d2.log; exit 1; }
tail -1 $OUT/t_d2.log
bash tools/ab_bench.sh r4aj "" "TRPO_ENGINE_LIB=trpo_amd/libtrpo_engine_hb2.so" "" "TRPO_ENGINE_LIB=trpo_amd/libtrpo_engine_hb2.so"
