#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r4af}; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests/test_gpu_full_size.py -x -v -s --timeout 800 --timeout-method thread > $OUT/pytest_full.log 2>&1
rc=$?; grep "rel L2\|passed\|failed\|Error" $OUT/pytest_full.log | tail -16; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for v in "" "TRPO_SPLITS=64 TRPO_PG_SPLITS=256"; do
  timeout -k 10 300 env $v python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-alt > $OUT/c5_$r.json 2> $OUT/c5_$r.err || { tail $OUT/c5_$r.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/c5_$r.json').read().strip().splitlines()[-1]); print('[$v]', round(d['value'],4), round(d['ms_per_step'],1))"
done
done
