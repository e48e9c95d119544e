#!/bin/bash
# Time the C4 bench for each wide row-GEMM config (TRPO_ROWCFG), one process each.
set -o pipefail
OUT=gpurun_out/sweep_rowcfg; mkdir -p $OUT
for c in "$@"; do
  TRPO_ROWCFG=$c timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile-out $OUT/prof_$c.json > $OUT/bench_$c.log 2>&1 || { echo "cfg $c failed rc=$?"; exit 1; }
  echo "cfg $c: $(python -c "import json;d=json.loads(open('$OUT/bench_$c.log').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],1),'ms/update')")"
done
