#!/bin/bash
# Same-box A/B of engine option env settings on one bench config, interleaved rounds.
# usage: bash tools/ab_env.sh <outdir> <config> <rounds> "<envA>" "<envB>" ...   (env "" = defaults)
set -o pipefail
OUT=gpurun_out/$1; CFG=$2; R=$3; shift 3; mkdir -p $OUT
for r in $(seq 1 $R); do
  i=0
  for e in "$@"; do
    timeout -k 10 300 env $e python -u bench.py --config $CFG --steps ${AB_STEPS:-5} --warmup 2 --no-cpu-baseline --no-alt \
      > $OUT/ab_${i}_$r.json 2> $OUT/ab_${i}_$r.err || { echo "variant [$e] failed"; tail -5 $OUT/ab_${i}_$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('$OUT/ab_${i}_$r.json').read().strip().splitlines()[-1]); print('[$e]', 'round $r', round(d['value'],4), 'upd/s', round(d['ms_per_step'],2), 'ms', round(d['fvp']['ms_per_fvp'],3), 'ms/fvp')"
    i=$((i+1))
  done
done
