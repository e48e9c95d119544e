#!/bin/bash
# A/B of kernel-variant env settings on one bench config (GPU box, repo root).
# usage: bash tools/ab_cfg.sh <outdir> <config> "ENV=V ..." "ENV=V" ...
set -o pipefail
NAME=$1; CFG=$2; shift 2
OUT=gpurun_out/$NAME; mkdir -p $OUT
i=0
for SETTING in "$@"; do
  i=$((i+1))
  env $SETTING timeout -k 10 300 python -u bench.py --config $CFG --no-cpu-baseline --no-alt --steps 20 --warmup 3 \
      --profile-out $OUT/prof_${CFG}_$i.json > $OUT/bench_${CFG}_$i.json 2> $OUT/bench_${CFG}_$i.err || { echo "run $i ($SETTING) failed"; tail -5 $OUT/bench_${CFG}_$i.err; exit 1; }
  python -c "
import json
d=json.loads(open('$OUT/bench_${CFG}_$i.json').read().strip().splitlines()[-1])
p=json.load(open('$OUT/prof_${CFG}_$i.json'))['profile']
top=' '.join('%s=%.3f' % (k, ms/c) for k,(c,ms) in sorted(p.items(), key=lambda x:-x[1][1])[:4])
print('$CFG [$SETTING] %.2f upd/s %.3f ms/upd | %s' % (d['value'], d['ms_per_step'], top))
" | tee -a $OUT/summary.txt
done
