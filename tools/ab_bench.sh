#!/bin/bash
# A/B of kernel-variant switches on the default bench (GPU box, repo root).
# usage: bash tools/ab_bench.sh <outdir-name> "ENV=V ENV2=V" "ENV=V" ...   (one bench run per argument)
set -o pipefail
NAME=$1; shift
OUT=gpurun_out/$NAME
mkdir -p $OUT
i=0
for SETTING in "$@"; do
  i=$((i+1))
  echo "== run $i: $SETTING" | tee -a $OUT/summary.txt
  env $SETTING timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-alt --steps 3 --warmup 1 \
      --profile-out $OUT/prof$i.json > $OUT/bench$i.json 2> $OUT/bench$i.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "run $i failed rc=$rc" | tee -a $OUT/summary.txt; tail -5 $OUT/bench$i.err; exit $rc; fi
  python -c "
import json,sys
d=json.loads(open('$OUT/bench$i.json').read().strip().splitlines()[-1])
p=json.load(open('$OUT/prof$i.json'))['profile']
print('updates/s %.4f  ms/update %.1f  ms/FVP %.2f' % (d['value'], d['ms_per_step'], d['fvp']['ms_per_fvp']))
for k,(c,ms) in sorted(p.items(), key=lambda x:-x[1][1])[:10]: print('   %-18s %3d %8.3f ms' % (k, c, ms/c))
" | tee -a $OUT/summary.txt
done
