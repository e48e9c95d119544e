#!/bin/bash
# round 4: small-N scaling probe (C4 dims at 1M / 2M / 4M states on one GPU), C3 / C2 lines, rocprof stats of C4
set -o pipefail
OUT=gpurun_out/${1:-r4e}; mkdir -p $OUT
for r in 1000000 2000000 4000000; do
  timeout -k 10 300 python -u bench.py --rows $r --steps 10 --warmup 2 --no-cpu-baseline --no-alt --profile-out $OUT/events_c4_$r.json > $OUT/bench_c4_$r.json 2> $OUT/bench_c4_$r.err || { tail $OUT/bench_c4_$r.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_c4_$r.json').read().strip().splitlines()[-1]); print($r, round(d['value'],3), round(d['ms_per_step'],2))"
done
for c in c3 c2; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-alt --profile-out $OUT/events_$c.json > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail $OUT/bench_$c.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_$c.json').read().strip().splitlines()[-1]); print('$c', round(d['value'],3), round(d['ms_per_step'],3))"
done
