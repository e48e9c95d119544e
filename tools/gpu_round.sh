#!/bin/bash
# Full GPU validation of the current tree (GPU box, repo root): the -m gpu suite, smoke(), the
# default C4 bench line (with the CPU baseline) and C3 / C2 lines.  usage: bash tools/gpu_round.sh <outdir>
set -o pipefail
OUT=gpurun_out/${1:-round}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 600 python -u bench.py --profile-out $OUT/events_c4.json > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail $OUT/bench_c4.err; exit 1; }
tail -1 $OUT/bench_c4.json | cut -c1-300
for c in c3 c2; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --profile-out $OUT/events_$c.json > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail $OUT/bench_$c.err; exit 1; }
  tail -1 $OUT/bench_$c.json | cut -c1-200
done
