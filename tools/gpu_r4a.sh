#!/bin/bash
# round 4 first GPU pass: GPU suite, C4 bench, the self-launched 2-rank rehearsal, --gpus 8 refusal
set -o pipefail
OUT=gpurun_out/${1:-r4a}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --profile-out $OUT/events_c4.json > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail $OUT/bench_c4.err; exit 1; }
tail -1 $OUT/bench_c4.json | cut -c1-400
timeout -k 10 300 python -u bench.py --gpus 2 --rehearsal --rows 400000 --no-alt > $OUT/bench_2rank.json 2> $OUT/bench_2rank.err || { tail $OUT/bench_2rank.err; exit 1; }
tail -1 $OUT/bench_2rank.json | cut -c1-300
timeout -k 10 120 python -u bench.py --gpus 8 > $OUT/bench_8.out 2> $OUT/bench_8.err; echo "gpus8 rc=$? stdout_lines=$(wc -l < $OUT/bench_8.out)"; tail -2 $OUT/bench_8.err
for a in 0 1 2; do timeout -k 10 120 tools/bin/pbench_a$a 8000000 5 0 1 > $OUT/pbench_a$a.txt 2>&1 || { echo "pbench $a failed"; cat $OUT/pbench_a$a.txt; exit 1; }; cat $OUT/pbench_a$a.txt; done
