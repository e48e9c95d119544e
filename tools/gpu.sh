#!/bin/bash
# The one GPU-box recipe (run from the repo root on the box; every GPU step has its own time limit and the
# steps are chained so the first failure ends the call).  Results go to gpurun_out/<name>/.
#
#   bash tools/gpu.sh tests <name> [pytest -k expr]     -m gpu suite (or a -k selection of it)
#   bash tools/gpu.sh smoke <name>                      __graft_entry__.smoke()
#   bash tools/gpu.sh bench <name> <config>... [-- bench args]   one bench line per config (+ HIP-event profile)
#   bash tools/gpu.sh ab <name> <config> <rounds> "<env A>" "<env B>" ...   interleaved same-box A/B of env
#                                                        settings ("" = defaults; TRPO_ENGINE_LIB=... picks a build;
#                                                        AB_STEPS / AB_ARGS: steps and extra bench arguments)
#   bash tools/gpu.sh prof <name> [bench args]          rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes
#   bash tools/gpu.sh sq <name> [bench args]            SQ / GRBM counter passes per kernel (pmc_kernels.sh)
#   bash tools/gpu.sh round <name>                      tests + smoke + C4 (with CPU baseline) / C3 / C2 / C5 lines
#   bash tools/gpu.sh rehearsal <name>                  2-rank rehearsal line on the one GPU (rank digest check)
#   bash tools/gpu.sh rccl <name>                       C4 line at one rank through a one-rank RCCL communicator
#   bash tools/gpu.sh final <name>                      round + rehearsal + rccl + prof
# Several steps: bash tools/gpu.sh chain <name> "tests" "bench c4 c3" "prof" ...  (each a sub-command above
# without its <name>)
set -o pipefail
CMD=$1; NAME=$2; shift 2
OUT=gpurun_out/$NAME
mkdir -p $OUT

summ() {   # one line of a bench JSON file
  python -c "
import json,sys
d=json.loads(open('$1').read().strip().splitlines()[-1])
f=d.get('fvp') or {}
print('%s %.4f upd/s  %.2f ms/update  %.3f ms/FVP  dominant %s %.3f ms frac %.3f' % ('$2', d['value'], d['ms_per_step'],
      f.get('ms_per_fvp', float('nan')), d['roofline']['kernel'], d['roofline']['avg_launch_ms'], d['roofline']['frac']))"
}

case $CMD in
  tests)
    if [ -n "$1" ]; then K=(-k "$1"); else K=(); fi
    TRPO_MARGIN_LOG=$OUT/margins.txt timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 \
      --timeout-method thread "${K[@]}" \
      > $OUT/pytest_gpu.log 2>&1
    rc=$?; tail -3 $OUT/pytest_gpu.log; exit $rc ;;
  smoke)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
    rc=$?; tail -3 $OUT/smoke.log; exit $rc ;;
  bench)
    CFGS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do CFGS+=("$1"); shift; done; [ "$1" == "--" ] && shift
    for c in "${CFGS[@]}"; do
      case $c in
        c4) X="--steps ${STEPS:-20} --warmup 2" ;;
        c5) X="--steps 2 --warmup 1 --no-cpu-baseline --no-alt" ;;
        *)  X="--steps 20 --warmup 3 --no-cpu-baseline --no-alt" ;;
      esac
      timeout -k 10 900 python -u bench.py --config $c $X --profile-out $OUT/events_$c.json "$@" \
        > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -5 $OUT/bench_$c.err; exit 1; }
      summ $OUT/bench_$c.json $c
    done ;;
  ab)
    CFG=$1; R=$2; shift 2
    for r in $(seq 1 $R); do
      i=0
      for e in "$@"; do
        timeout -k 10 300 env $e python -u bench.py --config $CFG --steps ${AB_STEPS:-5} --warmup 2 --no-cpu-baseline \
          --no-alt ${AB_ARGS:-} --profile-out $OUT/ab_${i}_$r.prof.json > $OUT/ab_${i}_$r.json 2> $OUT/ab_${i}_$r.err \
          || { echo "variant [$e] failed"; tail -5 $OUT/ab_${i}_$r.err; exit 1; }
        summ $OUT/ab_${i}_$r.json "[$e] round $r" | tee -a $OUT/ab.txt
        i=$((i+1))
      done
    done ;;
  prof)
    bash tools/prof.sh $NAME "$@" || exit $?
    python tools/pmc_traffic.py gpurun_out/$NAME $OUT/traffic.json > $OUT/traffic.txt 2>&1; tail -3 $OUT/traffic.txt ;;
  sq)
    bash tools/pmc_kernels.sh $NAME "$@" || exit $?
    python tools/pmc_summary.py gpurun_out/$NAME > $OUT/sq_counters.txt 2>&1; tail -3 $OUT/sq_counters.txt ;;
  round)
    bash tools/gpu.sh tests $NAME && bash tools/gpu.sh smoke $NAME && bash tools/gpu.sh bench $NAME c4 c3 c2 c5 ;;
  rehearsal)   # 2 ranks sharing the one GPU (host all-reduce): the launcher and the per-rank digest check
    timeout -k 10 600 python -u bench.py --gpus 2 --rehearsal --rows 400000 --steps 3 --warmup 1 --no-cpu-baseline \
      --no-alt > $OUT/bench_2rank_rehearsal.json 2> $OUT/bench_2rank_rehearsal.err || { tail -5 $OUT/bench_2rank_rehearsal.err; exit 1; }
    python -c "
import json; d=json.loads(open('$OUT/bench_2rank_rehearsal.json').read().strip().splitlines()[-1])
print('rehearsal', d['value'], d['comm'].get('transport'), d['comm'].get('ranks'), d['comm'].get('ranks_bitwise_equal'))" ;;
  rccl)   # every all-reduce through RCCL at world 1 (the N>1 code path minus the peers)
    timeout -k 10 600 python -u bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-alt --rccl-world1 \
      > $OUT/bench_c4_rccl1.json 2> $OUT/bench_c4_rccl1.err || { tail -5 $OUT/bench_c4_rccl1.err; exit 1; }
    summ $OUT/bench_c4_rccl1.json c4-rccl1 ;;
  final)
    bash tools/gpu.sh round $NAME && bash tools/gpu.sh rehearsal $NAME && bash tools/gpu.sh rccl $NAME && bash tools/gpu.sh prof $NAME --steps 3 --warmup 1 --no-alt ;;
  chain)
    for step in "$@"; do
      set -- $step
      sub=$1; shift
      bash tools/gpu.sh $sub $NAME "$@" || exit $?
    done ;;
  *) echo "unknown command $CMD"; exit 2 ;;
esac
