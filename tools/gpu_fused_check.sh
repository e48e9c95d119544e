set -o pipefail
mkdir -p gpurun_out/r2b
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "fused_fvp or fvp_and_grad or update_vs_golden or chain_shapes or graph_replay" > gpurun_out/r2b/pytest_fused.log 2>&1 || { tail -30 gpurun_out/r2b/pytest_fused.log; exit 1; }
tail -5 gpurun_out/r2b/pytest_fused.log
for c in c3 c2; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --profile-out gpurun_out/r2b/events_$c.json > gpurun_out/r2b/bench_$c.json 2> gpurun_out/r2b/bench_$c.err || { tail -20 gpurun_out/r2b/bench_$c.err; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/r2b/bench_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d['fvp']['ms_per_fvp'])
p=json.load(open('gpurun_out/r2b/events_$c.json'))['profile']
for k,(c,ms) in sorted(p.items(), key=lambda x:-x[1][1])[:8]: print('   %-18s %3d %8.3f ms' % (k, c, ms/c))
"
done
