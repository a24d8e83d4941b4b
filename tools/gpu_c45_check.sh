# C4 / C5 bench lines (no CPU baseline) -> gpurun_out/bench_c4.json, bench_c5.json
set -o pipefail
mkdir -p gpurun_out
for c in c4 c5; do
  timeout -k 10 400 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { tail -30 gpurun_out/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_$c.json').read().strip().splitlines()[-1]); s=d['config']['stages_ms_per_step']; print('$c', d['ms_per_step'], d['value'], {k: s[k] for k in sorted(s) if s[k] > 1})"
done
