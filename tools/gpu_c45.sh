# Parity of the key paths (canonical, split, goldens, config-scale incl. full-size key checks),
# then the C4 / C5 bench lines -> gpurun_out/bench_c4.json, bench_c5.json
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_canonical.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/c45_tests.log 2>&1 || { tail -40 gpurun_out/c45_tests.log; exit 1; }
tail -2 gpurun_out/c45_tests.log
for c in ${CONFIGS:-c4 c5}; do
  timeout -k 10 400 python -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { tail -20 gpurun_out/bench_$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/bench_$c.json'))
print('$c', d['ms_per_step'], round(d['value']/1e9,2), 'G/s', d['config']['stages_ms_per_step'])"
done
