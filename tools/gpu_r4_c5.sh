# Every GPU test, then the C5 bench line (8-bit canonical L0 default) -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 600 python -u bench.py --config c5 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { tail -20 gpurun_out/bench_c5.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_c5.json').read().strip().splitlines()[-1]); print('c5', d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'])"
