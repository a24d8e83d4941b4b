# GPU check: all GPU tests, then the C4 / C5 benches (GRCh38-shaped surrogate).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for c in ${CONFIGS:-c4 c5}; do
  timeout -k 10 500 python -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b_$c.json 2> gpurun_out/b_$c.err || { tail -20 gpurun_out/b_$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_$c.json'));print('$c', d['value'], d['ms_per_step'], {k:v for k,v in d['config']['stages_ms_per_step'].items() if v>1})"
done
