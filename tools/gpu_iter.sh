# Fast iteration on the GPU: a parity subset (golden sorts, oracle checks incl. C2), then the C3
# bench without the CPU leg.  Extra bench flags via BENCH_ARGS.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread -k "golden or oracle or c2 or small_chunks" > gpurun_out/iter_tests.log 2>&1 || { tail -40 gpurun_out/iter_tests.log; exit 1; }
tail -2 gpurun_out/iter_tests.log
timeout -k 10 300 python -u bench.py --steps 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/iter_bench.json 2> gpurun_out/iter_bench.err || { tail -30 gpurun_out/iter_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/iter_bench.json'))
print(d['ms_per_step'], round(d['value']/1e9,2), 'G/s', d['roofline']['frac'], d['config']['stages_ms_per_step'])"
