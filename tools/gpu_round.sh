# Round GPU check: every GPU test (progress in gpurun_out/gpu_tests.log), then the default bench
# (C3, with the CPU baseline) -> gpurun_out/bench_c3.json.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -30 gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
