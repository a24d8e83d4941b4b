# Session-7 end: every GPU test, smoke(), the default bench (C3 with the CPU baseline), then the C3
# rocprofv3 kernel stats + SQ / FETCH_SIZE / WRITE_SIZE passes (tools/profile_r2.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -30 gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
CONFIG=c3 bash tools/profile_r2.sh > gpurun_out/profile.log 2>&1 || { tail -30 gpurun_out/profile.log; exit 1; }
tail -2 gpurun_out/profile.log
