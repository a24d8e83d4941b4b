# Round-end check on one MI355X: GPU tests, smoke, the default bench line, then the C3 profile
# (kernel stats, SQ counters, FETCH / WRITE passes) -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
tail -1 gpurun_out/bench_default.json | cut -c1-600
[ -n "${NO_PROFILE:-}" ] || TAG=${TAG:-final} bash tools/profile_r3.sh
