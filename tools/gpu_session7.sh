# Session-7 evidence on one box: the default bench (C3, CPU baseline included), then the C3
# rocprofv3 kernel-trace stats and the SQ / FETCH_SIZE / WRITE_SIZE passes (tools/profile_r2.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -30 gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
CONFIG=c3 bash tools/profile_r2.sh > gpurun_out/profile.log 2>&1 || { tail -30 gpurun_out/profile.log; exit 1; }
tail -5 gpurun_out/profile.log
