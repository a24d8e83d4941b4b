# Every GPU test, then the C5 kernel stats + bench line (the key-table fix-up path) -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash tools/gpu_c5prof.sh | head -5 | cut -c1-100
