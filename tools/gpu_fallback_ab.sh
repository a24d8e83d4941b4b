# Forced ballot-match ranking parity tests, then an interleaved C3 bench A/B of the in-tree library
# against abl/libgkm_base.so (the cost of the ranking-mode branch) -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rank_fallback.py tests/test_gpu_reference_order.py tests/test_gpu_xfer.py -x -q --timeout 300 --timeout-method thread > gpurun_out/fallback_tests.log 2>&1 || { tail -40 gpurun_out/fallback_tests.log; exit 1; }
tail -2 gpurun_out/fallback_tests.log
SKIP_TESTS=1 LIBS="${LIBS:-abl/libgkm_base.so intree}" bash tools/gpu_ab_multi.sh
