set -o pipefail
GKM_LIB=abl/libgkm_l0c.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_variant.log 2>&1 || { tail -40 gpurun_out/gpu_tests_variant.log; exit 1; }
tail -2 gpurun_out/gpu_tests_variant.log
SKIP_TESTS=1 LIBS="intree abl/libgkm_l0c.so" bash tools/gpu_ab_multi.sh
