# Parity subset on a variant library (GKM_LIB=$VARIANT), then an interleaved bench A/B against $BASE
# (tuning only): VARIANT=abl/x.so BASE=abl/base.so bash tools/gpu_ab_variant.sh -> gpurun_out/abm.txt
set -o pipefail
mkdir -p gpurun_out
GKM_LIB=$VARIANT timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_canonical.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_variant.log 2>&1 || { tail -40 gpurun_out/gpu_tests_variant.log; exit 1; }
tail -2 gpurun_out/gpu_tests_variant.log
SKIP_TESTS=1 LIBS="$BASE $VARIANT" bash tools/gpu_ab_multi.sh
