set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_canonical.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/kt_tests.log 2>&1 || { tail -40 gpurun_out/kt_tests.log; exit 1; }
tail -n 1 gpurun_out/kt_tests.log
CONFIG=c5 bash tools/sweep.sh "" "GKM_NO_KEY_TABLE=1"
