# Every GPU test, then a C3 A/B sweep of one environment setting (tuning loop)
# usage: bash tools/gpu_full_ab.sh NAME=VALUE
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -n 1 gpurun_out/gpu_tests.log
bash tools/sweep.sh "" "$1" "" "$1"
