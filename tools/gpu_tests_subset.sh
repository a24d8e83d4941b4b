# GPU run of selected test files (TESTS, default: contracts + distributed), verbose log in gpurun_out/subset.log
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_contracts.py tests/test_distributed.py} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/subset.log 2>&1 || { tail -60 gpurun_out/subset.log; exit 1; }
tail -5 gpurun_out/subset.log
