# GPU check of the config-scale parity tests (C2 bit-exact, C3/C4/C5 full-size properties,
# small-chunk branches); progress goes to gpurun_out/configs.log.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v -s --timeout 900 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/configs.log 2>&1 || { tail -60 gpurun_out/configs.log; exit 1; }
tail -30 gpurun_out/configs.log
