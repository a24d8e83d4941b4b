# key-range iteration: the distributed + config GPU tests, then the C3 per-rank emulation at N = 8
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_distributed.py tests/test_gpu_configs.py -m gpu -x -q --timeout 600 --timeout-method thread -k "not full_size" > gpurun_out/range_tests.log 2>&1 || { tail -40 gpurun_out/range_tests.log; exit 1; }
tail -2 gpurun_out/range_tests.log
timeout -k 10 400 python -u tools/range_emulate.py --config ${CONFIG:-c3} --scheme range --worlds ${WORLDS:-8} > gpurun_out/emulate_iter.json 2> gpurun_out/emulate_iter.err || { tail -20 gpurun_out/emulate_iter.err; exit 1; }
cat gpurun_out/emulate_iter.json
