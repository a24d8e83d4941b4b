set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_distributed.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread -k "key_range or small_chunks or shards" > gpurun_out/range_tests.log 2>&1 || { tail -40 gpurun_out/range_tests.log; exit 1; }
tail -2 gpurun_out/range_tests.log
timeout -k 10 300 python -u tools/range_emulate.py --config c3 --scheme range --worlds 8,4,2 > gpurun_out/emulate_c3_range.json 2> gpurun_out/emulate_c3_range.err || { tail -20 gpurun_out/emulate_c3_range.err; exit 1; }
cat gpurun_out/emulate_c3_range.json
GKM_SELECT_2PASS=1 timeout -k 10 300 python -u tools/range_emulate.py --config c3 --scheme range --worlds 8 > gpurun_out/emulate_c3_range_2pass.json 2> gpurun_out/emulate_c3_range_2pass.err || { tail -20 gpurun_out/emulate_c3_range_2pass.err; exit 1; }
cat gpurun_out/emulate_c3_range_2pass.json
