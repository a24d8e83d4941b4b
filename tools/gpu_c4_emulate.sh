set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_distributed.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/dist_tests.log 2>&1 || { tail -40 gpurun_out/dist_tests.log; exit 1; }
tail -2 gpurun_out/dist_tests.log
timeout -k 10 500 python -u tools/range_emulate.py --config c4 --worlds 8,4,2 > gpurun_out/emulate_c4_gather.json 2> gpurun_out/emulate_c4_gather.err || { tail -30 gpurun_out/emulate_c4_gather.err; exit 1; }
cat gpurun_out/emulate_c4_gather.json
timeout -k 10 300 python -u tools/range_emulate.py --config c4 --worlds 8 --b-scan > gpurun_out/emulate_c4_scan.json 2> gpurun_out/emulate_c4_scan.err || { tail -30 gpurun_out/emulate_c4_scan.err; exit 1; }
cat gpurun_out/emulate_c4_scan.json
