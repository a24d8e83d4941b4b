set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u tools/range_emulate.py --config c4 --worlds 8 > gpurun_out/emu.json 2> gpurun_out/emu.err || { tail -30 gpurun_out/emu.err; exit 1; }
grep '^{' gpurun_out/emu.json | cut -c1-1500
