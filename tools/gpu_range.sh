# GPU check of the key-range multi-GPU scheme: all GPU tests, the one-GPU per-rank emulation,
# and bench.py through the distributed path at N = 1.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u tools/range_emulate.py > gpurun_out/range_emulate.json 2> gpurun_out/range_emulate.err || { tail -20 gpurun_out/range_emulate.err; exit 1; }
cat gpurun_out/range_emulate.json
timeout -k 10 300 python -u bench.py --sharded --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_range1.json 2> gpurun_out/b_range1.err || { tail -20 gpurun_out/b_range1.err; exit 1; }
cat gpurun_out/b_range1.json
