# GPU check of the multi-word / canonical paths: parity tests, then the bench at C3, C4, C5.
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_canonical.py tests/test_distributed.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1 || { tail -30 gpurun_out/par.log; exit 1; }
tail -2 gpurun_out/par.log
for c in ${CONFIGS:-c4 c5}; do
  timeout -k 10 500 python -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b_$c.json 2> gpurun_out/b_$c.err || { tail -20 gpurun_out/b_$c.err; exit 1; }
  cat gpurun_out/b_$c.json
done
