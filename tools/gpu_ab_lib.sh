set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for mode in B A B A; do
  if [ $mode = B ]; then export GKM_LIB=abl/libgkm_base.so; else unset GKM_LIB; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$mode.json 2> gpurun_out/ab_$mode.err || { tail -20 gpurun_out/ab_$mode.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_$mode.json').read().strip().splitlines()[-1]); s=d['config']['stages_ms_per_step']; print('$mode', d['ms_per_step'], {k: s[k] for k in sorted(s) if s[k] > 1})" | tee -a gpurun_out/ab.txt
done
