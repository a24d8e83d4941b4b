# GPU tests on the in-tree library, then an interleaved bench A/B (tuning only) over library builds
# and/or environment settings:
# LIBS="abl/a.so intree env:GKM_SELECT_2PASS=1" bash tools/gpu_ab_multi.sh   -> gpurun_out/abm.txt
set -o pipefail
mkdir -p gpurun_out
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTS:-} > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
for rep in 1 2; do
  for lib in ${LIBS}; do
    unset GKM_LIB
    envs=()
    case "$lib" in
      intree) ;;
      env:*) envs=("${lib#env:}") ;;
      *) export GKM_LIB=$lib ;;
    esac
    timeout -k 10 300 env "${envs[@]}" python bench.py --config ${CONFIG:-c3} --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline > gpurun_out/abm.json 2> gpurun_out/abm.err || { tail -20 gpurun_out/abm.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/abm.json').read().strip().splitlines()[-1]); s=d['config']['stages_ms_per_step']; print('$lib', d['ms_per_step'], {k: s[k] for k in sorted(s) if s[k] > 1})" | tee -a gpurun_out/abm.txt
  done
done
