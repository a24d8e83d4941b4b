# Canonical parity subset, then a C5 bench A/B over $LIBS (tuning only) -> gpurun_out/abm.txt
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "key_rows or canonical" > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
rm -f gpurun_out/abm.txt
SKIP_TESTS=1 CONFIG=c5 STEPS=2 bash tools/gpu_ab_multi.sh > /dev/null || exit 1
python3 - <<'PY'
for l in open('gpurun_out/abm.txt'):
    name, rest = l.split(' ', 1)
    import ast
    ms, d = rest.split(' ', 1)
    d = ast.literal_eval(d.strip())
    print(name, ms, {k: d[k] for k in ('reencode_keys', 'msd_l0_count', 'msd_total') if k in d})
PY
