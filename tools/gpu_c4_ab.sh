# Split/merge parity subset, then a C4 bench A/B over $LIBS (tuning only) -> gpurun_out/abm.txt
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  -k "split or iupac or grch38 or surrogate or distributed or range" > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
rm -f gpurun_out/abm.txt
SKIP_TESTS=1 CONFIG=c4 STEPS=3 bash tools/gpu_ab_multi.sh > /dev/null || exit 1
python3 - <<'PY'
import ast
for l in open('gpurun_out/abm.txt'):
    name, rest = l.split(' ', 1)
    ms, d = rest.split(' ', 1)
    d = ast.literal_eval(d.strip())
    print(name, ms, {k: d[k] for k in ('split_merge', 'msd_total', 'unique_counts') if k in d})
PY
