# C5 bench A/B of environment settings (tuning only) -> gpurun_out/abm.txt
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/abm.txt
SKIP_TESTS=1 CONFIG=c5 STEPS=2 bash tools/gpu_ab_multi.sh > /dev/null || exit 1
python3 - <<'PY'
import ast
for l in open('gpurun_out/abm.txt'):
    name, rest = l.split(' ', 1)
    ms, d = rest.split(' ', 1)
    d = ast.literal_eval(d.strip())
    print(name, ms, {k: v for k, v in d.items() if k.startswith('msd_pass') or k in ('msd_total', 'reencode_keys')})
PY
