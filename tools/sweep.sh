# Tuning sweep on one box: one bench run per environment setting (tuning knobs only).
# usage: CONFIG=c3 bash tools/sweep.sh "" "GKM_LEVEL_BITS=8,8,8" "GKM_WAVE_OCC=4 GKM_LEVEL_BITS=7,8,8" ...
# ("" = defaults).  One summary line per setting in gpurun_out/sweep.txt.
set -o pipefail
mkdir -p gpurun_out
C=${CONFIG:-c3}
S=${STEPS:-3}
i=0
for setting in "$@"; do
  i=$((i + 1))
  env $setting timeout -k 10 300 python bench.py --config $C --steps $S --warmup 1 --no-cpu-baseline \
      > gpurun_out/sweep_$i.json 2> gpurun_out/sweep_$i.err || { tail -20 gpurun_out/sweep_$i.err; exit 1; }
  python3 -c "
import json, sys
d = json.loads(open('gpurun_out/sweep_$i.json').read().strip().splitlines()[-1])
s = d['config']['stages_ms_per_step']
print('[$C] ${setting:-default}:', d['ms_per_step'], 'ms', {k: s[k] for k in sorted(s) if s[k] > 0.5})
" | tee -a gpurun_out/sweep.txt
done
