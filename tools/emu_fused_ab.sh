# A/B of the key-range ranks' fused select (GKM_RANGE_FUSED=1) against the select pass (=0): the
# C3 per-rank emulation at N = 8, 4, 2 for each (tools/range_emulate.py), one process each
set -o pipefail
mkdir -p gpurun_out
for v in 1 0; do
  GKM_RANGE_FUSED=$v timeout -k 10 600 python -u tools/range_emulate.py --config "${1:-c3}" --worlds 8,4,2 \
    > gpurun_out/emu_fused_$v.json 2> gpurun_out/emu_fused_$v.err || { tail -20 gpurun_out/emu_fused_$v.err; exit 1; }
  grep '"world"' gpurun_out/emu_fused_$v.json | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); s=d['slowest_rank_stages_ms']
    print('FUSED=$v', d['world'], d['max_rank_ms'], d['speedup_vs_single'], {k: s[k] for k in s if k.startswith('msd_pass') or k in ('msd_select', 'msd_l0_count', 'histogram')})"
done
