# Back-to-back C3 bench processes with the GPU's clocks / temperature / power read (read-only) before
# each: does the level passes' slowdown under sustained load follow the clocks? -> gpurun_out/drift/
set -o pipefail
mkdir -p gpurun_out/drift
for i in 1 2 3 4 5 6 7; do
  { echo "== run $i $(date +%s)"; timeout -k 5 30 rocm-smi --showtemp --showpower --showclocks 2>&1 | grep -v "^=\|^$" | head -40; } >> gpurun_out/drift/smi.txt || true
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/drift/b$i.json 2> gpurun_out/drift/b$i.err || { tail -20 gpurun_out/drift/b$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/drift/b$i.json').read().strip().splitlines()[-1]); s=d['config']['stages_ms_per_step']; print($i, d['ms_per_step'], s['msd_pass_l1'], s['msd_pass_l2c'], s['msd_local_wave8'], s['msd_pass_l0'])" | tee -a gpurun_out/drift/summary.txt
done
{ echo "== end $(date +%s)"; timeout -k 5 30 rocm-smi --showtemp --showpower --showclocks 2>&1 | grep -v "^=\|^$" | head -40; } >> gpurun_out/drift/smi.txt || true
