# gpu_sel_ab.sh, then the key-range emulation of C3 and C4 at N = 8, 4, 2 on the in-tree library
set -o pipefail
bash tools/gpu_sel_ab.sh || exit 1
for cfg in c3 c4; do
  timeout -k 10 500 python -u tools/range_emulate.py --config $cfg --worlds 8,4,2 > gpurun_out/emulate_${cfg}_end.json 2> gpurun_out/emulate_${cfg}_end.err || { tail -20 gpurun_out/emulate_${cfg}_end.err; exit 1; }
  python3 - $cfg <<'PY'
import json, sys
l = [json.loads(x) for x in open(f"gpurun_out/emulate_{sys.argv[1]}_end.json") if x.startswith("{")]
print(sys.argv[1], "single", l[0]["single_gpu_ms"], [(w["world"], w["max_rank_ms"], w["speedup_vs_single"]) for w in l[1:]])
PY
done
