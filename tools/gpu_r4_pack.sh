# Pre-packed sequence (GKM_PACK=1: pack2_kernel once per sort, every L0-type pass reads 2-bit words)
# against the in-tile packing, C3 single GPU (stage times) and the N = 8 rank emulation; plus the
# packed-pair tests at k = 24 / 32 -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/pack_ab.txt
for v in "GKM_X=0" "GKM_PACK=1"; do
  env $v timeout -k 10 400 python -u tools/range_emulate.py --config c3 --worlds 8 --reps 2 > gpurun_out/sel_one.txt 2>&1 || { tail -20 gpurun_out/sel_one.txt; exit 1; }
  python3 - "$v" >> gpurun_out/pack_ab.txt <<'PY'
import json, sys
ls = [json.loads(l) for l in open("gpurun_out/sel_one.txt") if l.startswith("{")]
w = [d for d in ls if d.get("world") == 8][0]
print(json.dumps({"label": "emulate c3 N=8 " + sys.argv[1], "single": ls[0]["single_gpu_ms"], "max_rank": w["max_rank_ms"], "x": w["speedup_vs_single"], "stages": w["slowest_rank_stages_ms"]}))
PY
  tail -1 gpurun_out/pack_ab.txt
done
