# Pre-packed sequence (GKM_PACK=1: pack2_kernel once per sort, every L0-type pass reads 2-bit words)
# against the in-tile packing, C3 single GPU (stage times) and the N = 8 rank emulation; plus the
# packed-pair tests at k = 24 / 32 -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "packed_pair" --timeout 200 --timeout-method thread > gpurun_out/gpu_pairs.log 2>&1 || { tail -40 gpurun_out/gpu_pairs.log; exit 1; }
tail -1 gpurun_out/gpu_pairs.log
for rep in 1 2; do
  for v in "GKM_X=0" "GKM_PACK=1"; do
    timeout -k 10 300 env $v python -u tools/exp_stages.py --label "$v" > gpurun_out/pack_one.json 2>&1 && tail -1 gpurun_out/pack_one.json | tee -a gpurun_out/pack_ab.txt || { tail -5 gpurun_out/pack_one.json; exit 1; }
  done
done
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
