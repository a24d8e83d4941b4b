# select-kernel prefetch depth A/B on the key-range emulation (tuning only) -> gpurun_out/sel_ab.txt
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_distributed.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/dist_tests.log 2>&1 || { tail -40 gpurun_out/dist_tests.log; exit 1; }
tail -1 gpurun_out/dist_tests.log
for cfg in ${CFGS:-c3 c4}; do
  for lib in ${LIBS:-abl/libgkm_sel1.so intree abl/libgkm_sel3.so}; do
    unset GKM_LIB
    [ "$lib" = intree ] || export GKM_LIB=$lib
    timeout -k 10 400 python -u tools/range_emulate.py --config $cfg --worlds 8 > gpurun_out/sel_ab.json 2> gpurun_out/sel_ab.err || { tail -30 gpurun_out/sel_ab.err; exit 1; }
    python3 - "$cfg" "$lib" <<'PY' | tee -a gpurun_out/sel_ab.txt
import json, sys
lines = [json.loads(l) for l in open("gpurun_out/sel_ab.json") if l.startswith("{")]
s, w = lines[0], lines[1]
st = w["slowest_rank_stages_ms"]
print(sys.argv[1], sys.argv[2], "single", s["single_gpu_ms"], "max", w["max_rank_ms"], "x", w["speedup_vs_single"],
      "select", st.get("msd_select"), "ranks", w["per_rank_ms"])
PY
  done
done
