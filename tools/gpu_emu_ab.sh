# interleaved A/B of the key-range emulation over library builds (tuning only):
#   LIBS="abl/libgkm_x.so intree" CFGS="c3 c4" bash tools/gpu_emu_ab.sh  -> gpurun_out/emu_ab.txt
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for cfg in ${CFGS:-c3}; do
  for lib in ${LIBS}; do
    unset GKM_LIB
    [ "$lib" = intree ] || export GKM_LIB=$lib
    timeout -k 10 400 python -u tools/range_emulate.py --config $cfg --worlds ${WORLDS:-8} > gpurun_out/emu_ab.json 2> gpurun_out/emu_ab.err || { tail -30 gpurun_out/emu_ab.err; exit 1; }
    python3 - $cfg $lib <<'PY' | tee -a gpurun_out/emu_ab.txt
import json, sys
l = [json.loads(x) for x in open("gpurun_out/emu_ab.json") if x.startswith("{")]
w = l[1]; st = w["slowest_rank_stages_ms"]
print(sys.argv[1], sys.argv[2], "single", l[0]["single_gpu_ms"], "max", w["max_rank_ms"], "x", w["speedup_vs_single"], "select", st.get("msd_select"), "mean", w["mean_rank_ms"])
PY
  done
done
done
