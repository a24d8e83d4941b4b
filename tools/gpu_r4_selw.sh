# Key-range select with registers capped for 8 waves per SIMD (abl/libgkm_selw8.so) against the
# in-tree build: key-range GPU tests on the variant, then the N = 8 rank emulation of C3 and C4
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/selw_ab.txt
GKM_LIB=abl/libgkm_selw8.so timeout -k 10 400 python -u -m pytest tests/test_distributed.py tests/test_gpu_configs.py -m gpu -x -q -k "key_range or key_ranges" --timeout 300 --timeout-method thread > gpurun_out/sel_tests.log 2>&1 || { tail -30 gpurun_out/sel_tests.log; exit 1; }
tail -1 gpurun_out/sel_tests.log
for cfg in c3 c4; do
  for v in "" abl/libgkm_selw8.so; do
    GKM_LIB=$v timeout -k 10 400 python -u tools/range_emulate.py --config $cfg --worlds 8 --reps 2 > gpurun_out/sel_one.txt 2>&1 || { tail -20 gpurun_out/sel_one.txt; exit 1; }
    python3 - "$cfg" "${v:-intree}" >> gpurun_out/selw_ab.txt <<'PY'
import json, sys
ls = [json.loads(l) for l in open("gpurun_out/sel_one.txt") if l.startswith("{")]
w = [d for d in ls if d.get("world") == 8][0]
st = w["slowest_rank_stages_ms"]
print(sys.argv[1], sys.argv[2], "single", ls[0]["single_gpu_ms"], "max_rank", w["max_rank_ms"], "x", w["speedup_vs_single"], "select", st.get("msd_select"), "hist", st.get("histogram"), "total", st.get("msd_total"))
PY
    tail -1 gpurun_out/selw_ab.txt
  done
done
