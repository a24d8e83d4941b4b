# key-range select change: distributed + parity GPU tests, then the C3 / C4 emulation at N = 8
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_distributed.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sel_tests.log 2>&1 || { tail -40 gpurun_out/sel_tests.log; exit 1; }
tail -1 gpurun_out/sel_tests.log
for cfg in c3 c4; do
  timeout -k 10 400 python -u tools/range_emulate.py --config $cfg --worlds 8 > gpurun_out/emu_$cfg.json 2> gpurun_out/emu_$cfg.err || { tail -30 gpurun_out/emu_$cfg.err; exit 1; }
  python3 - $cfg <<'PY'
import json, sys
l = [json.loads(x) for x in open(f"gpurun_out/emu_{sys.argv[1]}.json") if x.startswith("{")]
w = l[1]; st = w["slowest_rank_stages_ms"]
print(sys.argv[1], "single", l[0]["single_gpu_ms"], "max", w["max_rank_ms"], "x", w["speedup_vs_single"], "select", st.get("msd_select"), "ranks", w["per_rank_ms"])
PY
done
