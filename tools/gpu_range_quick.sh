# Key-range GPU tests and the C3 N=8 per-rank emulation (tuning loop)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_distributed.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread -k "key_range or small_chunks or shards" > gpurun_out/range_tests.log 2>&1 || { tail -40 gpurun_out/range_tests.log; exit 1; }
tail -n 1 gpurun_out/range_tests.log
timeout -k 10 300 python -u tools/range_emulate.py --config c3 --scheme range --worlds ${WORLDS:-8} > gpurun_out/emulate_q.json 2> gpurun_out/emulate_q.err || { tail -20 gpurun_out/emulate_q.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/emulate_q.json'):
    d = json.loads(l)
    if 'world' in d: print(d['world'], d['max_rank_ms'], d['speedup_vs_single'], {k: v for k, v in d['slowest_rank_stages_ms'].items() if v > 0.1})
    else: print('single', d['single_gpu_ms'])
"
