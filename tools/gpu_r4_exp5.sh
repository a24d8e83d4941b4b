# Packed-pair levels: every GPU test, then C3 stage times with and without them (GKM_NO_PAIRS=1),
# then the default bench line -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "packed_pair or wide_l0" --timeout 200 --timeout-method thread > gpurun_out/gpu_pairs.log 2>&1 || { tail -40 gpurun_out/gpu_pairs.log; exit 1; }
tail -2 gpurun_out/gpu_pairs.log
timeout -k 10 300 python -u tools/xfer_numa2.py > gpurun_out/xfer_numa2.txt 2>&1 || { tail -20 gpurun_out/xfer_numa2.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/xfer_numa2.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for rep in 1 2 3; do
  for v in "GKM_NO_PAIRS=1" "GKM_X=0"; do
    timeout -k 10 300 env $v python -u tools/exp_stages.py --label "$v" > gpurun_out/exp5_one.json 2>&1 && tail -1 gpurun_out/exp5_one.json | tee -a gpurun_out/exp5.txt || { tail -5 gpurun_out/exp5_one.json; exit 1; }
  done
done
timeout -k 10 500 python -u bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -20 gpurun_out/bench_c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_c3.json').read().strip().splitlines()[-1]); print('c3', d['ms_per_step'], d['value'], 'e2e', d['e2e_ms'], d['value_e2e'], d.get('e2e'), d['roofline']['kernel'], d['roofline']['frac'], d['config']['stages_ms_per_step'])"
