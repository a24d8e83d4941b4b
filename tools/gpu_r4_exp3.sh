# Round-4 check of the wide L0 + 8192-key block class (GKM_WIDE_L0=1) -> gpurun_out/:
# every GPU test (routing changed for all sorts: buckets <= 8192 now finish locally), then the C3
# stage times default vs wide, the host side of the packed transfer, the ref_profile 'none' line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for rep in 1 2; do
  for v in 0 1; do
    timeout -k 10 300 env GKM_WIDE_L0=$v python -u tools/exp_stages.py --label "wide=$v" > gpurun_out/exp3_one.json 2>&1 && tail -1 gpurun_out/exp3_one.json | tee -a gpurun_out/exp3.txt || { tail -5 gpurun_out/exp3_one.json; exit 1; }
  done
done
g++ -O3 -mavx2 -pthread tools/host_bw.cpp -o /tmp/host_bw && timeout -k 10 120 /tmp/host_bw | tee gpurun_out/host_bw.txt
timeout -k 10 300 python -u tools/xfer_threads.py 1 4 8 16 32 2>&1 | tee gpurun_out/xfer_threads.txt
timeout -k 10 400 python -u bench.py --config ref_profile --max-kmer-len none --steps 5 --warmup 2 > gpurun_out/bench_ref_none.json 2> gpurun_out/bench_ref_none.err || { tail -20 gpurun_out/bench_ref_none.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_ref_none.json').read().strip().splitlines()[-1]); print('ref none', d['ms_per_step'], d['value'], d['roofline'], d['config']['stages_ms_per_step'])"
