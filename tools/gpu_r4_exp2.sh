# Block-local finishing on C3-sized buckets: level digit widths 7,6,7 / 7,7,6 leave ~3 K-key buckets
# after three global levels, finished by msd_local_kernel (the block class) -> stage times
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for lb in default 7,6,7 7,7,6; do
    if [ "$lb" = default ]; then E=""; else E="GKM_LEVEL_BITS=$lb"; fi
    timeout -k 10 300 env $E python -u tools/exp_stages.py --label "lb=$lb" > gpurun_out/exp2_one.json 2>&1 && tail -1 gpurun_out/exp2_one.json | tee -a gpurun_out/exp2.txt || { tail -5 gpurun_out/exp2_one.json; exit 1; }
  done
done
# host side of the packed transfer: memory bandwidth of the box's CPU share, set_sequence by threads
g++ -O3 -mavx2 -pthread tools/host_bw.cpp -o /tmp/host_bw && timeout -k 10 120 /tmp/host_bw | tee gpurun_out/host_bw.txt
timeout -k 10 300 python -u tools/xfer_threads.py 1 4 8 16 32 2>&1 | tee gpurun_out/xfer_threads.txt
# prefix doubling stops once every tie is a shared '$'-terminated tail: parity, then the ref_profile line
timeout -k 10 600 python -u -m pytest tests/test_gpu_ref_profile.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "suffix or maxNone or doubling or ref_profile or golden" > gpurun_out/doubling_tests.log 2>&1 || { tail -30 gpurun_out/doubling_tests.log; exit 1; }
tail -1 gpurun_out/doubling_tests.log
timeout -k 10 400 python -u bench.py --config ref_profile --max-kmer-len none --steps 5 --warmup 2 > gpurun_out/bench_ref_none.json 2> gpurun_out/bench_ref_none.err || { tail -20 gpurun_out/bench_ref_none.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_ref_none.json').read().strip().splitlines()[-1]); print('ref none', d['ms_per_step'], d['value'], d['roofline'], d['config']['stages_ms_per_step'])"
