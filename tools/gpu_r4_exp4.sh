# Round-4 bench lines on one MI355X -> gpurun_out/: the default C3 line (end to end from pinned
# memory), ref_profile (max_kmer_len 20), and the host topology behind the packed transfer.
set -o pipefail
mkdir -p gpurun_out
(lscpu; numactl --hardware 2>&1 || true; cat /sys/devices/system/node/node*/cpulist 2>/dev/null; nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true) > gpurun_out/topology.txt 2>&1
timeout -k 10 500 python -u bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -20 gpurun_out/bench_c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_c3.json').read().strip().splitlines()[-1]); print('c3', d['ms_per_step'], d['value'], 'e2e', d['e2e_ms'], d['value_e2e'], d.get('e2e'), d['config']['transfers'], d['roofline']['kernel'], d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'])"
timeout -k 10 400 python -u bench.py --config ref_profile --max-kmer-len 20 --steps 5 --warmup 2 > gpurun_out/bench_ref_20.json 2> gpurun_out/bench_ref_20.err || { tail -20 gpurun_out/bench_ref_20.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_ref_20.json').read().strip().splitlines()[-1]); print('ref 20', d['ms_per_step'], d['value'], d['roofline'], d['config']['stages_ms_per_step'], 'cpu', d['cpu_baseline']['value'])"
timeout -k 10 300 env XFER_NUMA_AB=1 python -u tools/xfer_threads.py 8 16 32 2>&1 | tee gpurun_out/xfer_threads_numa.txt
for rep in 1 2; do
  for v in 0 1 2; do
    if [ $v = 0 ]; then E=""; else E="GKM_EXP_WAVECOPY=$v"; fi
    timeout -k 10 300 env $E python -u tools/exp_stages.py --label "wavecopy=$v" > gpurun_out/exp4_one.json 2>&1 && tail -1 gpurun_out/exp4_one.json | tee -a gpurun_out/exp4.txt || { tail -5 gpurun_out/exp4_one.json; exit 1; }
  done
done
