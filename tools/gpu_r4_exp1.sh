# Round-4 session measurements on one MI355X -> gpurun_out/:
#   ref_profile GPU tests; the default bench line (C3, now with the measured end-to-end interval);
#   bench --config ref_profile for max_kmer_len 20 and none; stage times with the wave kernel's
#   copy-only variant (GKM_EXP_WAVECOPY, timing only) against the real one.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ref_profile.py -x -q --timeout 240 --timeout-method thread > gpurun_out/refprof_tests.log 2>&1 || { tail -30 gpurun_out/refprof_tests.log; exit 1; }
tail -1 gpurun_out/refprof_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -20 gpurun_out/bench_c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_c3.json').read().strip().splitlines()[-1]); print('c3', d['ms_per_step'], d['value'], 'e2e', d['e2e_ms'], d['value_e2e'], d.get('e2e'), d['config']['transfers'], 'cpu', d['cpu_baseline']['value'])"
for M in 20 none; do
  timeout -k 10 400 python -u bench.py --config ref_profile --max-kmer-len $M --steps 5 --warmup 2 > gpurun_out/bench_ref_$M.json 2> gpurun_out/bench_ref_$M.err || { tail -20 gpurun_out/bench_ref_$M.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_ref_$M.json').read().strip().splitlines()[-1]); print('ref $M', d['ms_per_step'], d['value'], d['roofline']['frac'], d['config']['stages_ms_per_step'], 'cpu', d['cpu_baseline']['value'])"
done
for rep in 1 2; do
  timeout -k 10 300 python -u tools/exp_stages.py --label real > gpurun_out/exp_real.json 2>&1 && tail -1 gpurun_out/exp_real.json | tee -a gpurun_out/exp.txt
  timeout -k 10 300 env GKM_EXP_WAVECOPY=1 python -u tools/exp_stages.py --label wavecopy > gpurun_out/exp_copy.json 2>&1 && tail -1 gpurun_out/exp_copy.json | tee -a gpurun_out/exp.txt
done
