# Round-4 final check on one MI355X: every GPU test, smoke, the default C3 bench line, and the
# reference's profiled workload at max 10 / 20 / 50 / None -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
NO_PROFILE=1 bash tools/gpu_round_end.sh || exit 1
for mx in 10 20 50 none; do
  timeout -k 10 300 python -u bench.py --config ref_profile --max-kmer-len $mx > gpurun_out/bench_ref_$mx.json 2> gpurun_out/bench_ref_$mx.err || { tail -20 gpurun_out/bench_ref_$mx.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_ref_$mx.json').read().strip().splitlines()[-1]); print('$mx', d['ms_per_step'], d['value'], d['roofline']['kernel'][:60], d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))"
done
