# Round-4 check on one MI355X -> gpurun_out/: the whole GPU suite with the first doubling round on
# seed keys for every shift, then the reference's profiled workload at max 50 and None.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/s2b_tests.log 2>&1 || { tail -30 gpurun_out/s2b_tests.log; exit 1; }
tail -2 gpurun_out/s2b_tests.log
for mx in 50 none; do
  timeout -k 10 300 python -u bench.py --config ref_profile --max-kmer-len $mx > gpurun_out/s2b_ref_$mx.json 2> gpurun_out/s2b_ref_$mx.err || { tail -20 gpurun_out/s2b_ref_$mx.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/s2b_ref_$mx.json').read().strip().splitlines()[-1]); print('$mx', d['ms_per_step'], d['value'], d['config']['sort_path'])"
done
