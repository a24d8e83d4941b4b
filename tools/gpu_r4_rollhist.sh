# Round-4 A/B on one MI355X -> gpurun_out/: the rolling bounded encode with the LSD digit
# histograms fused (default) against the generic encode (GKM_NO_ROLL_HIST=1), at the reference's
# profiled workload, max 10 (the LSD route); the whole GPU suite first.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/rh_tests.log 2>&1 || { tail -30 gpurun_out/rh_tests.log; exit 1; }
tail -2 gpurun_out/rh_tests.log
for rep in 1 2; do
  for v in new old; do
    if [ $v = old ]; then E="GKM_NO_ROLL_HIST=1"; else E="GKM_NONE=0"; fi
    timeout -k 10 300 env $E python -u bench.py --config ref_profile --max-kmer-len 10 > gpurun_out/rh_$v.json 2> gpurun_out/rh_$v.err || { tail -20 gpurun_out/rh_$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/rh_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['value'], d['config']['stages_ms_per_step'])" | tee -a gpurun_out/rh_ab.txt
  done
done
