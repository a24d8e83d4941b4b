# Round-4 A/B on one MI355X -> gpurun_out/: prefix-doubling seeds of 29 2-bit symbols + a length
# field (default) against 21 3-bit symbols (GKM_SEED3=1), at the reference's profiled workload,
# max 50 and None; the whole GPU suite first.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/s2_tests.log 2>&1 || { tail -30 gpurun_out/s2_tests.log; exit 1; }
tail -2 gpurun_out/s2_tests.log
for rep in 1 2; do
  for mx in none 50; do
    for v in seed2 seed3; do
      if [ $v = seed3 ]; then E="GKM_SEED3=1"; else E="GKM_NONE=0"; fi
      timeout -k 10 300 env $E python -u bench.py --config ref_profile --max-kmer-len $mx > gpurun_out/s2_$v.json 2> gpurun_out/s2_$v.err || { tail -20 gpurun_out/s2_$v.err; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/s2_$v.json').read().strip().splitlines()[-1]); print('$mx $v', d['ms_per_step'], d['value'], d['config']['stages_ms_per_step'])" | tee -a gpurun_out/s2_ab.txt
    done
  done
done
