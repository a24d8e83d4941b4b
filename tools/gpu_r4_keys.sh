# MSD over in-memory keys for whole-array sorts (variable length, prefix doubling): every GPU test,
# then the reference's profiled workload (max 20 / None) against the LSD passes (GKM_SORT_KEYS_LSD=1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "${TESTS_K:-not nothing}" --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
rm -f gpurun_out/keys_ab.txt
for mx in 10 20 50 none; do
  for v in "GKM_SORT_KEYS_LSD=1" "GKM_X=0"; do
    env $v timeout -k 10 300 python -u bench.py --config ref_profile --max-kmer-len $mx --no-cpu-baseline > gpurun_out/keys_one.json 2> gpurun_out/keys_one.err || { tail -20 gpurun_out/keys_one.err; exit 1; }
    python3 - "$mx $v" >> gpurun_out/keys_ab.txt <<'PY'
import json, sys
d = json.loads(open("gpurun_out/keys_one.json").read().strip().splitlines()[-1])
print(json.dumps({"label": sys.argv[1], "ms_per_step": d["ms_per_step"], "value": d["value"], "kernel": d["roofline"]["kernel"], "frac": d["roofline"]["frac"], "stages": d["config"].get("stages_ms_per_step")}))
PY
    tail -1 gpurun_out/keys_ab.txt
  done
done
