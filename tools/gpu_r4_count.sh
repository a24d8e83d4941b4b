# Persistent digit-byte count (default) against one workgroup per tile (GKM_COUNT_ONE_PER_TILE=1):
# every GPU test on the new default, then C3 stage times alternating x3 -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/count_ab.txt
for rep in 1 2 3; do
  for v in "GKM_COUNT_ONE_PER_TILE=1" "GKM_X=0"; do
    timeout -k 10 300 env $v python -u tools/exp_stages.py --label "$v" > gpurun_out/count_one.json 2>&1 && tail -1 gpurun_out/count_one.json | tee -a gpurun_out/count_ab.txt || { tail -5 gpurun_out/count_one.json; exit 1; }
  done
done
