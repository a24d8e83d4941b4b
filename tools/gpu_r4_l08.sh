# An 8-bit L0 for C4 / C5 (GKM_LEVEL_BITS=8: with it the canonical L0 count keeps its fast path,
# the level behind L0 writes packed pairs and the next is compact) against the default 7-bit L0;
# stage times, alternating x2 -> gpurun_out/l08_ab.txt
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/l08_ab.txt
for cfg in c5 c4; do
  for rep in 1 2; do
    for v in "GKM_X=0" "GKM_LEVEL_BITS=8"; do
      timeout -k 10 300 env $v python -u tools/exp_stages.py --config $cfg --label "$cfg $v" > gpurun_out/l08_one.json 2>&1 && tail -1 gpurun_out/l08_one.json | tee -a gpurun_out/l08_ab.txt || { tail -5 gpurun_out/l08_one.json; exit 1; }
    done
  done
done
