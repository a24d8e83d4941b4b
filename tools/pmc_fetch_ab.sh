# FETCH_SIZE / WRITE_SIZE per kernel for one C3 step, default and with an environment setting
# (tuning A/B of traffic).  usage: bash tools/pmc_fetch_ab.sh NAME=VALUE
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/pmcab
for mode in B A; do
  if [ $mode = A ]; then export ${1%%=*}="${1#*=}"; fi
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcab/f$mode -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmcab/f$mode.log 2>&1
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcab/w$mode -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmcab/w$mode.log 2>&1
  python3 tools/pmc_traffic.py gpurun_out/pmcab/f$mode/run_counter_collection.csv gpurun_out/pmcab/w$mode/run_counter_collection.csv gpurun_out/pmcab/traffic_$mode.json --label $mode | grep -E "wave|pipe" | sed "s/^/$mode /"
done
