# C5 kernel stats (rocprofv3) and the C5 bench line -> gpurun_out/prof_c5 (tuning / evidence)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_c5
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5/stats -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c5/log.txt 2>&1 || { tail -20 gpurun_out/prof_c5/log.txt; exit 1; }
cp $(find gpurun_out/prof_c5/stats -name "*kernel_stats.csv" | head -1) gpurun_out/prof_c5/kernel_stats.csv
rm -rf gpurun_out/prof_c5/stats
cut -c1-100 gpurun_out/prof_c5/kernel_stats.csv | head -24
