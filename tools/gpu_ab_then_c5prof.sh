# A/B of level-count histogram copies and the packed L0, then C5 kernel stats (tuning only)
set -o pipefail
SKIP_TESTS=1 LIBS="abl/libgkm_cc1.so intree abl/libgkm_cc2.so env:GKM_PACK=1" bash tools/gpu_ab_multi.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_c5
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5/stats -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c5/log.txt 2>&1
cp $(find gpurun_out/prof_c5/stats -name "*kernel_stats.csv" | head -1) gpurun_out/prof_c5/kernel_stats.csv
head -14 gpurun_out/prof_c5/kernel_stats.csv | cut -c1-120
