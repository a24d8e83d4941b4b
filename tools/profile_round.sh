# Round profile: bench line (with CPU baseline), rocprofv3 kernel stats, PMC FETCH/WRITE traffic.
# Usage (GPU box): bash tools/profile_round.sh  -> gpurun_out/prof/*
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof
mkdir -p $OUT
cd $R
timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log > $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/write.log 2>&1
find $OUT -name "*.csv" | sort
