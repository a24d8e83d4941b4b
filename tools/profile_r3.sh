# Round-3 profile of the bench command: rocprofv3 kernel-trace stats, then one PMC pass each for
# the SQ counters, FETCH_SIZE and WRITE_SIZE (separate passes, MI355X_MICROARCH.md), summarised
# into per-kernel instruction mix and HBM bytes per launch.
# Usage (GPU box): CONFIG=c3 TAG=name bash tools/profile_r3.sh  -> gpurun_out/prof_$CONFIG_$TAG/
set -e
R=$GRAFT_REPO_ROOT
C=${CONFIG:-c3}
OUT=$R/gpurun_out/prof_${C}_${TAG:-r3}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd $R
B="bench.py --config $C --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 $B --steps 3 --warmup 1 > $OUT/stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $OUT/sq -o run --output-format csv -- python3 $B --steps 1 --warmup 1 > $OUT/sq.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $B --steps 1 --warmup 1 > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $B --steps 1 --warmup 1 > $OUT/write.log 2>&1
python3 tools/pmc_summary.py $(find $OUT/sq -name "*counter_collection.csv" | head -1) > $OUT/pmc_sq_summary.txt
python3 tools/pmc_traffic.py $(find $OUT/fetch -name "*counter_collection.csv" | head -1) $(find $OUT/write -name "*counter_collection.csv" | head -1) $OUT/traffic.json --label "${C} ${TAG:-r3}" > $OUT/traffic.txt
cp $(find $OUT/stats -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
grep -h '"metric"' $OUT/stats.log > $OUT/bench_line.json || true
cat $OUT/pmc_sq_summary.txt | head -8; cat $OUT/traffic.txt | head -20
