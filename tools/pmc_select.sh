# Counters of one key-range rank (tools/range_rank.py): kernel stats, SQ mix, FETCH, WRITE passes
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_rank_${CONFIG:-c3}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd $R
P="tools/range_rank.py --config ${CONFIG:-c3} --reps 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 $P > $OUT/stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $OUT/sq -o run --output-format csv -- python3 $P > $OUT/sq.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $P > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $P > $OUT/write.log 2>&1
python3 tools/pmc_summary.py $(find $OUT/sq -name "*counter_collection.csv" | head -1) > $OUT/pmc_sq_summary.txt
python3 tools/pmc_traffic.py $(find $OUT/fetch -name "*counter_collection.csv" | head -1) $(find $OUT/write -name "*counter_collection.csv" | head -1) $OUT/traffic.json --label "rank ${CONFIG:-c3}" > $OUT/traffic.txt
cp $(find $OUT/stats -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
head -12 $OUT/kernel_stats.csv | cut -c1-150
cat $OUT/pmc_sq_summary.txt | head -6; head -12 $OUT/traffic.txt
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $OUT/sq2 -o run --output-format csv -- python3 $P > $OUT/sq2.log 2>&1 && python3 tools/pmc_summary.py $(find $OUT/sq2 -name "*counter_collection.csv" | head -1) > $OUT/pmc_sq2_summary.txt && head -6 $OUT/pmc_sq2_summary.txt
