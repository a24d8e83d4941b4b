# rocprofv3 kernel stats + SQ counters of the key-range per-rank emulation at N = 8 (C3)
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_range8
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd $R
E="tools/range_emulate.py --config ${CONFIG:-c3} --scheme ${SCHEME:-range} --worlds 8 --reps 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 $E > $OUT/stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $OUT/sq -o run --output-format csv -- python3 $E > $OUT/sq.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $E > $OUT/fetch.log 2>&1
find $OUT -name "*.csv" | sort
