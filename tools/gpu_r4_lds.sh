# LDS / issue-stall counters of the C3 passes (one --pmc pass; counters checked against rocprofv3 -L first)
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_c3_lds
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
WANT="SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS"
HAVE=""
for c in $WANT; do grep -q "\b$c\b" $OUT/counters.txt && HAVE="$HAVE $c"; done
echo "counters:$HAVE"
timeout -s KILL 150 rocprofv3 --pmc $HAVE -d $OUT/sq -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/sq.log 2>&1 || { tail -20 $OUT/sq.log; exit 1; }
python3 tools/pmc_summary.py $(find $OUT/sq -name "*counter_collection.csv" | head -1) > $OUT/pmc_summary.txt
head -8 $OUT/pmc_summary.txt
