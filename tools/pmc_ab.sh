# SQ counters per kernel over one bench step, for several library builds (tuning only):
#   LIBS="abl/a.so intree" bash tools/pmc_ab.sh   -> gpurun_out/pmc_ab/<name>/ + summary.txt
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_ab
mkdir -p $O
cd $R
for lib in ${LIBS}; do
  n=$(basename $lib .so)
  if [ "$lib" = intree ]; then unset GKM_LIB; else export GKM_LIB=$lib; fi
  timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $O/$n -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/$n.log 2>&1
  f=$(find $O/$n -name "*counter_collection.csv" | head -1)
  echo "== $n" >> $O/summary.txt
  python3 tools/pmc_summary.py $f | grep -E "wave_kernel|pipe_kernel|msd0" >> $O/summary.txt
done
cat $O/summary.txt
