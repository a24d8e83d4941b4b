# kernel trace of one key-range rank (tools/range_rank.py) -> gpurun_out/trace_rank_<cfg>_<rank>/
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
cd $R
for r in ${RANKS:-0 1}; do
  OUT=$R/gpurun_out/trace_rank_${CONFIG:-c4}_$r
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT -o run --output-format csv -- python3 tools/range_rank.py --config ${CONFIG:-c4} --rank $r --reps 2 > $OUT/log.txt 2>&1
  grep rep $OUT/log.txt
done
