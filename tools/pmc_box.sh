# Where the memory-bound passes differ from box to box (round 6): one unprofiled
# C3 bench line to place the box, then one rocprofv3 --pmc pass per counter group over a 2-step
# bench (each pass within the per-block slot limits of MI355X_MICROARCH.md: <= 4 TCC, <= 4 TCP,
# <= 2 GRBM), summarised per kernel by tools/pmc_summary_any.py.
#   bash tools/pmc_box.sh TAG "CTR1 CTR2 ..." ["CTR ..."] ...   -> gpurun_out/box_TAG/
set -o pipefail
TAG=$1; shift
O=gpurun_out/box_$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline --no-boundary ${BENCH_ARGS:-} \
  > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 tools/line_brief.py $O/bench.json
i=0
for pass in "$@"; do
  i=$((i + 1))
  timeout -s KILL 300 rocprofv3 --pmc $pass -d $O/pmc$i -o run --output-format csv -- python3 bench.py --config c3 \
    --steps 2 --warmup 1 --no-cpu-baseline --no-boundary ${BENCH_ARGS:-} > $O/pmc$i.log 2>&1 || { tail -5 $O/pmc$i.log; exit 1; }
  python3 tools/pmc_summary_any.py "$(find $O/pmc$i -name '*counter_collection.csv' | head -1)" > $O/pass$i.txt
  rm -rf $O/pmc$i
  head -14 $O/pass$i.txt
done
