# Round-4 last profiles on one MI355X -> gpurun_out/: the C3 bench under rocprofv3 (kernel stats,
# SQ counters, FETCH / WRITE passes; tools/profile_r3.sh), kernel stats of the reference's
# profiled workload at max 10 / 20 / 50 / None, then the C4 bench line.
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
CONFIG=c3 TAG=r4last bash tools/profile_r3.sh > gpurun_out/prof_c3_r4last.log 2>&1 || { tail -30 gpurun_out/prof_c3_r4last.log; exit 1; }
tail -12 gpurun_out/prof_c3_r4last.log
cd /tmp && export TMPDIR=/tmp && cd $R
for mx in 10 20 50 none; do
  OUT=$R/gpurun_out/prof_ref_last_${mx}
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 bench.py --config ref_profile --max-kmer-len $mx --no-cpu-baseline --steps 5 --warmup 1 > $OUT/stats.log 2>&1 || { tail -20 $OUT/stats.log; exit 1; }
  cp $(find $OUT/stats -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
  grep -h '"metric"' $OUT/stats.log > $OUT/bench_line.json || true
  rm -rf $OUT/stats
  echo "ref $mx done"
done
timeout -k 10 600 python -u bench.py --config c4 --no-cpu-baseline > gpurun_out/bench_c4_last.json 2> gpurun_out/bench_c4_last.err || { tail -20 gpurun_out/bench_c4_last.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_c4_last.json').read().strip().splitlines()[-1]); print('c4', d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'])"
