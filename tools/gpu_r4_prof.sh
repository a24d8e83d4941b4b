# Round-4 profiles on one MI355X: the C3 bench under rocprofv3 (kernel stats, SQ counters, FETCH /
# WRITE passes; tools/profile_r3.sh), the reference's profiling workload (kernel stats), then the
# C4 and C5 bench lines -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
CONFIG=c3 TAG=r4 bash tools/profile_r3.sh > gpurun_out/prof_c3_r4.log 2>&1 || { tail -30 gpurun_out/prof_c3_r4.log; exit 1; }
tail -30 gpurun_out/prof_c3_r4.log
cd /tmp && export TMPDIR=/tmp && cd $R
for mx in 20 none; do
  OUT=$R/gpurun_out/prof_ref_${mx}
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 bench.py --config ref_profile --max-kmer-len $mx --no-cpu-baseline --steps 5 --warmup 1 > $OUT/stats.log 2>&1 || { tail -20 $OUT/stats.log; exit 1; }
  cp $(find $OUT/stats -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
  grep -h '"metric"' $OUT/stats.log > $OUT/bench_line.json || true
  head -12 $OUT/kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
done
for cfg in c4 c5; do
  timeout -k 10 600 python -u bench.py --config $cfg --no-cpu-baseline > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err || { tail -20 gpurun_out/bench_$cfg.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_$cfg.json').read().strip().splitlines()[-1]); print('$cfg', d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'], d['config'].get('stages_ms_per_step'))"
done
