# Round-4 prefix doubling on one MI355X -> gpurun_out/: the doubling / variable-length GPU tests,
# the reference's profiled workload at max 50 and None, and a kernel-trace profile of max None.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -x -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/dbl_tests.log 2>&1 || { tail -30 gpurun_out/dbl_tests.log; exit 1; }
tail -2 gpurun_out/dbl_tests.log
for mx in 50 none; do
  timeout -k 10 300 python -u bench.py --config ref_profile --max-kmer-len $mx > gpurun_out/dbl_ref_$mx.json 2> gpurun_out/dbl_ref_$mx.err || { tail -20 gpurun_out/dbl_ref_$mx.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/dbl_ref_$mx.json').read().strip().splitlines()[-1]); print('$mx', d['ms_per_step'], d['value'], d['config']['stages_ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_dbl -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config ref_profile --max-kmer-len none --steps 5 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_dbl.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_dbl.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof_dbl -name "*kernel_stats.csv" | head -3
