# Clocks, power and temperatures sampled by rocm-smi (about 3 per second) while bench.py runs C3
# steps back to back: does the chip leave its clocks under the sustained memory-bound load (the
# box-to-box and in-process spread of the latency-bound passes)?
#   bash tools/power_sample.sh STEPS  -> gpurun_out/power_samples.txt, gpurun_out/power_bench.json
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/power_samples.txt
: > $O
( while true; do echo "t=$(date +%s.%N)" >> $O; rocm-smi --showpower --showclocks --showtemp --showmemuse --csv >> $O 2>&1; sleep 0.2; done ) &
S=$!
timeout -k 10 600 python -u bench.py --config c3 --steps "${1:-60}" --warmup 5 --no-cpu-baseline --no-boundary \
  > gpurun_out/power_bench.json 2> gpurun_out/power_bench.err
rc=$?
sleep 2
kill $S
wait $S 2>/dev/null
exit $rc
