# Round-2 (session 4) GPU evidence: every GPU test, the C3 bench, rocprof summaries of C4 and C5,
# and the per-rank multi-GPU emulation of both schemes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -n 2 gpurun_out/gpu_tests.log
for c in c4 c5; do CONFIG=$c bash tools/profile_r2.sh > /dev/null 2>&1 || { echo "profile $c failed"; tail -20 gpurun_out/prof_$c/stats.log; exit 1; }; done
SPECS="c3:range c3:a2a c4:range" bash tools/gpu_emulate.sh
