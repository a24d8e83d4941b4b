# Key-table parity subset, a C5 bench A/B (abl/libgkm_base.so vs in-tree) and the C5 kernel stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  -k "key_rows or canonical or grch38" > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
rm -f gpurun_out/abm.txt
SKIP_TESTS=1 CONFIG=c5 STEPS=2 LIBS="abl/libgkm_base.so intree" bash tools/gpu_ab_multi.sh > /dev/null || exit 1
cat gpurun_out/abm.txt | cut -c1-60
bash tools/gpu_c5prof.sh | head -6 | cut -c1-100
