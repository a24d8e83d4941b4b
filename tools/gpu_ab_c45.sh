# Parity subset for the key table / merge paths, then interleaved C5 and C4 bench A/B of abl/libgkm_base.so
# against the in-tree library (tuning only) -> gpurun_out/abm.txt
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  -k "key_rows or canonical or split or grch38 or surrogate" > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
SKIP_TESTS=1 CONFIG=c5 STEPS=2 LIBS="abl/libgkm_base.so intree" bash tools/gpu_ab_multi.sh || exit 1
SKIP_TESTS=1 CONFIG=c4 STEPS=3 LIBS="abl/libgkm_base.so intree" bash tools/gpu_ab_multi.sh || exit 1
