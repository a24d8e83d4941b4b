# Key-range parity subset on a variant library, then the C3 N = 8 emulation A/B (tuning only)
set -o pipefail
mkdir -p gpurun_out
GKM_LIB=$VAR timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  -k "range or shard or distributed" > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
rm -f gpurun_out/emu_ab.txt
LIBS="$VAR intree" CFGS=c3 bash tools/gpu_emu_ab.sh > /dev/null || exit 1
cat gpurun_out/emu_ab.txt
