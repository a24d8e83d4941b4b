set -o pipefail
bash tools/gpu_c4_emulate.sh || exit 1
rm -f gpurun_out/abm.txt
SKIP_TESTS=1 LIBS="intree abl/libgkm_occ4.so" bash tools/gpu_ab_multi.sh
