# L0 store-group split A/B (tuning only): in-tree (2 top, 2 scan) vs 4 top vs 4 scan
set -o pipefail
SKIP_TESTS=1 LIBS="${LIBS:-intree abl/libgkm_t4.so abl/libgkm_s4.so}" bash tools/gpu_ab_multi.sh
