# Build a compile-time variant of libgkm.so for A/B runs (tuning only):
#   bash tools/build_variant.sh NAME "-DGKM_X=1 ..."   -> abl/libgkm_NAME.so
#   experiments that write wrong output on purpose (GKM_EXP_*, GKM_L0_PROF) need -DGKM_EXPERIMENTS
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; F=$2
W=/tmp/gkm_variant_$N
rm -rf $W && mkdir -p $W && cp -r $R/genome-kmers_amd/csrc $W/ && mkdir -p $W/genome_kmers $R/abl
make -s -j8 -C $W/csrc ROOT=$R OUT=$R/abl/libgkm_$N.so \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include -Wall -Wno-unused-function -Wno-unused-value -Wno-unused-result $F" >/dev/null
echo "built abl/libgkm_$N.so ($F)"
