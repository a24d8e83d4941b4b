# Build libgkm.so of an earlier commit into abl/ for A/B runs (tuning only):
#   bash tools/build_rev.sh REV NAME   -> abl/libgkm_NAME.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; N=$2
W=/tmp/gkm_rev_$N
rm -rf $W && mkdir -p $W $R/abl
git -C $R archive $REV genome-kmers_amd/csrc include | tar -x -C $W
make -s -j8 -C $W/genome-kmers_amd/csrc ROOT=$W OUT=$R/abl/libgkm_$N.so >/dev/null
echo "built abl/libgkm_$N.so ($REV)"
