set -o pipefail
for cfg in "GKM_PREFETCH_REGIONS=1" "GKM_PREFETCH_REGIONS=16 GKM_XFER_THREADS=1" "GKM_PREFETCH_REGIONS=16 GKM_PACK_BLOCKS=1" "GKM_PREFETCH_REGIONS=16 GKM_TEST_CHUNK_TILES=1024" "GKM_PREFETCH_REGIONS=16"; do
  echo "== $cfg"
  env $cfg timeout -k 10 200 python -u tools/prefetch_check.py 300000000 || exit 1
done
