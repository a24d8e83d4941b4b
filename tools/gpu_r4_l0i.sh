# L0 tile of 1024 x 18 (in-tree) / 20 / 22 / 24 / 28 positions (abl/ variants): C3 stage times, alternating x2
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/l0i_ab.txt
for rep in 1 2; do
  for v in "" abl/libgkm_l0i20.so abl/libgkm_l0i22.so abl/libgkm_l0i24.so abl/libgkm_l0i28.so; do
    GKM_LIB=$v timeout -k 10 300 python -u tools/exp_stages.py --label "${v:-intree}" > gpurun_out/l0i_one.json 2>&1 && tail -1 gpurun_out/l0i_one.json | tee -a gpurun_out/l0i_ab.txt || { tail -5 gpurun_out/l0i_one.json; exit 1; }
  done
done
