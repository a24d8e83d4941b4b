# Round-4 A/B on one MI355X -> gpurun_out/heads.txt (profiles/r4/exp_heads_chunk.txt): the 8-key
# wave class storing head flags per element or per aligned 4-flag chunk (GKM_WAVE_HS=1: a variant
# measured no faster and removed afterwards), and the copy-only floors (GKM_EXP_WAVECOPY=1 per
# element, 3 per chunk, 4 without head flags; timing only).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 env GKM_WAVE_HS=1 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "msd or pair or golden or large" > gpurun_out/heads_tests.log 2>&1 || { tail -30 gpurun_out/heads_tests.log; exit 1; }
tail -2 gpurun_out/heads_tests.log
for rep in 1 2; do
  for v in real hs copy1 copy3 copy4; do
    case $v in
      real) E="GKM_NONE=0";; hs) E="GKM_WAVE_HS=1";; copy1) E="GKM_EXP_WAVECOPY=1";;
      copy3) E="GKM_EXP_WAVECOPY=3";; copy4) E="GKM_EXP_WAVECOPY=4";;
    esac
    timeout -k 10 300 env $E python -u tools/exp_stages.py --label "$v" > gpurun_out/heads_one.json 2>&1 && tail -1 gpurun_out/heads_one.json | tee -a gpurun_out/heads.txt || { tail -5 gpurun_out/heads_one.json; exit 1; }
  done
done
