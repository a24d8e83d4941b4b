# MSD partition-tile shape sweep (tuning only): bench once per GKM_MSD_SHAPE value
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1
tail -2 gpurun_out/t.log
for s in 0 1 2 3; do
  GKM_MSD_SHAPE=$s timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/shape_$s.log 2>&1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/shape_$s.log').read().strip().splitlines()[-1]); print($s, d['ms_per_step'], d['config']['stages_ms_per_step'])"
done
