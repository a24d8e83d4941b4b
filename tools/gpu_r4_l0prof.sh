# L0 partition phase profile (GKM_L0_PROF=1: per-phase clock sums of the first and last wave) at C3
set -o pipefail
mkdir -p gpurun_out
GKM_L0_PROF=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/l0prof.json 2> gpurun_out/l0prof.err || { tail -20 gpurun_out/l0prof.err; exit 1; }
grep l0prof gpurun_out/l0prof.err | tail -4
