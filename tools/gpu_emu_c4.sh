set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/range_emulate.py --config ${CFG:-c4} --worlds ${WORLDS:-8} > gpurun_out/emu.json 2> gpurun_out/emu.err || { tail -30 gpurun_out/emu.err; exit 1; }
grep '^{' gpurun_out/emu.json
