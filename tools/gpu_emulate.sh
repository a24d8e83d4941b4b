# Multi-GPU per-rank emulation on one GPU (tools/range_emulate.py): both schemes for C3, the
# key-range scheme for C4 -> gpurun_out/emulate_*.json
set -o pipefail
mkdir -p gpurun_out
for spec in ${SPECS:-c3:range c3:a2a c4:range}; do
  cfg=${spec%%:*}; sch=${spec##*:}
  timeout -k 10 400 python -u tools/range_emulate.py --config $cfg --scheme $sch --worlds ${WORLDS:-8,4,2} > gpurun_out/emulate_${cfg}_${sch}.json 2> gpurun_out/emulate_${cfg}_${sch}.err || { tail -20 gpurun_out/emulate_${cfg}_${sch}.err; exit 1; }
  cat gpurun_out/emulate_${cfg}_${sch}.json
done
