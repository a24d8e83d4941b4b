# LDS and issue counters per kernel over one C3 bench step (tuning; summarised by
# tools/pmc_summary.py).  First lists the box's SQ counters into gpurun_out/pmc/counters.txt.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd $R
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmc/counters_all.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*" gpurun_out/pmc/counters_all.txt | sort -u > gpurun_out/pmc/counters.txt || true
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_LDS -d gpurun_out/pmc/lds -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc/lds.log 2>&1
