# One GPU lease, parameterised (replaces the round-4 one-off gpu_r4_*.sh scripts).  Everything goes
# under gpurun_out/; each GPU step has its own time limit and the script stops at the first failure.
#   bash tools/gpu_run.sh TASK...
#     tests[=K_EXPR]      the GPU test suite (pytest -m gpu), optionally -k K_EXPR
#     smoke               __graft_entry__.smoke()
#     bench=CFG[:TAG]     one unprofiled bench line, 20 steps after 5 warm-up -> bench_TAG.json
#     prof=CFG[:TAG]      the same-lease roofline protocol -> prof_TAG/: rocm-smi before, the
#                         unprofiled bench, the SAME command under rocprofv3 --kernel-trace --stats,
#                         --pmc passes (SQ mix, FETCH_SIZE, WRITE_SIZE: one pass each), rocm-smi after,
#                         and tools/trace_summary.py (steady-state kernel times vs the bench's stages)
#     ab=CFG              interleaved A/B over $LIBS ("abl/x.so intree env:VAR=1 opt:GKM_X=1 ..."), $REPS rounds
#     emu=CFG             tools/range_emulate.py (multi-GPU per-rank emulation) -> emu_CFG.json
#     cmd=SHELL           any other command (its own 600 s limit)
set -o pipefail
mkdir -p gpurun_out
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
export TMPDIR=/tmp
STEPS=${STEPS:-20}
WARM=${WARMUP:-5}
smi() { rocm-smi --showclocks --showpower --showtemp --showuse > "$1" 2>&1 || true; }
die() { echo "FAILED: $*"; exit 1; }
for task in "$@"; do
  name=${task%%=*}
  arg=${task#*=}
  [ "$arg" = "$task" ] && arg=""
  echo "== $task ($(date +%T))"
  case "$name" in
    tests)
      K=()
      [ -n "$arg" ] && K=(-k "$arg")
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${K[@]}" \
        > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; die tests; }
      tail -2 gpurun_out/gpu_tests.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
        || { tail -20 gpurun_out/smoke.log; die smoke; }
      tail -1 gpurun_out/smoke.log ;;
    bench)
      cfg=${arg%%:*}; tag=${arg#*:}; [ "$tag" = "$arg" ] && tag=$cfg
      timeout -k 10 600 python -u bench.py --config "$cfg" --steps "$STEPS" --warmup "$WARM" ${BENCH_ARGS:-} \
        > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { tail -20 gpurun_out/bench_$tag.err; die bench; }
      python3 tools/line_brief.py gpurun_out/bench_$tag.json ;;
    prof)
      cfg=${arg%%:*}; tag=${arg#*:}; [ "$tag" = "$arg" ] && tag=$cfg
      O=gpurun_out/prof_$tag
      mkdir -p $O
      B=(bench.py --config "$cfg" --steps "$STEPS" --warmup "$WARM" --no-cpu-baseline)
      smi $O/smi_before.txt
      timeout -k 10 600 python -u "${B[@]}" > $O/bench_unprofiled.json 2> $O/bench_unprofiled.err \
        || { tail -20 $O/bench_unprofiled.err; die prof-bench; }
      python3 tools/line_brief.py $O/bench_unprofiled.json
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 "${B[@]}" \
        > $O/bench_profiled.json 2> $O/bench_profiled.err || { tail -20 $O/bench_profiled.err; die prof-trace; }
      smi $O/smi_after_trace.txt
      cp "$(find $O/trace -name '*kernel_stats.csv' | head -1)" $O/kernel_stats.csv
      python3 tools/trace_summary.py "$(find $O/trace -name '*kernel_trace.csv' | head -1)" $O/bench_unprofiled.json \
        $O/trace_summary.json --warmup "$WARM" --steps "$STEPS" | tee $O/trace_summary.txt
      P=(bench.py --config "$cfg" --steps 2 --warmup 1 --no-cpu-baseline --no-boundary)
      timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM \
        SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $O/sq -o run --output-format csv -- python3 "${P[@]}" \
        > $O/sq.log 2>&1 || { tail -20 $O/sq.log; die prof-sq; }
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 "${P[@]}" \
        > $O/fetch.log 2>&1 || { tail -20 $O/fetch.log; die prof-fetch; }
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 "${P[@]}" \
        > $O/write.log 2>&1 || { tail -20 $O/write.log; die prof-write; }
      smi $O/smi_after.txt
      python3 tools/pmc_summary.py "$(find $O/sq -name '*counter_collection.csv' | head -1)" > $O/pmc_sq_summary.txt
      python3 tools/pmc_traffic.py "$(find $O/fetch -name '*counter_collection.csv' | head -1)" \
        "$(find $O/write -name '*counter_collection.csv' | head -1)" $O/traffic.json --label "$cfg $tag" > $O/traffic.txt
      rm -rf $O/trace/*/*/*counter* $O/sq $O/fetch $O/write
      find $O/trace -name '*.csv' ! -name '*kernel_stats.csv' ! -name '*kernel_trace.csv' -delete
      head -12 $O/traffic.txt ;;
    ab)
      for rep in $(seq 1 ${REPS:-2}); do
        for lib in ${LIBS}; do
          unset GKM_LIB
          envs=(); extra=()
          case "$lib" in
            intree) ;;
            env:*) envs=("${lib#env:}") ;;
            opt:*) envs=(GKM_AB_OPT=1); extra=(--opt "${lib#opt:}") ;;
            *) export GKM_LIB=$lib ;;
          esac
          timeout -k 10 300 env "${envs[@]}" python bench.py --config "$arg" --steps ${AB_STEPS:-5} --warmup 1 \
            --no-cpu-baseline --no-boundary "${extra[@]}" > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; die ab; }
          python3 tools/line_brief.py gpurun_out/ab.json --label "$lib" | tee -a gpurun_out/ab_$arg.txt
        done
      done ;;
    emu)
      timeout -k 10 900 python -u tools/range_emulate.py --config "$arg" ${EMU_ARGS:-} > gpurun_out/emu_$arg.json \
        2> gpurun_out/emu_$arg.err || { tail -20 gpurun_out/emu_$arg.err; die emu; }
      tail -5 gpurun_out/emu_$arg.err ;;
    cmd)
      timeout -k 10 600 bash -c "$arg" || die "cmd $arg" ;;
    *) die "unknown task $task" ;;
  esac
done
echo "== done ($(date +%T))"
