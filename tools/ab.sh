# A/B on one box: bench with and without an environment setting (tuning only)
# usage: bash tools/ab.sh NAME[=VALUE] [steps]     (VALUE defaults to 1)
A=$1; S=${2:-5}
V=${A%%=*}; X=1; [ "$A" != "$V" ] && X=${A#*=}
mkdir -p gpurun_out
for mode in B A B A; do
  if [ $mode = A ]; then export $V="$X"; else unset $V; fi
  timeout -k 10 300 python bench.py --steps $S --warmup 1 --no-cpu-baseline > gpurun_out/ab_$mode.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_$mode.log').read().strip().splitlines()[-1]); s=d['config']['stages_ms_per_step']; print('$mode', '$A' if '$mode'=='A' else 'default', d['ms_per_step'], {k: s[k] for k in sorted(s) if s[k] > 1})"
done
