# Submit one gpurun call; resubmit only while gpurun reports that no box ran it (a transient
# infrastructure status: slot busy, box lost while being prepared -- nothing charged), at most 12
# times, 2 minutes apart.  A call that ran (any exit status) is never resubmitted.
# Usage: bash tools/gpurun_retry.sh OUT.txt TIMEOUT 'command'
OUT=$1; TO=$2; CMD=$3
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$OUT" 2>&1
  if grep -q "status=transient" "$OUT" && grep -q "run 0.0s\|run Nones" "$OUT"; then
    # honour a back-off the service announces ("retry in Ns"), else wait 2 minutes
    w=$(grep -o "retry in [0-9]*s" "$OUT" | grep -o "[0-9]*" | tail -1)
    sleep $(( ${w:-110} + 10 ))
    continue
  fi
  break
done
