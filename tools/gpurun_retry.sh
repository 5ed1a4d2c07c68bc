#!/bin/bash
# gpurun_retry.sh OUT SCRIPT [TIMEOUT] -- submit `bash SCRIPT` through gpurun, re-submitting only
# when the pool had no slot / box free (nothing ran, nothing charged); never after a run.
out=$1; script=$2; lim=${3:-1200}
for i in 1 2 3 4 5 6 7 8; do
  timeout $((lim + 900)) /usr/local/graft/bin/gpurun --timeout "$lim" -- bash "$script" > "$out" 2>&1
  # (also "stopped responding while being prepared": the box failed before the command started)
  if grep -q "slot(s) on this pod are busy\|has no free box right now\|stopped responding while being prepared" "$out" && ! grep -q "status=ok" "$out"; then
    sleep 150
    continue
  fi
  break
done
tail -3 "$out"
