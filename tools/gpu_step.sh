#!/bin/bash
# gpu_step.sh NAME SECONDS CMD... — run one GPU step under its own time limit, log to
# gpurun_out/NAME.log and propagate its status: 0 ok (pytest "no tests collected" counts as ok),
# 1 test failures, 99 when the step ended in a way that may have left the GPU faulted (abort 134,
# segfault 139, time limit 124/137, a harness-reported HIP error 2) -- chain steps with && so
# nothing runs on the GPU after a failed or faulted step.
name=$1; secs=$2; shift 2
mkdir -p gpurun_out
echo "[$(date -u +%T)] start $name" >> gpurun_out/steps.log
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "[$(date -u +%T)] end $name rc=$rc" >> gpurun_out/steps.log
tail -3 "gpurun_out/$name.log"
case $rc in
  0|5) exit 0 ;;
  1) echo "FAILED $name (rc=1)"; exit 1 ;;
  *) echo "STOP after $name rc=$rc"; exit 99 ;;
esac
