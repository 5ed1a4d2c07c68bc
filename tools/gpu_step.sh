#!/bin/bash
# gpu_step.sh NAME SECONDS CMD... — run one GPU step under its own time limit, log to
# gpurun_out/NAME.log, and stop the whole call (exit 99) when the step ended in a way that
# may have left the GPU faulted: abort (134), segfault (139), time limit (124/137), or a
# HIP error reported by a harness (rc 2).  Ordinary test failures (pytest rc 1) continue.
name=$1; secs=$2; shift 2
mkdir -p gpurun_out
echo "[$(date -u +%T)] start $name" >> gpurun_out/steps.log
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "[$(date -u +%T)] end $name rc=$rc" >> gpurun_out/steps.log
tail -3 "gpurun_out/$name.log"
case $rc in
  0|1) exit 0 ;;
  5) exit 0 ;;            # pytest: no tests collected
  *) echo "STOP after $name rc=$rc"; exit 99 ;;
esac
