#!/bin/bash
# qw_fd_ab.sh — QW fragment prefetch depth A/B: the default library (FD = 3) vs a build with
# FD = 2 (hc-rag_amd/lib/ab/libhcrag_fd2.so via HCRAG_LIB), alternating on one box.
export TMPDIR=/tmp
B="python bench.py --encoder none --no-cpu-baseline --no-configs0 --sweep , --steps 30 --warmup 3"
for v in 3 2 3 2; do
  if [ $v = 3 ]; then timeout -k 10 240 $B > gpurun_out/fd_$v.log 2>&1 || exit 1
  else HCRAG_LIB=$PWD/hc-rag_amd/lib/ab/libhcrag_fd2.so timeout -k 10 240 $B > gpurun_out/fd_$v.log 2>&1 || exit 1; fi
  echo "FD $v $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*' gpurun_out/fd_$v.log | tr '\n' ' ')" | tee -a gpurun_out/fd_ab.txt
done
echo ALLDONE
