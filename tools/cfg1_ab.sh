#!/bin/bash
# cfg1_ab.sh — configs[1] (1M x 384, B = 256, k = 10) routing A/B: QS (default) vs QW from 129
# queries (HCRAG_QW_MIN=129), alternating, same box.
export TMPDIR=/tmp
C1="python bench.py --rows 1000000 --dim 384 --global-batch 256 --k 10 --steps 50 --warmup 5 --encoder none --no-cpu-baseline --no-configs0 --sweep ,"
for v in 0 129 0 129; do
  if [ $v = 0 ]; then timeout -k 10 200 $C1 > gpurun_out/c1_$v.log 2>&1 || exit 1
  else HCRAG_QW_MIN=$v timeout -k 10 200 $C1 > gpurun_out/c1_$v.log 2>&1 || exit 1; fi
  echo "qw_min $v $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*\|"score_kernel": [0-9]*' gpurun_out/c1_$v.log | tr '\n' ' ')" | tee -a gpurun_out/c1_ab.txt
done
echo ALLDONE
