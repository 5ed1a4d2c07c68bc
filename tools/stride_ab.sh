#!/bin/bash
# stride_ab.sh — MAXONLY pre-pass sampling stride A/B on the headline (64 = default, 128, 256).
export TMPDIR=/tmp
B="python bench.py --encoder none --no-cpu-baseline --no-configs0 --sweep , --steps 30 --warmup 3"
for v in 64 128 256 64; do
  HCRAG_SAMPLE_STRIDE=$v timeout -k 10 240 $B > gpurun_out/stride_$v.log 2>&1 || exit 1
  echo "stride $v $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*\|"widened_queries": [0-9]*\|"fallback_queries": [0-9]*' gpurun_out/stride_$v.log | tr '\n' ' ')" | tee -a gpurun_out/stride_ab.txt
done
echo ALLDONE
