#!/bin/bash
# cfg1_stride.sh — configs[1] with the pre-pass stride 64 vs 128 (default), alternating.
export TMPDIR=/tmp
C1="python bench.py --rows 1000000 --dim 384 --global-batch 256 --k 10 --steps 50 --warmup 5 --encoder none --no-cpu-baseline --no-configs0 --sweep ,"
for v in 64 128 64 128; do
  HCRAG_SAMPLE_STRIDE=$v timeout -k 10 200 $C1 > gpurun_out/c1s_$v.log 2>&1 || exit 1
  echo "stride $v $(grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*' gpurun_out/c1s_$v.log | tr '\n' ' ')" | tee -a gpurun_out/c1_stride.txt
done
echo ALLDONE
