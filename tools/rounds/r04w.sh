#!/bin/bash
# r04w: the strong-scaling bench's per-rank work on one GPU at HEAD (10M / W rows x the full
# 1024-query batch, W = 2 / 4 / 8) and the W = 8 kernel trace; also configs[3]'s rank shape
# (1.25M rows x 4096 queries).
export TMPDIR=/tmp
T=tools/gpu_step.sh
B="python bench.py --encoder none --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --steps 30 --warmup 3"
$T r04w_w2 200 $B --rows 5000000 && \
$T r04w_w4 200 $B --rows 2500000 && \
$T r04w_w8 200 $B --rows 1250000 && \
$T r04w_c3 200 $B --rows 1250000 --global-batch 4096 && \
$T r04w_w8_kt 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04w_w8_kt -o run -- $B --rows 1250000 && \
echo ALLDONE_W
