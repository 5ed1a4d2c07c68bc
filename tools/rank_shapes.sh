#!/bin/bash
# rank_shapes.sh — the strong-scaling bench's per-rank work on one GPU: 10M/W rows x the full
# 1024-query global batch (W = 2, 4, 8), plus a kernel trace of the W = 8 shape.
export TMPDIR=/tmp
T=tools/gpu_step.sh
B="python bench.py --encoder none --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --sweep , --steps 30 --warmup 3"
$T rs_w2 300 $B --rows 5000000 && \
$T rs_w4 300 $B --rows 2500000 && \
$T rs_w8 300 $B --rows 1250000 && \
$T rs_w8_kt 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rs_w8_kt -o run -- $B --rows 1250000 && echo ALLDONE
