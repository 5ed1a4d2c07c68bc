#!/bin/bash
# r04x: QW stage shape at the W = 8 rank shape (1.25M x 768, B = 1024) and at the headline
export TMPDIR=/tmp
T=tools/gpu_step.sh
A="--no-cpu-baseline --encoder none --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --steps 30 --warmup 3"
$T r04x_w8 400 tools/ab_env.sh r04x_w8 2 HCRAG_QW_SR=32 X=0 $A --rows 1250000 && \
$T r04x_hl 500 tools/ab_env.sh r04x_hl 2 HCRAG_QW_SR=32 X=0 && \
echo ALLDONE_X
