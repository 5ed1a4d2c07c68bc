#!/bin/bash
# r04h: QW's stage shape at B = 256 on 10M x 768 (48-row 2-deep ring vs 32-row 3-deep: one
# query block per partition streams every row tile from HBM once), and configs[1] on QS vs QW.
export TMPDIR=/tmp
T=tools/gpu_step.sh
B256="--no-cpu-baseline --encoder none --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --steps 20 --warmup 3 --global-batch 256"
$T r04h_b256 500 tools/ab_env.sh r04h_b256 2 HCRAG_QW_SR=32 X=0 $B256 && \
$T r04h_c1 300 tools/ab_c1.sh r04h_c1 2 X=0 HCRAG_QW_MIN=129 && \
echo ALLDONE_H
