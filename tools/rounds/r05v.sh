#!/bin/bash
# r05v: the fused merge + rescore kernel (finish_kernel, RU = 16 and side-by-side wave sums since
# r05t) at 1024 queries (HCRAG_FINISH_MAX=1024) vs the separate launches, alternating processes:
# W = 8 rank shape and the headline.
export TMPDIR=/tmp
T=tools/gpu_step.sh
N="env HCRAG_FINISH_MAX=1024"
for r in 1 2; do
  $T r05v_w8_fin_$r 200 $N python tools/opt_ab.py 1250000 768 1024 32 2 default && \
  $T r05v_w8_sep_$r 200 python tools/opt_ab.py 1250000 768 1024 32 2 default || exit 1
done && \
$T r05v_c2_fin 300 $N python tools/opt_ab.py 10000000 768 1024 32 2 default && \
$T r05v_c2_sep 300 python tools/opt_ab.py 10000000 768 1024 32 2 default && \
echo ALLDONE_V
