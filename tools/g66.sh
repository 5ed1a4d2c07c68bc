#!/bin/bash
# 33-64 queries: 256 x 64 (HCRAG_Q64_ROWS=0) vs 256 x 256 (HCRAG_Q64_ROWS=huge) by corpus size
T=tools/gpu_step.sh
for R in 1000000 2500000 5000000 10000000; do
  for Q in 0 1000000000000; do
    $T q64_${R}_${Q} 200 env HCRAG_Q64_ROWS=$Q python bench.py --rows $R --batch 256 --encoder none --no-cpu-baseline --steps 3 --sweep 33,48,64 || exit 1
  done
done
$T sw1 200 python bench.py --rows 1000000 --dim 384 --batch 256 --k 10 --encoder none --no-cpu-baseline --steps 3 --sweep 33,48,64 && \
$T sw1_narrow 200 env HCRAG_Q64_ROWS=0 python bench.py --rows 1000000 --dim 384 --batch 256 --k 10 --encoder none --no-cpu-baseline --steps 3 --sweep 33,48,64 && \
$T tests 400 python -u -m pytest tests/test_search_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "batch_sizes or rank_shapes or random_parity"
