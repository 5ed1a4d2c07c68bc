#!/bin/bash
# Rank shapes of the W-GPU scaling bench, simulated on one GPU: the per-rank local search
# (rows N/W, nq = W*1024) parity test, then bench.py at those shapes (no collectives at W=1)
T=tools/gpu_step.sh
$T rank_tests 400 python -u -m pytest tests/test_search_gpu.py -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k rank_shapes && \
$T shape2 300 python bench.py --rows 5000000 --batch 2048 --encoder none --no-cpu-baseline --steps 10 && \
$T shape4 300 python bench.py --rows 2500000 --batch 4096 --encoder none --no-cpu-baseline --steps 10 && \
$T shape8 300 python bench.py --rows 1250000 --batch 8192 --encoder none --no-cpu-baseline --steps 10
