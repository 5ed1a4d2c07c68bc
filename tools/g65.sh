#!/bin/bash
# 65-128 queries on 256 x 256: GPU suite, sweeps vs HCRAG_QT128=1 (old 256 x 128), default bench
T=tools/gpu_step.sh
S10="python bench.py --encoder none --no-cpu-baseline --steps 5 --sweep 64,65,80,100,128,129,200"
S1="python bench.py --rows 1000000 --dim 384 --batch 256 --k 10 --encoder none --no-cpu-baseline --steps 10 --sweep 64,65,80,100,128,129,200"
$T gpu_tests 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread && \
$T sw10_new 300 $S10 && \
$T sw10_old 300 env HCRAG_QT128=1 $S10 && \
$T sw1_new 300 $S1 && \
$T sw1_old 300 env HCRAG_QT128=1 $S1 && \
$T bench 400 python bench.py
