#!/bin/bash
# 17-64 queries on 256 x 256 up to 1.5e9 corpus elements: GPU suite, sweeps vs forced 256 x 64
T=tools/gpu_step.sh
S1="python bench.py --rows 1000000 --dim 384 --batch 256 --k 10 --encoder none --no-cpu-baseline --steps 3 --sweep 17,20,32,48,64"
S2="python bench.py --rows 1500000 --dim 768 --batch 256 --encoder none --no-cpu-baseline --steps 3 --sweep 17,20,32,48,64"
$T gpu_tests 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread && \
$T s1_new 200 $S1 && $T s1_old 200 env HCRAG_Q64_ELEMS=0 $S1 && \
$T s2_new 200 $S2 && $T s2_old 200 env HCRAG_Q64_ELEMS=0 $S2 && \
$T bench 400 python bench.py
