#!/bin/bash
# padded query columns bounded at +inf: GPU suite, then 10M x 768 and 1M x 384 batch sweeps
# with and without (HCRAG_NO_PAD_BOUND=1) in one call
T=tools/gpu_step.sh
S10="python bench.py --encoder none --no-cpu-baseline --steps 5 --sweep 1,8,16,32,48,64,100,128,200,256,512"
S1="python bench.py --rows 1000000 --dim 384 --batch 256 --k 10 --encoder none --no-cpu-baseline --steps 10 --sweep 1,8,16,32,48,64,100,128,200,256"
$T gpu_tests 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread && \
$T sw10_new 300 $S10 && \
$T sw10_old 300 env HCRAG_NO_PAD_BOUND=1 $S10 && \
$T sw1_new 300 $S1 && \
$T sw1_old 300 env HCRAG_NO_PAD_BOUND=1 $S1
