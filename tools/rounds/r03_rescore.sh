#!/bin/bash
# r03_rescore.sh — K4 with both 512-dim row halves gathered together: the full -m gpu suite, a
# kernel trace of the W = 8 rank shape (K4 at B = 1024, D = 768), and the configs[1] stride A/B at
# the 128-deep QS stages.
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T rs_tests 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T rs_kt_w8 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_w8_rs -o run -- python tools/qw1_ab.py --shapes w8 --rounds 1 --reps 10 --variants=-1 && \
$T rs_ab_c1 300 python tools/qw1_ab.py --shapes c1 --rounds 4 --reps 7 --variants=-1:0:0:0,-1:0:32:0,-1:0:8:0 && \
echo ALLDONE
