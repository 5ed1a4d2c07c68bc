#!/bin/bash
# r03_prepass.sh — the sampling pre-pass on QW's MAXONLY form: the full -m gpu suite, the A/B of
# the pre-pass kernel (HCR_OPT_PREPASS 1 = v4, 2 = QW) at the W = 8 rank shape and the headline,
# and a kernel trace of the W = 8 rank shape.
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T pp_tests 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T pp_ab_w8 300 python tools/qw1_ab.py --shapes w8,w4 --rounds 3 --reps 7 --variants=-1:0:0:0:1,-1:0:0:0:2 && \
$T pp_ab_c2 300 python tools/qw1_ab.py --shapes c2 --rounds 3 --reps 3 --variants=-1:0:0:0:1,-1:0:0:0:2 && \
$T pp_kt_w8 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_w8_pp -o run -- python tools/qw1_ab.py --shapes w8 --rounds 1 --reps 10 --variants=-1 && \
echo ALLDONE
