#!/bin/bash
# r03_stride2.sh — the pre-pass stride again with the pre-pass on QW's MAXONLY form (cheaper than
# v4's): W = 8 / 4 rank shapes and the headline.
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T st2_w8 300 python tools/qw1_ab.py --shapes w8,w4 --rounds 3 --reps 7 --variants=-1:0:0,-1:0:16,-1:0:32,-1:0:64 && \
$T st2_c2 300 python tools/qw1_ab.py --shapes c2 --rounds 3 --reps 3 --variants=-1:0:0,-1:0:64,-1:0:256 && \
echo ALLDONE
