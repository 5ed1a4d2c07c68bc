#!/bin/bash
# r03_qs4.sh — after the QS4 default (129-256 queries at D <= 384) and the sample-stride rule:
# the full -m gpu suite, the configs[1] A/B of the new defaults against the r02/r03a ones, the
# QS stamps (wait / issue / epilogue split and the in-kernel clock) of both QS forms, and a
# kernel trace of the W = 8 rank shape (1.25M x 768, B = 1024: the fixed per-search kernels).
export TMPDIR=/tmp
T=tools/gpu_step.sh
S=hc-rag_amd/lib/stamps/libhcrag_hip.so
$T qs4_all_tests 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T qs4_ab_c1 300 python tools/qw1_ab.py --shapes c1 --rounds 3 --reps 7 --variants=-1:0:0:0,-1:0:64:1,-1:0:64:2,-1:0:16:1 && \
HCRAG_LIB=$S $T qs4_stamps_f1 120 python tools/qs_stamps.py 1000000 384 256 1 16 && \
HCRAG_LIB=$S $T qs4_stamps_f2 120 python tools/qs_stamps.py 1000000 384 256 2 16 && \
$T qs4_kt_w8 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_w8_r03 -o run -- python tools/qw1_ab.py --shapes w8 --rounds 1 --reps 10 --variants=-1 && \
echo ALLDONE
