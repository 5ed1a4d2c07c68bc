#!/bin/bash
# r03_seed.sh — QS4 parity tests, then A/B in one process per shape of the sampling pre-pass
# stride (HCR_OPT_SAMPLE_STRIDE) and the QS form (HCR_OPT_QS_FORM: 8-wave vs QS4) on configs[1]
# (1M x 384, B = 256), the W = 8 / W = 4 rank shapes of the strong-scaling bench (1.25M / 2.5M
# x 768, B = 1024) and the headline (10M x 768, B = 1024).
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T qs4_tests 400 python -u -m pytest tests/test_qs4_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider && \
$T seed_c1 300 python tools/qw1_ab.py --shapes c1 --rounds 3 --reps 7 --variants=-1:0:0:0,-1:0:0:2,-1:0:32:0,-1:0:32:2,-1:0:16:2 && \
$T seed_w8 300 python tools/qw1_ab.py --shapes w8,w4 --rounds 3 --reps 5 --variants=-1:0:0,-1:0:32,-1:0:16,-1:0:8 && \
$T seed_c2 300 python tools/qw1_ab.py --shapes c2 --rounds 2 --reps 3 --variants=-1:0:0,-1:0:64,-1:0:32 && \
echo ALLDONE
