#!/bin/bash
# r03_fixed.sh — after the wave-level seed selection and small sorts and the 128-deep QS stages
# at D = 384: the full -m gpu suite, kernel traces of configs[1] and of the W = 8 rank shape (the
# fixed per-search kernels: prep, pre-pass, seed, merge / finish, rescore), the configs[1] A/B of
# the QS stage depth.
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T fx_tests 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T fx_kt_c1 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_c1_fx -o run -- python tools/qw1_ab.py --shapes c1 --rounds 1 --reps 20 --variants=-1 && \
$T fx_kt_w8 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_w8_fx -o run -- python tools/qw1_ab.py --shapes w8 --rounds 1 --reps 10 --variants=-1 && \
$T fx_ab_c1 300 python tools/qw1_ab.py --shapes c1 --rounds 4 --reps 7 --variants=-1:0:0:0,-1:0:0:1 && \
echo ALLDONE
