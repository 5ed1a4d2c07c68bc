#!/bin/bash
# r05j: sampling pre-pass stride and kernel under the r05 seed rule (lambda from k), per shape,
# interleaved in one process.
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T r05j_c1 300 python tools/opt_ab.py 1000000 384 256 10 3 default SAMPLE_STRIDE=8 SAMPLE_STRIDE=32 PREPASS=1 PREPASS=1,SAMPLE_STRIDE=32 && \
$T r05j_w8 300 python tools/opt_ab.py 1250000 768 1024 32 3 default SAMPLE_STRIDE=16 SAMPLE_STRIDE=64 SAMPLE_STRIDE=128 && \
$T r05j_c2 400 python tools/opt_ab.py 10000000 768 1024 32 2 default SAMPLE_STRIDE=64 SAMPLE_STRIDE=256 && \
echo ALLDONE_J
