#!/bin/bash
# r03_qs_hs.sh — QS forms parity (QS4, 128- / 192-deep stages), the configs[1] A/B of the forms
# at the stride-rule default, and stamps of the deep-stage forms.
export TMPDIR=/tmp
T=tools/gpu_step.sh
S=hc-rag_amd/lib/stamps/libhcrag_hip.so
$T qshs_tests 400 python -u -m pytest tests/test_qs4_gpu.py tests/test_full_size_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider && \
$T qshs_ab_c1 300 python tools/qw1_ab.py --shapes c1 --rounds 4 --reps 7 --variants=-1:0:0:0,-1:0:0:3,-1:0:0:4,-1:0:0:2 && \
HCRAG_LIB=$S $T qshs_stamps_f3 120 python tools/qs_stamps.py 1000000 384 256 3 16 && \
HCRAG_LIB=$S $T qshs_stamps_f4 120 python tools/qs_stamps.py 1000000 384 256 4 16 && \
echo ALLDONE
