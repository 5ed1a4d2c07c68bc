#!/bin/bash
# r03_qw1.sh — QW1 parity tests, then the in-process QW / QW1 / v4 A/B (tools/qw1_ab.py).
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T r03a_qw1_tests 600 python -u -m pytest tests/test_qw1_gpu.py tests/test_qw_gpu.py tests/test_exact_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider && \
$T r03a_qw1_ab 600 python -u tools/qw1_ab.py --shapes c1,c2,c4 --rounds 3 && \
echo ALLDONE
