#!/bin/bash
# r03_qw1d.sh — QW1 / QW1P parity (v_max3 epilogue, the pipelined form), A/B of the large-batch
# kernels on configs[1] / [2] / [4] shapes, QW1 stamps with the new epilogue, then the default
# bench (its new configs[1], configs[4] and query-pipeline legs).
export TMPDIR=/tmp
T=tools/gpu_step.sh
S=hc-rag_amd/lib/stamps_qw1/libhcrag_hip.so
$T r03d_tests 700 python -u -m pytest tests/test_qw1_gpu.py tests/test_finish_gpu.py tests/test_qw_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T r03d_ab2 400 python -u tools/qw1_ab.py --shapes c2 --rounds 2 --variants 0,1,2:2,5 && \
$T r03d_ab4 400 python -u tools/qw1_ab.py --shapes c4 --rounds 2 --variants 1,5 && \
$T r03d_ab1 300 python -u tools/qw1_ab.py --shapes c1 --rounds 3 --variants 0,1,3,5 && \
HCRAG_LIB=$S $T r03d_st1 200 python -u tools/qw1_stamps.py 10000000 768 1024 1 0 && \
$T r03d_bench 600 python -u bench.py && \
echo ALLDONE
