#!/bin/bash
# r03_qw1c.sh — QW1 (incl. the 8-wave D = 384 form and the D = 768 tuning shapes) parity, the
# reference-data ingestion test, full-size configs[1]/[2] oracle checks; then the A/B.
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T r03c_tests 900 python -u -m pytest tests/test_qw1_gpu.py tests/test_ingest.py tests/test_exact_gpu.py tests/test_full_size_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T r03c_ab1 300 python -u tools/qw1_ab.py --shapes c1 --rounds 3 --variants 0,1,3,4 && \
$T r03c_ab2 400 python -u tools/qw1_ab.py --shapes c2 --rounds 2 --variants 0,2,2:1,2:2,2:3,1:2 && \
$T r03c_ab4 400 python -u tools/qw1_ab.py --shapes c4 --rounds 2 --variants 0,1,2 && \
HCRAG_LIB=hc-rag_amd/lib/stamps_qw1/libhcrag_hip.so $T r03c_st2 200 python -u tools/qw1_stamps.py 10000000 768 1024 2 0 && \
HCRAG_LIB=hc-rag_amd/lib/stamps_qw1/libhcrag_hip.so $T r03c_st1 200 python -u tools/qw1_stamps.py 10000000 768 1024 1 0 && \
HCRAG_LIB=hc-rag_amd/lib/stamps_qw1/libhcrag_hip.so $T r03c_st22 200 python -u tools/qw1_stamps.py 10000000 768 1024 2 2 && \
echo ALLDONE
