#!/bin/bash
# r05a: the bounds-checked candidate gather (planted out-of-range key -> HCR_EINTERNAL), the QW
# kernel without the r03 stage-test hook, and where a dense QW stage goes (stamps build) at the
# headline and at the W = 8 rank shape.
export TMPDIR=/tmp
T=tools/gpu_step.sh
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
$T r05a_tests 900 $P tests/test_exact_gpu.py tests/test_qw_gpu.py tests/test_search_gpu.py && \
$T r05a_stamps_c2 300 env HCRAG_LIB=hc-rag_amd/lib/stamps_qw/libhcrag_hip.so python tools/qw_stamps.py 10000000 768 1024 && \
$T r05a_stamps_w8 300 env HCRAG_LIB=hc-rag_amd/lib/stamps_qw/libhcrag_hip.so python tools/qw_stamps.py 1250000 768 1024 && \
echo ALLDONE_A
