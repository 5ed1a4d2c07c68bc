#!/bin/bash
# r05h: QW DM 5 (LDS-counter stage sync instead of the stage barrier): parity, stamps, interleaved
# A/B vs the defaults at configs[1], B = 256 and the headline.
export TMPDIR=/tmp
T=tools/gpu_step.sh
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
S="env HCRAG_LIB=hc-rag_amd/lib/stamps_qw/libhcrag_hip.so"
$T r05h_par5 300 env HCRAG_QW_DM=5 $P tests/test_qw_gpu.py -k "parity or small_corpus or duplicate or cold" && \
$T r05h_st5_c1 200 $S python tools/qw_stamps.py 1000000 384 256 10 QW_DM=5 && \
$T r05h_st5_c2 200 $S python tools/qw_stamps.py 10000000 768 1024 32 QW_DM=5 && \
$T r05h_ab_c1 300 python tools/opt_ab.py 1000000 384 256 10 3 default QW_DM=5 && \
$T r05h_ab_b256 300 python tools/opt_ab.py 10000000 768 256 32 3 default QW_DM=5 && \
$T r05h_ab_c2 300 python tools/opt_ab.py 10000000 768 1024 32 2 default QW_DM=5 && \
echo ALLDONE_H
