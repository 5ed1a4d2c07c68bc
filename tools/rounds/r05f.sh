#!/bin/bash
# r05f: the QW stage wait counting the epilogue's append stores (score_qw.h nst) vs the fixed
# count (lib/ab_old = r05e HEAD), separate processes alternating, per shape; QW tests.
export TMPDIR=/tmp
T=tools/gpu_step.sh
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
O="env HCRAG_LIB=hc-rag_amd/lib/ab_old/libhcrag_hip.so"
$T r05f_tests 600 $P tests/test_qw_gpu.py && \
for r in 1 2; do
  $T r05f_c1_new_$r 200 python tools/opt_ab.py 1000000 384 256 10 2 default && \
  $T r05f_c1_old_$r 200 $O python tools/opt_ab.py 1000000 384 256 10 2 default && \
  $T r05f_w8_new_$r 200 python tools/opt_ab.py 1250000 768 1024 32 2 default && \
  $T r05f_w8_old_$r 200 $O python tools/opt_ab.py 1250000 768 1024 32 2 default || exit 1
done && \
$T r05f_c2_new 300 python tools/opt_ab.py 10000000 768 1024 32 2 default QW_DM=3 && \
$T r05f_c2_old 300 $O python tools/opt_ab.py 10000000 768 1024 32 2 default QW_DM=3 && \
$T r05f_b256_new 300 python tools/opt_ab.py 10000000 768 256 32 2 default && \
$T r05f_b256_old 300 $O python tools/opt_ab.py 10000000 768 256 32 2 default && \
echo ALLDONE_F
