#!/bin/bash
# r05n: QW1 (D = 1024) appends from the wave ballot -- its tests, then new vs lib/ab_old (HEAD
# 244c13b) at 2M x 1024, B = 1024, k = 64, separate processes alternating.
export TMPDIR=/tmp
T=tools/gpu_step.sh
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
O="env HCRAG_LIB=hc-rag_amd/lib/ab_old/libhcrag_hip.so"
$T r05n_tests 400 $P tests/test_qw1_gpu.py tests/test_qw_gpu.py && \
for r in 1 2; do
  $T r05n_d1024_new_$r 200 python tools/opt_ab.py 2000000 1024 1024 64 2 default && \
  $T r05n_d1024_old_$r 200 $O python tools/opt_ab.py 2000000 1024 1024 64 2 default || exit 1
done && \
echo ALLDONE_N
