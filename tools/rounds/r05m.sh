#!/bin/bash
# r05m: QW appends take their slot from the wave's ballot (no LDS counter round trip) and the
# D = 384 stagger defaults to one accumulator set -- the GPU suite, then new vs lib/ab_old (HEAD
# 244c13b) in separate processes alternating, per shape.
export TMPDIR=/tmp
T=tools/gpu_step.sh
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
O="env HCRAG_LIB=hc-rag_amd/lib/ab_old/libhcrag_hip.so"
$T r05m_tests 600 $P tests -m gpu && \
for r in 1 2; do
  $T r05m_c1_new_$r 200 python tools/opt_ab.py 1000000 384 256 10 2 default QW_STAGGER=1 && \
  $T r05m_c1_old_$r 200 $O python tools/opt_ab.py 1000000 384 256 10 2 default && \
  $T r05m_w8_new_$r 200 python tools/opt_ab.py 1250000 768 1024 32 2 default && \
  $T r05m_w8_old_$r 200 $O python tools/opt_ab.py 1250000 768 1024 32 2 default || exit 1
done && \
$T r05m_c2_new 300 python tools/opt_ab.py 10000000 768 1024 32 2 default && \
$T r05m_c2_old 300 $O python tools/opt_ab.py 10000000 768 1024 32 2 default && \
$T r05m_b256_new 300 python tools/opt_ab.py 10000000 768 256 32 2 default && \
$T r05m_b256_old 300 $O python tools/opt_ab.py 10000000 768 256 32 2 default && \
echo ALLDONE_M
