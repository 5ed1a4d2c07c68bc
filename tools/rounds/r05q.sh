#!/bin/bash
# r05q: final lists gathered across a wave's queries (final_lists_wave) in QW / QW1 / QS -- the
# GPU suite, the stamps time line at configs[1] / W = 8, then new vs lib/ab_old (HEAD a401b18)
# in separate processes alternating.
export TMPDIR=/tmp
T=tools/gpu_step.sh
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
S="env HCRAG_LIB=hc-rag_amd/lib/stamps_qw/libhcrag_hip.so"
O="env HCRAG_LIB=hc-rag_amd/lib/ab_old/libhcrag_hip.so"
$T r05q_tests 600 $P tests -m gpu && \
$T r05q_st_c1 200 $S python tools/qw_stamps.py 1000000 384 256 10 && \
$T r05q_st_w8 200 $S python tools/qw_stamps.py 1250000 768 1024 32 && \
for r in 1 2; do
  $T r05q_c1_new_$r 200 python tools/opt_ab.py 1000000 384 256 10 2 default && \
  $T r05q_c1_old_$r 200 $O python tools/opt_ab.py 1000000 384 256 10 2 default && \
  $T r05q_w8_new_$r 200 python tools/opt_ab.py 1250000 768 1024 32 2 default && \
  $T r05q_w8_old_$r 200 $O python tools/opt_ab.py 1250000 768 1024 32 2 default && \
  $T r05q_b64_new_$r 200 python tools/opt_ab.py 1000000 768 64 32 2 default && \
  $T r05q_b64_old_$r 200 $O python tools/opt_ab.py 1000000 768 64 32 2 default || exit 1
done && \
echo ALLDONE_Q
