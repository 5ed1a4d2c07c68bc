#!/bin/bash
# r05ms: the merge's wave-scan of the list counts + v4's MAXONLY pre-pass for one query block --
# the GPU suite, then new vs lib/ab_old (HEAD) alternating: configs[1] and the headline.
export TMPDIR=/tmp
T=tools/gpu_step.sh
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
O="env HCRAG_LIB=hc-rag_amd/lib/ab_old/libhcrag_hip.so"
$T r05ms_tests 700 $P tests -m gpu && \
for r in 1 2 3; do
  $T r05ms_c1_new_$r 200 python tools/opt_ab.py 1000000 384 256 10 2 default && \
  $T r05ms_c1_old_$r 200 $O python tools/opt_ab.py 1000000 384 256 10 2 default || exit 1
done && \
$T r05ms_c2_new 300 python tools/opt_ab.py 10000000 768 1024 32 2 default && \
$T r05ms_c2_old 300 $O python tools/opt_ab.py 10000000 768 1024 32 2 default && \
echo ALLDONE_MS
