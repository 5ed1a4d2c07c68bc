#!/bin/bash
# r05s: finish_kernel rescoring 16 candidates per wave per round (one row-gather round at k' = 64)
# -- tests, the finish stamps at configs[1], then new vs lib/ab_old (HEAD 73f2b8f) alternating.
export TMPDIR=/tmp
T=tools/gpu_step.sh
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
F="env HCRAG_LIB=hc-rag_amd/lib/stamps_fin/libhcrag_hip.so"
O="env HCRAG_LIB=hc-rag_amd/lib/ab_old/libhcrag_hip.so"
$T r05s_tests 500 $P tests/test_search_gpu.py tests/test_exact_gpu.py tests/test_full_size_gpu.py && \
$T r05s_fs_c1 200 $F python tools/finish_stamps.py 1000000 384 256 10 && \
for r in 1 2; do
  $T r05s_c1_new_$r 200 python tools/opt_ab.py 1000000 384 256 10 2 default && \
  $T r05s_c1_old_$r 200 $O python tools/opt_ab.py 1000000 384 256 10 2 default && \
  $T r05s_b512_new_$r 200 python tools/opt_ab.py 1000000 768 512 32 2 default && \
  $T r05s_b512_old_$r 200 $O python tools/opt_ab.py 1000000 768 512 32 2 default || exit 1
done && \
echo ALLDONE_S
