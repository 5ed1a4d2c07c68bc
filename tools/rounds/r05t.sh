#!/bin/bash
# r05t: the rescore's wave sums side by side + lane-parallel candidate finish (and RU = 16 in
# finish_kernel) -- tests, finish stamps at configs[1], new vs lib/ab_old (HEAD 73f2b8f).
export TMPDIR=/tmp
T=tools/gpu_step.sh
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
F="env HCRAG_LIB=hc-rag_amd/lib/stamps_fin/libhcrag_hip.so"
O="env HCRAG_LIB=hc-rag_amd/lib/ab_old/libhcrag_hip.so"
$T r05t_tests 500 $P tests/test_search_gpu.py tests/test_exact_gpu.py tests/test_full_size_gpu.py tests/test_configs0_gpu.py && \
$T r05t_fs_c1 200 $F python tools/finish_stamps.py 1000000 384 256 10 && \
for r in 1 2; do
  $T r05t_c1_new_$r 200 python tools/opt_ab.py 1000000 384 256 10 2 default && \
  $T r05t_c1_old_$r 200 $O python tools/opt_ab.py 1000000 384 256 10 2 default && \
  $T r05t_w8_new_$r 200 python tools/opt_ab.py 1250000 768 1024 32 2 default && \
  $T r05t_w8_old_$r 200 $O python tools/opt_ab.py 1250000 768 1024 32 2 default || exit 1
done && \
echo ALLDONE_T
