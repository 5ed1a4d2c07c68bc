#!/bin/bash
# r05e: the seed rank from k instead of k' (HCRAG_SEED_FROM_KP = the r04 rule), A/B per shape in
# separate processes (the hook is read once), alternating; widened / fallback counts printed.
export TMPDIR=/tmp
T=tools/gpu_step.sh
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
$T r05e_tests 600 $P tests/test_qw_gpu.py tests/test_search_gpu.py tests/test_exact_gpu.py -k "seed or qw_parity or planted or cert" && \
for r in 1 2; do
  $T r05e_c1_k_$r 200 python tools/opt_ab.py 1000000 384 256 10 2 default && \
  $T r05e_c1_kp_$r 200 env HCRAG_SEED_FROM_KP=1 python tools/opt_ab.py 1000000 384 256 10 2 default || exit 1
done && \
for r in 1 2; do
  $T r05e_w8_k_$r 200 python tools/opt_ab.py 1250000 768 1024 32 2 default && \
  $T r05e_w8_kp_$r 200 env HCRAG_SEED_FROM_KP=1 python tools/opt_ab.py 1250000 768 1024 32 2 default || exit 1
done && \
$T r05e_c2_k 300 python tools/opt_ab.py 10000000 768 1024 32 2 default && \
$T r05e_c2_kp 300 env HCRAG_SEED_FROM_KP=1 python tools/opt_ab.py 10000000 768 1024 32 2 default && \
echo ALLDONE_E
