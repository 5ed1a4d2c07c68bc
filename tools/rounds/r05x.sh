#!/bin/bash
# r05x: the global seed with the sample call's prep reused and no local seed in it -- its tests,
# the search / exact tests, the W = 8 per-rank emulation (3 rounds).
export TMPDIR=/tmp
T=tools/gpu_step.sh
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
$T r05x_tests 500 $P tests/test_global_seed_gpu.py tests/test_search_gpu.py tests/test_qw_gpu.py && \
$T r05x_rank8 400 python -u tools/global_seed_rank.py 10000000 768 1024 32 8 3 && \
echo ALLDONE_X
