#!/bin/bash
# r05w: the global seed across shards -- the GPU suite (rescore's bound output, the new entry
# points), then the W = 8 / W = 2 per-rank emulation on one GPU (tools/global_seed_rank.py).
export TMPDIR=/tmp
T=tools/gpu_step.sh
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
$T r05w_gs_tests 400 $P tests/test_global_seed_gpu.py && \
$T r05w_tests 700 $P tests -m gpu && \
$T r05w_rank8 400 python -u tools/global_seed_rank.py 10000000 768 1024 32 8 2 && \
$T r05w_rank2 300 python -u tools/global_seed_rank.py 10000000 768 1024 32 2 2 && \
echo ALLDONE_W
