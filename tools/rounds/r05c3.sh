#!/bin/bash
# r05c3: the default bench line at HEAD, then configs[3]'s per-rank shape (10M x 768 over 8
# shards, 4096 gathered queries) with and without the global seed, emulated on one GPU.
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T r05c3_bench 600 python bench.py && \
$T r05c3_rank8 500 python -u tools/global_seed_rank.py 10000000 768 4096 32 8 2 && \
echo ALLDONE_C3
