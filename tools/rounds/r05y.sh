#!/bin/bash
# r05y: the W = 8 emulation with the sample on v4's MAXONLY form (PREPASS=1: no 1024-query
# fragment prologue) vs QW's.
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T r05y_rank8_v4 400 python -u tools/global_seed_rank.py 10000000 768 1024 32 8 2 PREPASS=1 && \
$T r05y_rank8_qw 400 python -u tools/global_seed_rank.py 10000000 768 1024 32 8 2 && \
echo ALLDONE_Y
