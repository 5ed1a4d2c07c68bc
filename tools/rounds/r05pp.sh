#!/bin/bash
# r05pp: the sampling pre-pass on v4's MAXONLY form (PREPASS=1) vs QW's (default under QW),
# interleaved in one process: configs[1], 10M x 768 at B = 256 and the headline.
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T r05pp_c1 300 python tools/opt_ab.py 1000000 384 256 10 6 default PREPASS=1 && \
$T r05pp_b256 300 python tools/opt_ab.py 10000000 768 256 32 3 default PREPASS=1 && \
$T r05pp_c2 300 python tools/opt_ab.py 10000000 768 1024 32 3 default PREPASS=1 && \
echo ALLDONE_PP
