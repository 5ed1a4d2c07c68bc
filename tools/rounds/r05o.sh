#!/bin/bash
# r05o: QW stamps (in-kernel clock) at HEAD after the ballot appends: W = 8 rank shape, headline,
# configs[1] -- where the per-stage time goes now.
export TMPDIR=/tmp
T=tools/gpu_step.sh
S="env HCRAG_LIB=hc-rag_amd/lib/stamps_qw/libhcrag_hip.so"
$T r05o_st_w8 200 $S python tools/qw_stamps.py 1250000 768 1024 32 && \
$T r05o_st_c2 200 $S python tools/qw_stamps.py 10000000 768 1024 32 && \
$T r05o_st_c1 200 $S python tools/qw_stamps.py 1000000 384 256 10 QW_STAGGER=0 && \
echo ALLDONE_O
