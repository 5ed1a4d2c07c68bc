#!/bin/bash
# r05p: the QW dense launch's time line (entry skew, prologue, loop, final lists) from the
# stamps build: configs[1] (plain and staggered) and the W = 8 rank shape.
export TMPDIR=/tmp
T=tools/gpu_step.sh
S="env HCRAG_LIB=hc-rag_amd/lib/stamps_qw/libhcrag_hip.so"
$T r05p_st_c1 200 $S python tools/qw_stamps.py 1000000 384 256 10 QW_STAGGER=0 && \
$T r05p_st_c1s 200 $S python tools/qw_stamps.py 1000000 384 256 10 && \
$T r05p_st_w8 200 $S python tools/qw_stamps.py 1250000 768 1024 32 && \
echo ALLDONE_P
