#!/bin/bash
# r03_diag2.sh — configs[1] QW1 / QW1-nw8 stamps with and without the appends' global stores
# (diagnostic build), and the fused finish kernel vs separate merge + rescore at configs[1] and
# at the W = 8 rank shape.
export TMPDIR=/tmp
T=tools/gpu_step.sh
S=hc-rag_amd/lib/stamps_qw1/libhcrag_hip.so
NS=hc-rag_amd/lib/stamps_qw1ns/libhcrag_hip.so
C1="python bench.py --rows 1000000 --dim 384 --global-batch 256 --k 10 --steps 50 --warmup 5 --encoder none --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --sweep ,"
W8="python bench.py --encoder none --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --sweep , --steps 30 --warmup 3 --rows 1250000"
HCRAG_LIB=$S $T r03f_st1 200 python -u tools/qw1_stamps.py 1000000 384 256 1 0 && \
HCRAG_LIB=$NS $T r03f_st1ns 200 python -u tools/qw1_stamps.py 1000000 384 256 1 0 && \
HCRAG_LIB=$S $T r03f_st3 200 python -u tools/qw1_stamps.py 1000000 384 256 3 0 && \
HCRAG_LIB=$NS $T r03f_st3ns 200 python -u tools/qw1_stamps.py 1000000 384 256 3 0 && \
$T r03f_c1_fin 200 $C1 && \
HCRAG_NO_FINISH=1 $T r03f_c1_sep 200 $C1 && \
$T r03f_w8_fin 300 $W8 && \
HCRAG_NO_FINISH=1 $T r03f_w8_sep 300 $W8 && \
$T r03f_c1_fin2 200 $C1 && \
HCRAG_NO_FINISH=1 $T r03f_w8_sep2 300 $W8 && \
$T r03f_w8_fin2 300 $W8 && \
echo ALLDONE
