#!/bin/bash
# qw_sweep.sh — where QW should take over from QS: batch sweeps at 10M x 768 and at configs[1]'s
# 1M x 384 (k = 10) with the default routing and with QW from 129 queries (HCRAG_QW_MIN=129).
export TMPDIR=/tmp
T=tools/gpu_step.sh
H="python bench.py --steps 10 --warmup 2 --encoder none --no-cpu-baseline --no-configs0"
C1="python bench.py --rows 1000000 --dim 384 --global-batch 256 --k 10 --steps 30 --warmup 3 --encoder none --no-cpu-baseline --no-configs0"
$T sw_h0 300 $H --sweep 160,256,512 && \
HCRAG_QW_MIN=129 $T sw_h1 300 $H --sweep 160,256,512 && \
$T sw_c0 300 $C1 --sweep 160,256,512,1024 && \
HCRAG_QW_MIN=129 $T sw_c1 300 $C1 --sweep 160,256,512,1024 && echo ALLDONE
