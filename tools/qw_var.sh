#!/bin/bash
# qw_var.sh — QW stage-shape A/B on the headline (default vs HCRAG_QW_VARIANT=$V), the variant's
# parity tests first; each step under its own limit.
export TMPDIR=/tmp
V=${1:-1}
T=tools/gpu_step.sh
B="python bench.py --steps 20 --warmup 3 --encoder none --no-cpu-baseline --no-configs0 --sweep ,"
HCRAG_QW_VARIANT=$V $T qwv_tests 400 python -u -m pytest tests/test_qw_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider && \
$T qwv_bench0 300 $B && \
HCRAG_QW_VARIANT=$V $T qwv_bench1 300 $B && \
$T qwv_bench0b 300 $B && echo ALLDONE
