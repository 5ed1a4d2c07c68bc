#!/bin/bash
# qw_check.sh — QW kernel parity tests, then the headline bench with QW (default) and v4
# (HCRAG_QW_MIN=100000) in one call, each step under its own limit (tools/gpu_step.sh).
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T qw_tests 400 python -u -m pytest tests/test_qw_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider && \
$T qw_bench 300 python bench.py --steps 20 --warmup 3 --encoder none --no-cpu-baseline --no-configs0 --sweep "" && \
HCRAG_QW_MIN=100000 $T qw_bench_v4 300 python bench.py --steps 20 --warmup 3 --encoder none --no-cpu-baseline --no-configs0 --sweep "" && \
echo ALLDONE
