#!/bin/bash
# qw_ab.sh — QW parity tests + headline bench (QW) + SQ pass of the QW kernel, each step under its own limit
export TMPDIR=/tmp
T=tools/gpu_step.sh
B="python bench.py --steps 20 --warmup 3 --encoder none --no-cpu-baseline --no-configs0 --sweep ,"
$T qw_tests 400 python -u -m pytest tests/test_qw_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider && \
$T qw_bench 300 $B && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/qwab_sq -o run -- python bench.py --steps 3 --warmup 1 --encoder none --no-cpu-baseline --no-configs0 --sweep , > /dev/null 2>&1 && echo ALLDONE
