#!/bin/bash
# prof_qw.sh TAG — headline (configs[2]) with the QW kernel: kernel trace + stats, FETCH_SIZE and
# WRITE_SIZE passes, and one SQ pass (wave-cycle buckets, MFMA busy, LDS conflicts, clock).
export TMPDIR=/tmp
tag=${1:-qw}
mkdir -p gpurun_out
B="python bench.py --encoder none --no-cpu-baseline --no-configs0 --sweep ,"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_kt -o run -- $B --steps 10 --warmup 2 > gpurun_out/${tag}_kt.json 2>/dev/null && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_fetch -o run -- $B --steps 3 --warmup 1 > /dev/null 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${tag}_write -o run -- $B --steps 3 --warmup 1 > /dev/null 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${tag}_sq -o run -- $B --steps 3 --warmup 1 > /dev/null 2>&1 && echo done
