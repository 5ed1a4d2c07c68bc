#!/bin/bash
# profile.sh TAG — rocprofv3 passes over bench.py on the GPU box (one step per pass, each
# under its own time limit via gpu_step.sh): kernel trace + stats, then PMC passes
# (FETCH_SIZE alone; SQ cycle/wait/MFMA/LDS counters; L2 hit/miss).  Output: gpurun_out/prof_TAG*
tag=${1:-r01}
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline"
T=tools/gpu_step.sh
$T prof_kt 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_kt -o run -- $B --steps 10 --warmup 2 && \
$T prof_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_${tag}_fetch -o run -- $B --steps 3 --warmup 1 --encoder none && \
$T prof_sq 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/prof_${tag}_sq -o run -- $B --steps 3 --warmup 1 --encoder none && \
$T prof_tcc 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof_${tag}_tcc -o run -- $B --steps 3 --warmup 1 --encoder none
