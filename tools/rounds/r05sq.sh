#!/bin/bash
# r05sq: SQ counters at HEAD (separate --pmc passes, no trace domains): the headline search and
# configs[1] -- MFMA busy, wait / issue shares; then the LDS counters of the headline.
export TMPDIR=/tmp
T=tools/gpu_step.sh
H="python bench.py --no-cpu-baseline --encoder none --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --steps 4 --warmup 1"
C1="python bench.py --rows 1000000 --dim 384 --global-batch 256 --k 10 --encoder none --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --steps 10 --warmup 2"
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
LDS="SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES"
$T r05sq_head 200 timeout -s KILL 180 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/r05sq_head -o run -- $H && \
$T r05sq_c1 200 timeout -s KILL 180 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/r05sq_c1 -o run -- $C1 && \
$T r05sq_lds 200 timeout -s KILL 180 rocprofv3 --pmc $LDS --output-format csv -d gpurun_out/r05sq_lds -o run -- $H && \
echo ALLDONE_SQ
