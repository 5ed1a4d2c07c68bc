#!/bin/bash
# r04y: SQ counters of the headline search at HEAD (MFMA busy, wave-cycle buckets, LDS) and the
# configs[1] leg's kernel trace.
export TMPDIR=/tmp
T=tools/gpu_step.sh
H="python bench.py --no-cpu-baseline --encoder none --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0"
C="python bench.py --rows 200000 --encoder none --no-cpu-baseline --no-configs0 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --steps 3 --warmup 1"
$T r04y_sq 200 timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r04y_sq -o run -- $H --steps 4 --warmup 1 && \
$T r04y_c1kt 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04y_c1kt -o run -- $C && \
echo ALLDONE_Y
