#!/bin/bash
# r03_sq.sh — SQ counters of the headline search (configs[2], the QW dense pass + its QW MAXONLY
# pre-pass): MFMA busy, wave-cycle buckets, LDS bank conflicts; then GRBM_GUI_ACTIVE with the L2
# hit / miss counts (each pass its own run; tools/pmc_summary.py).
export TMPDIR=/tmp
T=tools/gpu_step.sh
H="python bench.py --no-cpu-baseline --encoder none --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --steps 3 --warmup 1"
$T sq_headline 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/sq_headline -o run -- $H && \
$T tcc_headline 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/tcc_headline -o run -- $H && \
echo ALLDONE
