#!/bin/bash
# r03_qw1_prof.sh — why QW1 is not faster than QW: kernel-choice debug on the configs[4] shape,
# then a kernel trace and one SQ counter pass of QW (variant 0) and QW1 (variant 2) on configs[2]
# in one process each (the two kernels have different names).
export TMPDIR=/tmp
T=tools/gpu_step.sh
A="python tools/qw1_ab.py --shapes c2 --rounds 1 --variants 0,2,1 --reps 2"
HCRAG_DEBUG_CFG=1 $T r03b_c4dbg 300 python -u tools/qw1_ab.py --shapes c4 --rounds 1 --variants 1 --reps 1 && \
$T r03b_kt 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03b_kt -o run -- $A && \
$T r03b_sq 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r03b_sq -o run -- $A && \
$T r03b_sq2 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC --output-format csv -d gpurun_out/r03b_sq2 -o run -- $A && \
echo ALLDONE
