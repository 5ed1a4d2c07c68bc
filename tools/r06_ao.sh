#!/bin/bash
# r06_ao.sh TAG -- SQ counter passes of the r06 deep-k path (K6h / K6c / K6r at 1M x 384, k = 5000).
export TMPDIR=/tmp
TAG=${1:-r06ao}
S=tools/gpu_step.sh
mkdir -p gpurun_out
T() { "$S" "$@"; r=$?; [ $r -eq 99 ] && exit 99; return $r; }
SQ1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE"
SQ2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
T ${TAG}_sq1 120 rocprofv3 --pmc $SQ1 --output-format csv -d gpurun_out/${TAG}_sq1 -o run -- python tools/deep_prof.py --steps 2 && \
T ${TAG}_sq2 120 rocprofv3 --pmc $SQ2 --output-format csv -d gpurun_out/${TAG}_sq2 -o run -- python tools/deep_prof.py --steps 2 && \
echo ALLDONE
