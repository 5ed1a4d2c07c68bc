#!/bin/bash
# r06_q.sh TAG -- round-6 evidence at HEAD: rocprofv3 kernel trace + stats of the default bench
# command (the roofline kernel's launches), the f32 encoder's kernel trace (per layer) and one SQ
# counter pass of it (DM 4, two sub-batch streams: the default).
export TMPDIR=/tmp
TAG=${1:-r06q}
S=tools/gpu_step.sh
mkdir -p gpurun_out
T() { "$S" "$@"; r=$?; [ $r -eq 99 ] && exit 99; return $r; }
SQ1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
T ${TAG}_kt_enc 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_enc -o run -- python tools/enc_prof.py --steps 5 && \
T ${TAG}_sq_enc 120 rocprofv3 --pmc $SQ1 --output-format csv -d gpurun_out/${TAG}_sq_enc -o run -- python tools/enc_prof.py --steps 3 && \
T ${TAG}_kt_bench 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_bench -o run -- python bench.py && \
echo ALLDONE
