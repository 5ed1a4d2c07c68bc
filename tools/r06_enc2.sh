#!/bin/bash
# r06_enc2.sh TAG — the split GEMM's DM = 3 (two stages in flight) against DM = 0: encoder GPU
# tests under DM 3, interleaved enc_prof A/B, kernel trace + SQ pass of DM 3.
export TMPDIR=/tmp
TAG=${1:-r06b}
S=tools/gpu_step.sh
mkdir -p gpurun_out
SQ1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
HCRAG_SPLIT_DM=3 $S ${TAG}_enc_tests_dm3 300 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 240 --timeout-method thread && \
for r in 1 2 3; do
  for dm in 0 3; do
    HCRAG_SPLIT_DM=$dm timeout -k 10 120 python tools/enc_prof.py --steps 10 >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || exit 99
    HCRAG_SPLIT_DM=$dm timeout -k 10 120 python tools/enc_prof.py --steps 5 --model bge-large >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || exit 99
  done
done && \
HCRAG_SPLIT_DM=3 $S ${TAG}_kt_dm3 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_dm3 -o run -- python tools/enc_prof.py --steps 5 && \
HCRAG_SPLIT_DM=3 $S ${TAG}_sq1_dm3 120 rocprofv3 --pmc $SQ1 --output-format csv -d gpurun_out/${TAG}_sq1_dm3 -o run -- python tools/enc_prof.py --steps 3 && \
echo ALLDONE
