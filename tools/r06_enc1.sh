#!/bin/bash
# r06_enc1.sh TAG — VERDICT r5 items 1 + 2, first measurements:
#  (1) the f32 encoder's split GEMM with the LDS-DMA issue placement DM = 0 / 1 / 2
#      (HCRAG_SPLIT_DM; gemm_split_kernel) -- encoder GPU tests under DM 2 and 1, interleaved
#      enc_prof A/B, kernel traces per DM, SQ counter passes (DM 0 / 2 and the vendor GEMM in
#      the same process: tools/enc_prof.py --mm);
#  (2) the QW vs QW64 matrix-loop microbenchmark (tools/mfma_shape_ab 64).
# Every GPU step under its own limit, chained with && (tools/gpu_step.sh).
export TMPDIR=/tmp
TAG=${1:-r06a}
S=tools/gpu_step.sh
mkdir -p gpurun_out
SQ1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
SQ2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
$S ${TAG}_qw64 120 tools/bin/mfma_shape_ab 40000 4 64 && \
HCRAG_SPLIT_DM=2 $S ${TAG}_enc_tests_dm2 300 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 240 --timeout-method thread && \
HCRAG_SPLIT_DM=1 $S ${TAG}_enc_tests_dm1 300 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 240 --timeout-method thread -k "reference_precision or split" && \
for r in 1 2 3; do
  for dm in 0 1 2; do
    HCRAG_SPLIT_DM=$dm timeout -k 10 120 python tools/enc_prof.py --steps 10 >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || exit 99
  done
done && \
for dm in 0 2; do
  HCRAG_SPLIT_DM=$dm $S ${TAG}_kt_dm$dm 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_dm$dm -o run -- python tools/enc_prof.py --steps 5 || exit 99
done && \
for dm in 0 2; do
  HCRAG_SPLIT_DM=$dm $S ${TAG}_sq1_dm$dm 120 rocprofv3 --pmc $SQ1 --output-format csv -d gpurun_out/${TAG}_sq1_dm$dm -o run -- python tools/enc_prof.py --steps 3 --mm 10 || exit 99
  HCRAG_SPLIT_DM=$dm $S ${TAG}_sq2_dm$dm 120 rocprofv3 --pmc $SQ2 --output-format csv -d gpurun_out/${TAG}_sq2_dm$dm -o run -- python tools/enc_prof.py --steps 3 --mm 10 || exit 99
done && echo ALLDONE
