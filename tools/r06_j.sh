#!/bin/bash
# r06_j.sh TAG -- split GEMM DM 7 / 8 (the slot-freeing barrier inside the MFMA phase) against
# DM 4: encoder tests under each, interleaved enc_prof A/B (bge-base, bge-large), kernel stats.
export TMPDIR=/tmp
TAG=${1:-r06j}
S=tools/gpu_step.sh
mkdir -p gpurun_out
T() { "$S" "$@"; r=$?; [ $r -eq 99 ] && exit 99; return $r; }
HCRAG_SPLIT_DM=7 T ${TAG}_enc_tests_dm7 300 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 240 --timeout-method thread -k "reference_precision or split or bge or two_stream" && \
HCRAG_SPLIT_DM=8 T ${TAG}_enc_tests_dm8 300 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 240 --timeout-method thread -k "reference_precision or bge" || exit 99
AB() { timeout -k 10 120 env "$@" python tools/enc_prof.py --steps 10 | sed "s|\"split_dm\"|\"env\": \"$*\", \"split_dm\"|" >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || exit 99; }
ABL() { timeout -k 10 120 env "$@" python tools/enc_prof.py --steps 5 --model bge-large | sed "s|\"split_dm\"|\"env\": \"$*\", \"split_dm\"|" >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || exit 99; }
for r in 1 2 3; do
  AB HCRAG_SPLIT_DM=4 && AB HCRAG_SPLIT_DM=7 && AB HCRAG_SPLIT_DM=8 || exit 99
done
ABL HCRAG_SPLIT_DM=4 && ABL HCRAG_SPLIT_DM=7 && ABL HCRAG_SPLIT_DM=8 && \
HCRAG_SPLIT_DM=7 T ${TAG}_kt_dm7 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_dm7 -o run -- python tools/enc_prof.py --steps 5 && \
HCRAG_SPLIT_DM=4 T ${TAG}_kt_dm4 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_dm4 -o run -- python tools/enc_prof.py --steps 5 && \
echo ALLDONE
