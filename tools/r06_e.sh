#!/bin/bash
# r06_e.sh TAG — deep-k fix check + deep/exact tests; encoder: DM 10 (one wave per SIMD) tests,
# LN-light (residual from xh) precision tests, A/B over DM {0,4,10} x {1 stream, 2 streams
# without the K-split remainder} and LN-light on/off.
export TMPDIR=/tmp
TAG=${1:-r06e}
S=tools/gpu_step.sh
mkdir -p gpurun_out
T() { "$S" "$@"; r=$?; [ $r -eq 99 ] && exit 99; return 0; }
T ${TAG}_dbg 120 python tools/dbg_deep.py && \
T ${TAG}_exact_deep 600 python -u -m pytest tests/test_exact_gpu.py -x -q --timeout 300 --timeout-method thread -k "deep" && \
T ${TAG}_enc_tests 300 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 240 --timeout-method thread && \
HCRAG_SPLIT_DM=10 T ${TAG}_enc_tests_dm10 300 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 240 --timeout-method thread -k "reference_precision or split or bge or minilm" && \
AB() { timeout -k 10 120 env "$@" python tools/enc_prof.py --steps 10 | sed "s|\"split_dm\"|\"env\": \"$*\", \"split_dm\"|" >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || exit 99; }
for r in 1 2; do
  AB HCRAG_SPLIT_DM=0 && AB HCRAG_SPLIT_DM=4 && AB HCRAG_SPLIT_DM=10 && \
  AB HCRAG_SPLIT_DM=0 HCRAG_ENC_STREAMS=2 HCRAG_SPLIT_NONE=1 && AB HCRAG_SPLIT_DM=4 HCRAG_ENC_STREAMS=2 HCRAG_SPLIT_NONE=1 && \
  AB HCRAG_SPLIT_DM=10 HCRAG_ENC_STREAMS=2 HCRAG_SPLIT_NONE=1 && AB HCRAG_SPLIT_DM=4 HCRAG_LN_WITHX=1 || exit 99
done && \
HCRAG_SPLIT_DM=10 T ${TAG}_kt_dm10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_dm10 -o run -- python tools/enc_prof.py --steps 5 && \
echo ALLDONE
