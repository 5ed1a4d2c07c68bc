#!/bin/bash
# r06_d.sh TAG — deep-k debug print, the exact tests except deep k, encoder DM 4 / 10 tests and
# A/B against DM 0, DM 8 / 9 diagnostics, QW vs QW64 microbenchmark.
export TMPDIR=/tmp
TAG=${1:-r06d}
S=tools/gpu_step.sh
mkdir -p gpurun_out
# T: a step whose test failures (rc 1) do not stop the call; a fault / time limit (99) does
T() { "$S" "$@"; r=$?; [ $r -eq 99 ] && exit 99; return 0; }
T ${TAG}_dbg 120 python tools/dbg_deep.py && \
$S ${TAG}_exact 600 python -u -m pytest tests/test_exact_gpu.py -x -q --timeout 300 --timeout-method thread -k "not deep" && \
$S ${TAG}_qw64 120 tools/bin/mfma_shape_ab 40000 3 64 && \
HCRAG_SPLIT_DM=4 T ${TAG}_enc_tests_dm4 300 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 240 --timeout-method thread -k "reference_precision or split or bge or minilm" && \
HCRAG_SPLIT_DM=10 T ${TAG}_enc_tests_dm10 300 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 240 --timeout-method thread -k "reference_precision or split or bge or minilm" && \
for r in 1 2; do
  for dm in 0 4 10; do
    HCRAG_SPLIT_DM=$dm timeout -k 10 120 python tools/enc_prof.py --steps 10 >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || exit 99
  done
done && \
for r in 1 2; do
  HCRAG_ENC_STREAMS=2 timeout -k 10 120 python tools/enc_prof.py --steps 10 | sed 's/"split_dm"/"streams": 2, "split_dm"/' >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || exit 99
  HCRAG_ENC_STREAMS=2 HCRAG_SPLIT_NONE=1 timeout -k 10 120 python tools/enc_prof.py --steps 10 | sed 's/"split_dm"/"streams": 2, "split_none": 1, "split_dm"/' >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || exit 99
done && \
for dm in 8 9; do
  HCRAG_SPLIT_DM=$dm timeout -k 10 120 python tools/enc_prof.py --steps 10 >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || exit 99
done && \
HCRAG_SPLIT_DM=10 $S ${TAG}_kt_dm10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_dm10 -o run -- python tools/enc_prof.py --steps 5 && \
echo ALLDONE
