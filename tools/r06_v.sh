#!/bin/bash
# r06_v.sh TAG -- encoder sub-batch stream count 2 / 3 / 4 (HCRAG_ENC_STREAMS), f32 and f16,
# bge-base and bge-large, interleaved on one box; encoder tests under 3 streams.
export TMPDIR=/tmp
TAG=${1:-r06v}
S=tools/gpu_step.sh
mkdir -p gpurun_out
T() { "$S" "$@"; r=$?; [ $r -eq 99 ] && exit 99; return $r; }
HCRAG_ENC_STREAMS=3 T ${TAG}_enc_tests_s3 300 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 240 --timeout-method thread -k "reference_precision or split or bge or two_stream" || exit 99
AB() { m=$1; shift; timeout -k 10 120 env "$@" python tools/enc_prof.py --steps 10 --mode $m | sed "s|\"split_dm\"|\"env\": \"$* $m\", \"split_dm\"|" >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || exit 99; }
ABL() { timeout -k 10 120 env "$@" python tools/enc_prof.py --steps 5 --model bge-large | sed "s|\"split_dm\"|\"env\": \"$* large\", \"split_dm\"|" >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || exit 99; }
for r in 1 2 3; do
  AB f32 HCRAG_ENC_STREAMS=2 && AB f32 HCRAG_ENC_STREAMS=3 && AB f32 HCRAG_ENC_STREAMS=4 || exit 99
done
for r in 1 2; do
  AB f16 HCRAG_ENC_STREAMS=2 && AB f16 HCRAG_ENC_STREAMS=3 && AB f16 HCRAG_ENC_STREAMS=4 && \
  ABL HCRAG_ENC_STREAMS=2 && ABL HCRAG_ENC_STREAMS=3 || exit 99
done
echo ALLDONE
