#!/bin/bash
# r06_p.sh TAG -- gemm_split_rs_kernel (loader / compute waves; DM 12) against DM 4: random
# operand check + kernel timing at the encoder's shapes, encoder tests under DM 12, interleaved
# enc_prof A/B, kernel trace.
export TMPDIR=/tmp
TAG=${1:-r06p}
S=tools/gpu_step.sh
mkdir -p gpurun_out
T() { "$S" "$@"; r=$?; [ $r -eq 99 ] && exit 99; return $r; }
for shape in "3072 12288 768" "2304 12288 768" "768 12288 3072" "768 12288 768" "3072 1500 768"; do
  timeout -k 10 60 ./tools/rs_check.bin $shape >> gpurun_out/${TAG}_check.txt 2>&1
  rc=$?
  echo "rc=$rc" >> gpurun_out/${TAG}_check.txt
  [ $rc -ne 0 ] && [ $rc -ne 2 ] && exit 99
done
grep -q 'bad=[1-9]' gpurun_out/${TAG}_check.txt && { echo "RS mismatch"; cat gpurun_out/${TAG}_check.txt; exit 0; }
HCRAG_SPLIT_DM=12 T ${TAG}_enc_tests_rs 300 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 240 --timeout-method thread -k "reference_precision or split or bge or two_stream or minilm or packed" || exit 99
AB() { timeout -k 10 120 env "$@" python tools/enc_prof.py --steps 10 | sed "s|\"split_dm\"|\"env\": \"$*\", \"split_dm\"|" >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || exit 99; }
for r in 1 2 3; do
  AB HCRAG_SPLIT_DM=4 && AB HCRAG_SPLIT_DM=12 || exit 99
done
AB HCRAG_SPLIT_DM=12 HCRAG_ENC_STREAMS=1 && \
HCRAG_SPLIT_DM=12 T ${TAG}_kt_rs 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_rs -o run -- python tools/enc_prof.py --steps 5 && \
echo ALLDONE
cat gpurun_out/${TAG}_check.txt
