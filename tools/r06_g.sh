#!/bin/bash
# r06_g.sh TAG — staggered split GEMM (DM 5, DM 6 = + s_setprio for waves 4-7) against DM 4 (the
# default, two streams): encoder tests under each, interleaved A/B (bge-base and bge-large), then
# the kernel trace and an SQ pass of the winner candidate DM 5.
export TMPDIR=/tmp
TAG=${1:-r06g}
S=tools/gpu_step.sh
mkdir -p gpurun_out
T() { "$S" "$@"; r=$?; [ $r -eq 99 ] && exit 99; return 0; }
SQ1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
HCRAG_SPLIT_DM=5 T ${TAG}_enc_tests_dm5 300 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 240 --timeout-method thread -k "reference_precision or split or bge or minilm or two_stream" && \
HCRAG_SPLIT_DM=6 T ${TAG}_enc_tests_dm6 300 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 240 --timeout-method thread -k "reference_precision or bge" && \
AB() { timeout -k 10 120 env "$@" python tools/enc_prof.py --steps 10 | sed "s|\"split_dm\"|\"env\": \"$*\", \"split_dm\"|" >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || exit 99; }
ABL() { timeout -k 10 120 env "$@" python tools/enc_prof.py --steps 5 --model bge-large | sed "s|\"split_dm\"|\"env\": \"$*\", \"split_dm\"|" >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || exit 99; }
for r in 1 2; do
  AB HCRAG_SPLIT_DM=4 && AB HCRAG_SPLIT_DM=5 && AB HCRAG_SPLIT_DM=6 && AB HCRAG_SPLIT_DM=5 HCRAG_ENC_STREAMS=1 && \
  ABL HCRAG_SPLIT_DM=4 && ABL HCRAG_SPLIT_DM=5 || exit 99
done && \
HCRAG_SPLIT_DM=5 T ${TAG}_kt_dm5 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_dm5 -o run -- python tools/enc_prof.py --steps 5 && \
HCRAG_SPLIT_DM=5 HCRAG_ENC_STREAMS=1 T ${TAG}_sq_dm5 120 rocprofv3 --pmc $SQ1 --output-format csv -d gpurun_out/${TAG}_sq_dm5 -o run -- python tools/enc_prof.py --steps 3 && \
BE() { tag=$1; ev=$2; shift 2; timeout -k 10 240 env $ev python -u bench.py "$@" --power-seconds 0 --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --pipe-modes '' --sweep '' --large-k '' --no-vendor-gemm --enc-modes f32 --steps 5 --warmup 2 > gpurun_out/${TAG}_be_${tag}.log 2>&1 || exit 99; }
BE small_s2 HCRAG_SPLIT_DM=4 --rows 200000 && BE small_s1 HCRAG_ENC_STREAMS=1 --rows 200000 && \
BE big_s2 HCRAG_SPLIT_DM=4 && BE big_s1 HCRAG_ENC_STREAMS=1 && BE big_s2_pow3 HCRAG_SPLIT_DM=4 --power-seconds 3 && \
echo ALLDONE
