#!/bin/bash
# r06_c.sh TAG — (1) the hand-written deep-k path (no hipCUB) and the shard merge: exact GPU
# tests; (2) split GEMM DM = 4 (two stages in flight, pieces spread evenly) vs DM = 0: encoder
# tests + interleaved A/B; (3) QW vs QW64 (compiled / pipelined) microbenchmark; (4) configs[1]
# leg with the k = 5000 deep point; (5) DM 8 / 9 diagnostics (no LDS reads / no DMA: timing only).
export TMPDIR=/tmp
TAG=${1:-r06c}
S=tools/gpu_step.sh
mkdir -p gpurun_out
$S ${TAG}_exact 600 python -u -m pytest tests/test_exact_gpu.py -x -q --timeout 300 --timeout-method thread && \
$S ${TAG}_qw64 120 tools/bin/mfma_shape_ab 40000 3 64 && \
HCRAG_SPLIT_DM=4 $S ${TAG}_enc_tests_dm4 300 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 240 --timeout-method thread && \
HCRAG_SPLIT_DM=10 $S ${TAG}_enc_tests_dm10 300 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 240 --timeout-method thread -k "reference_precision or split or bge or minilm" && \
for r in 1 2 3; do
  for dm in 0 4 10; do
    HCRAG_SPLIT_DM=$dm timeout -k 10 120 python tools/enc_prof.py --steps 10 >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || exit 99
  done
done && \
for dm in 8 9; do
  HCRAG_SPLIT_DM=$dm timeout -k 10 120 python tools/enc_prof.py --steps 10 >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || exit 99
done && \
$S ${TAG}_c1 300 python bench.py --rows 2000000 --steps 3 --warmup 1 --no-cpu-baseline --no-configs0 --sweep , --large-k , --encoder none --pipe-modes , --no-configs4 --no-vendor-gemm --power-seconds 0 && \
echo ALLDONE
