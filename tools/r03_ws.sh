#!/bin/bash
# r03_ws.sh — the weight-stationary encoder GEMM (gemm_ws.h): encoder GPU tests (incl. WS vs v4),
# encoder throughput A/B (WS default vs HCRAG_ENC_NO_WS), kernel trace of the f16 encoder, and the
# W = 8 rank shape at pre-pass strides 64 (default) / 128 / 256.
export TMPDIR=/tmp
T=tools/gpu_step.sh
E="python bench.py --rows 200000 --encoder bge-base --enc-modes f32,f16 --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --sweep , --pipe-modes , --steps 5 --warmup 2"
W8="python bench.py --encoder none --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --sweep , --steps 30 --warmup 3 --rows 1250000"
$T r03g_enc_tests 900 python -u -m pytest tests/test_exact_gpu.py tests/test_encoder_gpu.py -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider && \
$T r03g_enc_ws 300 $E && \
HCRAG_ENC_NO_WS=1 $T r03g_enc_v4 300 $E && \
$T r03g_enc_ws2 300 $E && \
$T r03g_enc_kt 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/enc_kt_r03 -o run -- python bench.py --rows 200000 --encoder bge-base --enc-modes f16 --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --sweep , --pipe-modes , --steps 3 --warmup 1 && \
HCRAG_SAMPLE_STRIDE=128 $T r03g_w8_s128 300 $W8 && \
HCRAG_SAMPLE_STRIDE=256 $T r03g_w8_s256 300 $W8 && \
$T r03g_w8_s64 300 $W8 && \
echo ALLDONE
