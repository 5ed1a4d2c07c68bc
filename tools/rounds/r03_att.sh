#!/bin/bash
# r03_att.sh — the register-staged f32 attention: encoder parity tests (full depth vs fp32
# BertModel), the encoder throughput leg of the bench (f32 / f16), and a kernel trace of the
# f32 encoder (attention per layer call).
export TMPDIR=/tmp
T=tools/gpu_step.sh
E="python bench.py --rows 200000 --encoder bge-base --enc-modes f32,f16 --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --pipe-modes , --steps 5 --warmup 2"
$T att_tests 600 python -u -m pytest tests/test_encoder_gpu.py tests/test_configs0_gpu.py tests/test_ingest.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T att_bench 300 $E && \
$T att_kt 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_enc_att -o run -- python bench.py --rows 200000 --encoder bge-base --enc-modes f32 --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --pipe-modes , --steps 3 --warmup 1 && \
echo ALLDONE
