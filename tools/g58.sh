#!/bin/bash
# bge-base / bge-large encoder parity, then bench lines for configs[1] (1M x 384, B = 256,
# top-10, MiniLM encoder) and the per-rank shape of configs[4] (100M x 1024 bf16 over 8 GPUs:
# 12.5M rows, nq = 8 x 1024, top-64, bge-large encoder) on one GPU
T=tools/gpu_step.sh
$T enc_tests 500 python -u -m pytest tests/test_encoder_gpu.py -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k bge_shapes && \
$T cfg1 300 python bench.py --rows 1000000 --dim 384 --batch 256 --k 10 --encoder minilm --cpu-queries 256 && \
$T cfg4r 500 python bench.py --rows 12500000 --dim 1024 --dtype bf16 --batch 8192 --k 64 --encoder bge-large --steps 3 --warmup 1 --enc-steps 3 --no-cpu-baseline
