#!/bin/bash
# configs[1] (1M x 384, B = 256, top-10): pre-pass threshold / stride sweep (env overrides)
T=tools/gpu_step.sh
C="python bench.py --rows 1000000 --dim 384 --batch 256 --k 10 --encoder none --no-cpu-baseline --steps 30"
$T c1_default 120 $C && \
$T c1_mt1 120 env HCRAG_PREPASS_MIN_TILES=1 $C && \
$T c1_mt1_s32 120 env HCRAG_PREPASS_MIN_TILES=1 HCRAG_SAMPLE_STRIDE=32 $C && \
$T c1_mt1_s16 120 env HCRAG_PREPASS_MIN_TILES=1 HCRAG_SAMPLE_STRIDE=16 $C && \
$T c1_mt1_s8 120 env HCRAG_PREPASS_MIN_TILES=1 HCRAG_SAMPLE_STRIDE=8 $C && \
$T c1_mt1_s4 120 env HCRAG_PREPASS_MIN_TILES=1 HCRAG_SAMPLE_STRIDE=4 $C && \
$T b64_default 120 python bench.py --rows 1000000 --dim 384 --batch 64 --k 10 --encoder none --no-cpu-baseline --steps 30 && \
$T b64_mt1 120 env HCRAG_PREPASS_MIN_TILES=1 python bench.py --rows 1000000 --dim 384 --batch 64 --k 10 --encoder none --no-cpu-baseline --steps 30 && \
$T b64_mt1_s64 120 env HCRAG_PREPASS_MIN_TILES=1 HCRAG_SAMPLE_STRIDE=64 python bench.py --rows 1000000 --dim 384 --batch 64 --k 10 --encoder none --no-cpu-baseline --steps 30
