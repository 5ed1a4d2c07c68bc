#!/bin/bash
# enc_gelu_ab.sh — the reference-precision FFN1 GELU on erf_as (default) vs the library erff
# (HCRAG_GELU_LIBERF=1): encoder GPU tests with their max |diff| printed, both ways, then the
# f32 encoder bench leg both ways on the same box.
export TMPDIR=/tmp
T=tools/gpu_step.sh
E="python bench.py --rows 200000 --steps 3 --warmup 1 --no-cpu-baseline --no-configs0 --sweep , --enc-modes f32"
P="python -u -m pytest tests/test_encoder_gpu.py tests/test_configs0_gpu.py -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider"
$T eg_tests 600 $P && \
HCRAG_GELU_LIBERF=1 $T eg_tests_lib 600 $P -k "precision or minilm" && \
$T eg_fast 300 $E && \
HCRAG_GELU_LIBERF=1 $T eg_lib 300 $E && \
$T eg_fast2 300 $E && echo ALLDONE
