#!/bin/bash
# enc_ft_ab.sh — 192- vs 256-feature tiles of the split GEMM (HCRAG_GEMM_FT=256 forces 256):
# encoder GPU tests, then the f32 encoder bench leg both ways and a kernel trace of the default.
export TMPDIR=/tmp
T=tools/gpu_step.sh
E="python bench.py --rows 200000 --steps 3 --warmup 1 --no-cpu-baseline --no-configs0 --sweep , --enc-modes f32"
$T ef_tests 600 python -u -m pytest tests/test_encoder_gpu.py tests/test_configs0_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider && \
$T ef_default 300 $E && \
HCRAG_GEMM_FT=256 $T ef_256 300 $E && \
$T ef_default2 300 $E && \
$T ef_kt 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ef_kt -o run -- $E && echo ALLDONE
