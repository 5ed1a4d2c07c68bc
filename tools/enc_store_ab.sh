#!/bin/bash
# enc_store_ab.sh — FFN1 split activations stored through LDS: encoder GPU tests (max |diff|
# printed), the f32 encoder bench leg, a kernel trace of it.
export TMPDIR=/tmp
T=tools/gpu_step.sh
E="python bench.py --rows 200000 --steps 3 --warmup 1 --no-cpu-baseline --no-configs0 --sweep , --enc-modes f32,f16"
$T est_tests 600 python -u -m pytest tests/test_encoder_gpu.py tests/test_configs0_gpu.py -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider && \
$T est_bench 300 $E && \
$T est_kt 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/est_kt -o run -- $E && echo ALLDONE
