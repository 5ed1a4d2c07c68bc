#!/bin/bash
# enc_split_ab.sh — reference-precision GEMMs on gemm_split_kernel: QW + encoder GPU tests, the
# encoder bench leg (f32 mode) with the split kernel and with the concatenated GEMM
# and a kernel trace of the split run, then the headline bench.
export TMPDIR=/tmp
T=tools/gpu_step.sh
E="python bench.py --rows 200000 --steps 3 --warmup 1 --no-cpu-baseline --no-configs0 --sweep , --enc-modes f32"
$T es_tests 600 python -u -m pytest tests/test_qw_gpu.py tests/test_encoder_gpu.py tests/test_configs0_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider && \
$T es_bench_split 300 $E && \
$T es_kt 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/es_kt -o run -- $E && \
$T es_head 300 python bench.py --encoder none --no-cpu-baseline --no-configs0 --sweep , && echo ALLDONE
