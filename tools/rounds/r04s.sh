#!/bin/bash
# r04s: f32 attention with 8-byte output stores -- encoder parity and the f32 encoder trace.
export TMPDIR=/tmp
T=tools/gpu_step.sh
E="python bench.py --rows 200000 --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --pipe-modes , --enc-modes f32 --steps 3 --warmup 1 --enc-steps 10"
$T r04s_enctests 500 python -u -m pytest tests/test_encoder_gpu.py tests/test_configs0_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T r04s_77 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04s_77 -o run -- $E --enc-seed 77 && \
$T r04s_enc 300 $E && \
echo ALLDONE_S
