#!/bin/bash
# r04e: the split GEMM's stream-K completion -- its parity tests (stream-K vs whole tiles, the
# two-stream and packing bit tests, full-depth reference precision), an A/B of the encoder legs
# against HCRAG_SPLIT_NOSK=1, and the f32 / f16 encoders' kernel trace.
export TMPDIR=/tmp
T=tools/gpu_step.sh
E="python bench.py --rows 200000 --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --pipe-modes , --steps 3 --warmup 1 --enc-steps 5"
$T r04e_tests 600 python -u -m pytest tests/test_encoder_gpu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "stream_k or two_stream or packed or full_depth or variants or ws_gemm" && \
$T r04e_ab 500 tools/ab_enc.sh r04e_ab 2 HCRAG_SPLIT_NOSK=1 X=0 && \
$T r04e_ekt 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04e_ekt -o run -- $E && \
echo ALLDONE_E
