#!/bin/bash
# r04q: the split GEMM's last round as K-chunks -- encoder parity, the encoder leg and f32
# pipeline A/B against whole-tile rounds (HCRAG_SPLIT_NONE=1), kernel traces at 96 / 97 tiles.
export TMPDIR=/tmp
T=tools/gpu_step.sh
E="python bench.py --rows 200000 --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --pipe-modes , --enc-modes f32 --steps 3 --warmup 1 --enc-steps 10"
$T r04q_enctests 500 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T r04q_pipe 700 tools/ab_pipe.sh r04q_pipe 2 HCRAG_SPLIT_NONE=1 X=0 && \
$T r04q_177 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04q_177 -o run -- $E --enc-seed 177 && \
$T r04q_77 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04q_77 -o run -- $E --enc-seed 77 && \
echo ALLDONE_Q
