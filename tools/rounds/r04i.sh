#!/bin/bash
# r04i: encoder parity after the split GEMM's sc1 slab reads (stream-K, packing, two streams,
# full depth), the configs[1] leg, the stream-K A/B, then r04h (B = 256 stage shape, configs[1]
# QS vs QW).
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T r04i_enctests 400 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "stream_k or two_stream or packed or full_depth" && \
$T r04i_c1 200 python bench.py --rows 200000 --encoder none --no-cpu-baseline --no-configs0 --no-configs4 --no-vendor-gemm --sweep 32,256 --large-k , --power-seconds 0 && \
$T r04i_ab 500 tools/ab_enc.sh r04i_ab 2 HCRAG_SPLIT_NOSK=1 X=0 && \
bash tools/rounds/r04h.sh && echo ALLDONE_I
