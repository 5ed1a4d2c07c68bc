#!/bin/bash
# r04o: split GEMM as two instantiations (whole-tile rounds without the segment loop, then the
# stream-K launch on 192-wide tiles): encoder parity, the encoder leg and the f32 pipeline A/B
# against whole tiles, and kernel traces at both token counts.
export TMPDIR=/tmp
T=tools/gpu_step.sh
E="python bench.py --rows 200000 --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --pipe-modes , --enc-modes f32 --steps 3 --warmup 1 --enc-steps 10"
$T r04o_enctests 400 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "stream_k or two_stream or packed or full_depth or variants" && \
$T r04o_pipe 700 tools/ab_pipe.sh r04o_pipe 2 HCRAG_SPLIT_NOSK=1 X=0 && \
$T r04o_177sk 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04o_177sk -o run -- $E --enc-seed 177 && \
$T r04o_77sk 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04o_77sk -o run -- $E --enc-seed 77 && \
echo ALLDONE_O
