#!/bin/bash
# r04n: the f32 encoder leg at the pipeline's token count (seed 177: T = 24680, 97 token tiles)
# vs the encoder leg's own (seed 77: T = 24571, 96 tiles), stream-K on / off, with kernel traces.
export TMPDIR=/tmp
T=tools/gpu_step.sh
E="python bench.py --rows 200000 --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --pipe-modes , --enc-modes f32 --steps 3 --warmup 1 --enc-steps 10"
$T r04n_177sk 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04n_177sk -o run -- $E --enc-seed 177 && \
$T r04n_177nosk 200 env HCRAG_SPLIT_NOSK=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04n_177nosk -o run -- $E --enc-seed 177 && \
$T r04n_77sk 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04n_77sk -o run -- $E --enc-seed 77 && \
$T r04n_77nosk 200 env HCRAG_SPLIT_NOSK=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04n_77nosk -o run -- $E --enc-seed 77 && \
echo ALLDONE_N
