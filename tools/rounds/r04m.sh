#!/bin/bash
# r04m: kernel traces of the f32 query pipeline leg (encoder on the 10M x 768 search's stream)
# with and without the split GEMM's stream-K
export TMPDIR=/tmp
T=tools/gpu_step.sh
P="python bench.py --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --enc-modes , --pipe-modes f32 --steps 3 --warmup 1"
$T r04m_sk 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04m_sk -o run -- $P && \
$T r04m_nosk 300 env HCRAG_SPLIT_NOSK=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04m_nosk -o run -- $P && \
echo ALLDONE_M
