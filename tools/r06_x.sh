#!/bin/bash
# r06_x.sh TAG -- the query pipeline leg with two batches in flight (encode of batch i+1 on a
# side stream beside the search of batch i), f32 and f16, on the headline corpus.
export TMPDIR=/tmp
TAG=${1:-r06x}
S=tools/gpu_step.sh
mkdir -p gpurun_out
T() { "$S" "$@"; r=$?; [ $r -eq 99 ] && exit 99; return $r; }
T ${TAG}_pipe 400 python -u bench.py --power-seconds 0 --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --sweep '' --large-k '' --no-vendor-gemm --enc-modes '' --steps 5 --warmup 2 --pipe-steps 10 && \
echo ALLDONE
