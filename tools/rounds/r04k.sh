#!/bin/bash
# r04k: the default bench line at HEAD (what the driver runs), then the headline traced in the
# bench's own process, its FETCH_SIZE / WRITE_SIZE passes, and the f32 / f16 encoder kernel trace.
export TMPDIR=/tmp
T=tools/gpu_step.sh
H="python bench.py --no-cpu-baseline --encoder none --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0"
E="python bench.py --rows 200000 --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --pipe-modes , --steps 3 --warmup 1 --enc-steps 5"
$T r04k_bench 600 python bench.py && \
$T r04k_hkt 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04k_hkt -o run -- $H --steps 20 --warmup 3 && \
$T r04k_fetch 200 timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r04k_fetch -o run -- $H --steps 4 --warmup 1 && \
$T r04k_write 200 timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r04k_write -o run -- $H --steps 4 --warmup 1 && \
$T r04k_ekt 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04k_ekt -o run -- $E && \
echo ALLDONE_K
