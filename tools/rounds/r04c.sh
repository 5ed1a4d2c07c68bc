#!/bin/bash
# r04c: evidence at HEAD -- the headline traced in the SAME process as a timed bench run (its
# JSON line next to the kernel stats), the headline's HBM traffic (FETCH_SIZE / WRITE_SIZE
# passes, tools/pmc_summary.py --traffic), and the f32 / f16 encoders' per-kernel trace with the
# token packing (bge-base, 1024 x S = 32 ragged).
export TMPDIR=/tmp
T=tools/gpu_step.sh
H="python bench.py --no-cpu-baseline --encoder none --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0"
E="python bench.py --rows 200000 --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --pipe-modes , --steps 3 --warmup 1 --enc-steps 5"
$T r04c_hkt 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04c_hkt -o run -- $H --steps 20 --warmup 3 && \
$T r04c_fetch 200 timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r04c_fetch -o run -- $H --steps 4 --warmup 1 && \
$T r04c_write 200 timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r04c_write -o run -- $H --steps 4 --warmup 1 && \
$T r04c_ekt 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04c_ekt -o run -- $E && \
echo ALLDONE
