#!/bin/bash
# kernel trace + FETCH/WRITE passes over the headline bench (score leg), then the GEMM calibration
export TMPDIR=/tmp
T=tools/gpu_step.sh
B="python bench.py --no-cpu-baseline --encoder none"
$T kt 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt -o run -- $B --steps 5 --warmup 2 && \
$T fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/fetch -o run -- $B --steps 3 --warmup 1 && \
$T write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/write -o run -- $B --steps 3 --warmup 1 && \
$T calib 300 python tools/calib_gemm.py
