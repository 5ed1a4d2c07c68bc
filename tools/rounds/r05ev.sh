#!/bin/bash
# r05ev: kernel traces + HBM traffic passes at HEAD (the headline and configs[1]), matching the
# r05c3 bench line (same code; GPU suite + smoke at this code: r05fin).
export TMPDIR=/tmp
T=tools/gpu_step.sh
TAG=r05ev
H="python bench.py --no-cpu-baseline --encoder none --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0"
C1="python bench.py --rows 1000000 --dim 384 --global-batch 256 --k 10 --encoder none --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k ,"
$T ${TAG}_kt 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt -o run -- $H --steps 10 --warmup 2 && \
$T ${TAG}_fetch 150 timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_fetch -o run -- $H --steps 4 --warmup 1 && \
$T ${TAG}_write 150 timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_write -o run -- $H --steps 4 --warmup 1 && \
$T ${TAG}_c1_kt 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_c1_kt -o run -- $C1 --steps 20 --warmup 3 && \
$T ${TAG}_c1_fetch 120 timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_c1_fetch -o run -- $C1 --steps 4 --warmup 1 && \
$T ${TAG}_c1_write 120 timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_c1_write -o run -- $C1 --steps 4 --warmup 1 && \
echo ALLDONE_EV
