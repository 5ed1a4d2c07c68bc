#!/bin/bash
# r05z: the round-end evidence set at HEAD (tools/evidence.sh) + the headline's FETCH_SIZE /
# WRITE_SIZE passes.
export TMPDIR=/tmp
T=tools/gpu_step.sh
H="python bench.py --no-cpu-baseline --encoder none --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0"
bash tools/evidence.sh r05z && \
$T r05z_fetch 150 timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r05z_fetch -o run -- $H --steps 4 --warmup 1 && \
$T r05z_write 150 timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r05z_write -o run -- $H --steps 4 --warmup 1 && \
echo ALLDONE_Z
