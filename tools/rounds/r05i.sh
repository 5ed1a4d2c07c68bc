#!/bin/bash
# r05i: the round-end evidence set at HEAD (tools/evidence.sh) + the headline's FETCH_SIZE /
# WRITE_SIZE passes (profiles/traffic_score.json is re-derived from them); then r05j.
export TMPDIR=/tmp
T=tools/gpu_step.sh
H="python bench.py --no-cpu-baseline --encoder none --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0"
bash tools/evidence.sh r05i && \
$T r05i_fetch 150 timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r05i_fetch -o run -- $H --steps 4 --warmup 1 && \
$T r05i_write 150 timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r05i_write -o run -- $H --steps 4 --warmup 1 && \
bash tools/rounds/r05j.sh && \
echo ALLDONE_I
