#!/bin/bash
# r01g evidence for the committed defaults: kernel trace + stats of the default bench command,
# FETCH_SIZE / WRITE_SIZE passes over the score leg (HBM traffic per score phase), bench line
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T kt 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01g_kt -o run -- python bench.py --no-cpu-baseline && \
$T fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r01g_fetch -o run -- python bench.py --no-cpu-baseline --encoder none --steps 3 --warmup 1 && \
$T write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r01g_write -o run -- python bench.py --no-cpu-baseline --encoder none --steps 3 --warmup 1 && \
$T bench 400 python bench.py
