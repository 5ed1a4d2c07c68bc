#!/bin/bash
# kernel trace of the W = 8 per-rank shape (1.25M rows, nq = 8192) on one GPU
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T kt8 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01g_kt8 -o run -- python bench.py --rows 1250000 --batch 8192 --encoder none --no-cpu-baseline --steps 10
