#!/bin/bash
# kernel trace of configs[1] (1M x 384, B = 256, top-10) after the pre-pass threshold change
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T kt1 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01g_kt1 -o run -- python bench.py --rows 1000000 --dim 384 --batch 256 --k 10 --encoder none --no-cpu-baseline --steps 50
