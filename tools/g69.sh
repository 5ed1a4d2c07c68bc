#!/bin/bash
# rescore: candidate norms gathered up front, 8 candidate gathers per wave in flight;
# kernel trace of configs[1], GPU suite, default bench
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T kt1 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01g_kt1b -o run -- python bench.py --rows 1000000 --dim 384 --batch 256 --k 10 --encoder none --no-cpu-baseline --steps 50 && \
$T gpu_tests 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread && \
$T bench 400 python bench.py
