#!/bin/bash
# 33-64 queries by corpus size: GPU suite, smoke, default bench, configs[1] bench
T=tools/gpu_step.sh
$T gpu_tests 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread && \
$T smoke 200 python -c "import __graft_entry__ as g; g.smoke()" && \
$T bench 400 python bench.py && \
$T cfg1 300 python bench.py --rows 1000000 --dim 384 --batch 256 --k 10 --encoder minilm --cpu-queries 256 --sweep 1,16,32,48,64,100,256,1024
