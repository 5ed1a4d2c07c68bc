#!/bin/bash
# rescore with 8 candidates per wave in flight: full GPU suite, smoke, configs[1], default
# bench, W = 8 rank shape
T=tools/gpu_step.sh
$T gpu_tests 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread && \
$T smoke 200 python -c "import __graft_entry__ as g; g.smoke()" && \
$T cfg1 300 python bench.py --rows 1000000 --dim 384 --batch 256 --k 10 --encoder minilm --cpu-queries 256 --sweep 1,16,64,128,256,1024 && \
$T bench 400 python bench.py && \
$T shape8 300 python bench.py --rows 1250000 --batch 8192 --encoder none --no-cpu-baseline --steps 10
