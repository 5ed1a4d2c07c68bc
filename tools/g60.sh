#!/bin/bash
# pre-pass threshold 32 -> 4 tiles per workgroup: full GPU suite, default bench, configs[1]
# bench, batch sweeps over 1M x 384 with the new and the old threshold
T=tools/gpu_step.sh
S="python bench.py --rows 1000000 --dim 384 --batch 256 --k 10 --encoder none --no-cpu-baseline --steps 20 --sweep 1,16,64,128,256,1024"
$T gpu_tests 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread && \
$T smoke 200 python -c "import __graft_entry__ as g; g.smoke()" && \
$T bench 400 python bench.py && \
$T cfg1 300 python bench.py --rows 1000000 --dim 384 --batch 256 --k 10 --encoder minilm --cpu-queries 256 && \
$T sweep_new 300 $S && \
$T sweep_old 300 env HCRAG_PREPASS_MIN_TILES=32 $S
